#!/bin/bash
# Round 5 final tree: per-step kernel tables (rocprofv3 --kernel-trace) for the 64-session 7B bench
# and the 70B fp8 bench.
set -o pipefail
O=gpurun_out/${1:-r5ktab}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p64 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b64_prof.json 2> $O/b64_prof.err || exit 1
DB=$(find $O/p64 -name "*.db" | head -1)
python3 lab/tools/rocpd_steps.py $DB --steps 20 --seq 16 > $O/b64_kernels_per_step.txt && rm -rf $O/p64 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/p70 -o run -- python3 bench.py --model llama3-70b --fp8 --steps 10 --warmup 3 > $O/b70_prof.json 2> $O/b70_prof.err || exit 1
DB=$(find $O/p70 -name "*.db" | head -1)
python3 lab/tools/rocpd_steps.py $DB --steps 10 --marker embedding_kernel --seq 16 > $O/b70_kernels_per_step.txt && rm -rf $O/p70 || exit 1
cat $O/b64_kernels_per_step.txt
cat $O/b70_kernels_per_step.txt
