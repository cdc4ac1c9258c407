#!/bin/bash
# Round 5: Llama-3-70B fp8 per-kernel decode profile, W8A16 (default) and W8A8, 64 sessions, 1 GPU.
set -o pipefail
O=gpurun_out/${1:-r5g}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/w8a16 -o run -- python3 bench.py --gpus 1 --model llama3-70b --fp8 --steps 10 --warmup 3 > $O/w8a16.json 2> $O/w8a16.err || exit 1
DB=$(find $O/w8a16 -name "*.db" | head -1)
python3 lab/tools/rocpd_steps.py $DB --steps 10 > $O/w8a16_kernels.txt && rm -f $DB
MPAMD_FP8_MODE=w8a8 timeout -k 10 500 rocprofv3 --kernel-trace -d $O/w8a8 -o run -- python3 bench.py --gpus 1 --model llama3-70b --fp8 --steps 10 --warmup 3 > $O/w8a8.json 2> $O/w8a8.err || exit 1
DB=$(find $O/w8a8 -name "*.db" | head -1)
python3 lab/tools/rocpd_steps.py $DB --steps 10 > $O/w8a8_kernels.txt && rm -f $DB
cat $O/w8a16_kernels.txt $O/w8a8_kernels.txt
