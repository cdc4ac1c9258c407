#!/bin/bash
# Round 5: where the 64-session decode step waits (kernel trace of the driver's bench command).
set -o pipefail
O=gpurun_out/${1:-r5e}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/b64 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b64.json 2> $O/b64.err || exit 1
DB=$(ls $O/b64/*/run_results.db 2>/dev/null | head -1); [ -z "$DB" ] && DB=$(find $O/b64 -name "*.db" | head -1)
python3 lab/tools/rocpd_steps.py $DB --steps 20 > $O/b64_kernels_per_step.txt
python3 lab/tools/prof_gaps.py $DB --steps 20 > $O/b64_gaps.txt
cat $O/b64_kernels_per_step.txt $O/b64_gaps.txt
