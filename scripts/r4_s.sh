#!/bin/bash
# Per-kernel time of batch 1 and of 128 sessions under rocprofv3 (rocpd database; summarised by scripts/rocpd_steps.py).
set -o pipefail
OUT=gpurun_out/${1:-r4s}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/b1 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --batch 1 > $OUT/b1.json 2> $OUT/b1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/b128 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --batch 128 > $OUT/b128.json 2> $OUT/b128.err || exit 1
