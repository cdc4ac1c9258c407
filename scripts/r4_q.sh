#!/bin/bash
# Per-kernel time of the driver bench (64 sessions) and batch 1 under rocprofv3.
set -o pipefail
OUT=gpurun_out/${1:-r4q}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/b64 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/b64.json 2> $OUT/b64.err || exit 1
