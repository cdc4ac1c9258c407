#!/bin/bash
# Per-kernel time of the Llama-3-70B fp8 (W8A16) decode step at 64 sessions.
set -o pipefail
OUT=gpurun_out/${1:-r4v}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/b70 -o run -- python3 bench.py --gpus 1 --model llama3-70b --fp8 --steps 10 --warmup 3 > $OUT/b70.json 2> $OUT/b70.err || exit 1
