#!/bin/bash
# Batch-1 decode kernel trace.
set -o pipefail
OUT=gpurun_out/${1:-r4l}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 1 --steps 40 --warmup 8 > $GRAFT_REPO_ROOT/$OUT/prof_b1.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python scripts/prof_db_summary.py "$(find /tmp/p1 -name '*.db' | head -1)" 40ms > $OUT/kernels_b1.txt 2>&1
