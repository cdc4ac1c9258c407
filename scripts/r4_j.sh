#!/bin/bash
# 256-session default path: where do the per-layer device copies come from (TunableOp on / off)?
set -o pipefail
OUT=gpurun_out/${1:-r4j}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 250 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/pa -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 256 --steps 8 --warmup 3 > $GRAFT_REPO_ROOT/$OUT/prof_tuned.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python scripts/prof_db_summary.py "$(find /tmp/pa -name '*.db' | head -1)" 40ms > $OUT/kernels_b256_tuned.txt 2>&1
cd /tmp && MPAMD_TUNED_GEMMS=0 timeout -k 10 250 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/pb -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 256 --steps 8 --warmup 3 > $GRAFT_REPO_ROOT/$OUT/prof_untuned.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python scripts/prof_db_summary.py "$(find /tmp/pb -name '*.db' | head -1)" 40ms > $OUT/kernels_b256_untuned.txt 2>&1
