#!/bin/bash
# Fold numerics + A/B of the qkv fold on the 64-session bench + a rocprofv3 kernel trace of the default tree.
set -o pipefail
OUT=gpurun_out/${1:-r4ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qkv_fold_gpu.py tests/test_kernels_gpu.py -k "fold or rope or attention or attn" > $OUT/pytest_fold.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/b64_default.log 2>&1 || exit 1
MPAMD_QKV_FOLD=0 timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/b64_nofold.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/b64_default2.log 2>&1 || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$OUT/prof_bench.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
DB=$(find /tmp/prof -name "*.db" | head -1)
python scripts/prof_db_summary.py "$DB" 20ms > $OUT/kernels_b64.txt 2>&1
