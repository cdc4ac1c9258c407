#!/bin/bash
# Row-split wide GEMM as a per-wave register ring: numerics, 128 / 192 / 256-session steps; 64 / 1-session steps.
set -o pipefail
OUT=gpurun_out/${1:-r4g}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_norm.py > $OUT/pytest_mw.log 2>&1 || exit 1
MPAMD_WIDE_ROWS=256 timeout -k 10 250 python bench.py --batch 256 --steps 12 --warmup 4 > $OUT/b256_mw.log 2>&1 || exit 1
timeout -k 10 250 python bench.py --batch 256 --steps 12 --warmup 4 > $OUT/b256_blas.log 2>&1 || exit 1
MPAMD_WIDE_KERNEL=mw timeout -k 10 200 python bench.py --batch 128 --steps 16 --warmup 4 > $OUT/b128_mw.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --batch 128 --steps 16 --warmup 4 > $OUT/b128.log 2>&1 || exit 1
cd /tmp && MPAMD_WIDE_ROWS=256 timeout -k 10 250 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof256 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 256 --steps 8 --warmup 3 > $GRAFT_REPO_ROOT/$OUT/prof256.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python scripts/prof_db_summary.py "$(find /tmp/prof256 -name '*.db' | head -1)" 40ms > $OUT/kernels_b256_mw.txt 2>&1
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/b64.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --batch 1 --steps 40 --warmup 8 > $OUT/b1.log 2>&1 || exit 1
