#!/bin/bash
# Round 5: the two-dimensionally tiled decode GEMM (csrc/gemm_t2d.h) at 129..256 sessions -
# GPU tests, per-kernel trace of the 256-session step, and the 128-session step with the tiled
# kernel forced below its default row range.
set -o pipefail
O=gpurun_out/${1:-r5x}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_norm.py \
  tests/test_executor_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 250 python3 lab/tools/t2d_bench.py --m 256 192 --splits 0 1 2 --gl --bm64 > $O/gemm.jsonl 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/b256 -o run -- python3 bench.py --batch 256 --steps 20 --warmup 5 > $O/b256_prof.json 2> $O/b256_prof.err || exit 1
DB=$(ls $O/b256/*/run_results.db 2>/dev/null | head -1); [ -z "$DB" ] && DB=$(find $O/b256 -name "*.db" | head -1)
python3 lab/tools/rocpd_steps.py $DB --steps 20 > $O/b256_kernels_per_step.txt
head -30 $O/b256_kernels_per_step.txt
timeout -k 10 200 python3 bench.py --batch 128 > $O/b128.json 2> $O/b128.err || exit 1
MPAMD_T2D_MIN=65 timeout -k 10 200 python3 bench.py --batch 128 > $O/b128_t2d.json 2> $O/b128_t2d.err || exit 1
MPAMD_T2D_MIN=65 timeout -k 10 200 python3 bench.py --batch 96 > $O/b96_t2d.json 2> $O/b96_t2d.err || exit 1
timeout -k 10 200 python3 bench.py --batch 96 > $O/b96.json 2> $O/b96.err || exit 1
timeout -k 10 200 python3 bench.py --batch 256 > $O/b256.json 2> $O/b256.err || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/b*.json
