#!/bin/bash
# fp8 (W8A16) split-K ring with a 16-tile column group at 49..64 rows: numerics with it forced
# (MPAMD_RWK_NT=16), then Llama-3-70B fp8 with it as an autotuner candidate (MPAMD_RWK_F8_WIDE=1) vs default.
set -o pipefail
OUT=gpurun_out/${1:-r4ad}
mkdir -p $OUT
export TMPDIR=/tmp
MPAMD_RWK_NT=16 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_qkv_fold_gpu.py tests/test_fp8.py -k "(fp8 or w8 or fold or f8) and not executor_fold_on_off" > $OUT/pytest_nt16.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_def1.json 2> $OUT/b70_def1.err || exit 1
MPAMD_RWK_F8_WIDE=1 timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_wide1.json 2> $OUT/b70_wide1.err || exit 1
MPAMD_RWK_NT=16 timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_nt16.json 2> $OUT/b70_nt16.err || exit 1
timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_def2.json 2> $OUT/b70_def2.err || exit 1
MPAMD_RWK_F8_WIDE=1 timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_wide2.json 2> $OUT/b70_wide2.err || exit 1
