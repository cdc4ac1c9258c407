#!/bin/bash
# Sampler: single-workgroup rows vs the chunked split path at the 32K vocabulary (MPAMD_SAMPLE_SPLIT).
set -o pipefail
OUT=gpurun_out/${1:-r4m}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 150 python bench.py --batch 1 --steps 40 --warmup 8 > $OUT/b1.log 2>&1 || exit 1
MPAMD_SAMPLE_SPLIT=32000 timeout -k 10 150 python bench.py --batch 1 --steps 40 --warmup 8 > $OUT/b1_split.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/b64.log 2>&1 || exit 1
MPAMD_SAMPLE_SPLIT=32000 timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/b64_split.log 2>&1 || exit 1
MPAMD_SAMPLE_SPLIT=32000 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sample" > $OUT/pytest_sample_split.log 2>&1 || exit 1
