#!/bin/bash
# GQA decode attention: query heads per block (MPAMD_GQA_HB) A/B at the 70B / 8B head shapes.
set -o pipefail
OUT=gpurun_out/${1:-r4k}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python scripts/attn_decode_bench.py --batch 64 256 --ctx 170 1024 --heads 64/8 32/8 > $OUT/gqa_hb_default.jsonl 2>&1 || exit 1
for hb in 4 2; do
  MPAMD_GQA_HB=$hb timeout -k 10 120 python scripts/attn_decode_bench.py --batch 64 256 --ctx 170 1024 --heads 64/8 32/8 > $OUT/gqa_hb$hb.jsonl 2>&1 || exit 1
done
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "mfma" > $OUT/pytest_mfma.log 2>&1 || exit 1
MPAMD_GQA_HB=4 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "mfma" > $OUT/pytest_mfma_hb4.log 2>&1 || exit 1
