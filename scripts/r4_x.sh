#!/bin/bash
# 8-wave GQA decode attention (MPAMD_GQA_WAVES=8): numerics under the GPU tests, cold micro-bench A/B, 70B fp8 bench A/B.
set -o pipefail
OUT=gpurun_out/${1:-r4x}
mkdir -p $OUT
export TMPDIR=/tmp
MPAMD_GQA_WAVES=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_qkv_fold_gpu.py -k "mfma or gqa or fold or attention" > $OUT/pytest_w8.log 2>&1 || exit 1
MPAMD_GQA_WAVES=8 timeout -k 10 200 python scripts/attn_decode_bench.py --cold --batch 1 16 64 --ctx 170 1024 --heads 64/8 32/8 > $OUT/gqa_w8.jsonl 2>&1 || exit 1
timeout -k 10 200 python scripts/attn_decode_bench.py --cold --batch 1 16 64 --ctx 170 1024 --heads 64/8 32/8 > $OUT/gqa_w4.jsonl 2>&1 || exit 1
MPAMD_GQA_WAVES=8 timeout -k 10 400 python bench.py --gpus 1 --model llama3-70b --fp8 --steps 20 --warmup 5 > $OUT/b70_w8.json 2> $OUT/b70_w8.err || exit 1
timeout -k 10 400 python bench.py --gpus 1 --model llama3-70b --fp8 --steps 20 --warmup 5 > $OUT/b70_w4.json 2> $OUT/b70_w4.err || exit 1
