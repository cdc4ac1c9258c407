#!/bin/bash
# GQA decode: block b = token b on the ROPE path (one dependent load fewer): GPU tests, cold micro-bench, Llama-3-8B / 70B fp8 bench.
set -o pipefail
OUT=gpurun_out/${1:-r4aa}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_qkv_fold_gpu.py tests/test_executor_gpu.py -k "mfma or gqa or fold or attention or executor" > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 200 python scripts/attn_decode_bench.py --cold --batch 1 16 64 --ctx 170 1024 --heads 64/8 32/8 > $OUT/gqa.jsonl 2>&1 || exit 1
timeout -k 10 200 python bench.py --model llama3-8b > $OUT/l3.json 2> $OUT/l3.err || exit 1
timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70.json 2> $OUT/b70.err || exit 1
