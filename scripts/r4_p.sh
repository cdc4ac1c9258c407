#!/bin/bash
# Confirms the 4-wave-only decode attention default: attention tests, attention A/B, driver bench, batch 1.
set -o pipefail
OUT=gpurun_out/${1:-r4p}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attn or attention" > $OUT/pytest_attn.log 2>&1 || exit 1
timeout -k 10 120 python scripts/attn_decode_bench.py --batch 1 2 4 8 16 64 --ctx 170 1024 2048 --heads 32/32 > $OUT/attn_default.jsonl 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 400 python bench.py --gpus 1 --batch 1 > $OUT/bench_b1.json 2> $OUT/bench_b1.err || exit 1
