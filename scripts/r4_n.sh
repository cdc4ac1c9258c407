#!/bin/bash
# 16-wave decode attention with the pipelined prologue (MPAMD_ATTN_WIDE_PIPE) at small batches.
set -o pipefail
OUT=gpurun_out/${1:-r4n}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python scripts/attn_decode_bench.py --batch 1 4 8 --ctx 170 1024 --heads 32/32 > $OUT/wide.jsonl 2>&1 || exit 1
MPAMD_ATTN_WIDE_PIPE=1 timeout -k 10 120 python scripts/attn_decode_bench.py --batch 1 4 8 --ctx 170 1024 --heads 32/32 > $OUT/wide_pipe.jsonl 2>&1 || exit 1
MPAMD_ATTN_WIDE_PIPE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "paged or rope or fold" > $OUT/pytest_wide_pipe.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --batch 1 --steps 40 --warmup 8 > $OUT/b1.log 2>&1 || exit 1
MPAMD_ATTN_WIDE_PIPE=1 timeout -k 10 150 python bench.py --batch 1 --steps 40 --warmup 8 > $OUT/b1_pipe.log 2>&1 || exit 1
