#!/bin/bash
# Llama-3-70B fp8: W8A8 (MPAMD_FP8_MODE=w8a8) vs the default W8A16 on the final tree.
set -o pipefail
OUT=gpurun_out/${1:-r4af}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_w8a16.json 2> $OUT/b70_w8a16.err || exit 1
MPAMD_FP8_MODE=w8a8 timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_w8a8.json 2> $OUT/b70_w8a8.err || exit 1
