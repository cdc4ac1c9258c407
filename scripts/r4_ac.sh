#!/bin/bash
# Llama-3-70B fp8: split-K column-group width of the W8A16 ring (MPAMD_RWK_NT ablation) vs the default choice (NT 8).
set -o pipefail
OUT=gpurun_out/${1:-r4ac}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_def.json 2> $OUT/b70_def.err || exit 1
MPAMD_RWK_NT=4 timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_nt4.json 2> $OUT/b70_nt4.err || exit 1
MPAMD_RWK_NT=2 timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_nt2.json 2> $OUT/b70_nt2.err || exit 1
timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_def2.json 2> $OUT/b70_def2.err || exit 1
