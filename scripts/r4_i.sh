#!/bin/bash
# GQA decode attention: context-split floor A/B at the 70B / 8B head shapes.
set -o pipefail
OUT=gpurun_out/${1:-r4i}
mkdir -p $OUT
export TMPDIR=/tmp
for mp in 256 128 64; do
  timeout -k 10 120 python scripts/attn_decode_bench.py --batch 64 --ctx 170 512 --heads 64/8 32/8 --min-part $mp > $OUT/gqa_mp$mp.jsonl 2>&1 || exit 1
done
