#!/bin/bash
# Split-K floor for the flash-decoding kernel at few (query, head) pairs now that the 16-wave form is off:
# attention micro-bench and batch-1 / batch-2 bench under MPAMD_ATTN_MIN_PART.
set -o pipefail
OUT=gpurun_out/${1:-r4t}
mkdir -p $OUT
export TMPDIR=/tmp
for mp in default 64 128; do
  if [ $mp = default ]; then unset MPAMD_ATTN_MIN_PART; else export MPAMD_ATTN_MIN_PART=$mp; fi
  timeout -k 10 120 python scripts/attn_decode_bench.py --batch 1 2 --ctx 170 512 1024 2048 --heads 32/32 > $OUT/attn_mp$mp.jsonl 2>&1 || exit 1
  timeout -k 10 300 python bench.py --gpus 1 --batch 1 > $OUT/b1_mp$mp.json 2> $OUT/b1_mp$mp.err || exit 1
done
