#!/bin/bash
# GQA decode attention: MFMA kernel vs the flash-decoding (SIMT) kernel, cold caches (in-situ-like).
set -o pipefail
OUT=gpurun_out/${1:-r4w}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/attn_decode_bench.py --cold --batch 1 16 64 --ctx 170 1024 --heads 64/8 32/8 > $OUT/gqa_auto.jsonl 2>&1 || exit 1
timeout -k 10 200 python scripts/attn_decode_bench.py --cold --kernel simt --batch 1 16 64 --ctx 170 1024 --heads 64/8 32/8 > $OUT/gqa_simt.jsonl 2>&1 || exit 1
timeout -k 10 200 python scripts/attn_decode_bench.py --cold --batch 64 --ctx 170 --heads 32/32 > $OUT/mha_cold.jsonl 2>&1 || exit 1
