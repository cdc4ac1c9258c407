#!/bin/bash
# Measured per-stage balance of the auto splits (7B pp4 / pp8, 70B fp8 pp8) + the prefill round breakdown.
set -o pipefail
OUT=gpurun_out/${1:-r4e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/prefill_round.py --batch 64 --prompt-len 128 > $OUT/prefill_round.log 2>&1 || exit 1
timeout -k 10 200 python scripts/stage_balance.py --model llama2-7b --stages 4 > $OUT/bal_7b_pp4.log 2>&1 || exit 1
timeout -k 10 250 python scripts/stage_balance.py --model llama2-7b --stages 8 > $OUT/bal_7b_pp8.log 2>&1 || exit 1
timeout -k 10 500 python scripts/stage_balance.py --model llama3-70b --fp8 --stages 8 > $OUT/bal_70b_pp8.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/b64.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --batch 1 --steps 40 --warmup 8 > $OUT/b1.log 2>&1 || exit 1
timeout -k 10 200 python scripts/attn_bench.py --seqs 1x2048 64x128 --heads 32/32 32/8 --kernels fa4 fa8 > $OUT/attn_prefill_auto.jsonl 2>&1 || exit 1
