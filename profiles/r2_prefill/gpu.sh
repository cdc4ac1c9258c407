set -o pipefail
# prefill round timing (bench.py prefill_round_s / prefill_tokens_per_s)
O=gpurun_out/r2_prefill
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 > $O/b64_p128.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 --prompt-len 2048 --steps 8 --warmup 2 > $O/b1_p2048.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 8 --prompt-len 2048 --steps 8 --warmup 2 > $O/b8_p2048.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-8b --batch 8 --prompt-len 2048 --steps 8 --warmup 2 > $O/l3_b8_p2048.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model llama3-70b --fp8 --batch 16 --prompt-len 512 --steps 4 --warmup 1 > $O/l70_b16_p512.log 2>&1
