set -o pipefail
# fp8-weight (W8A16) Llama-2-7B and Llama-3-8B bf16 rows for the README table
O=gpurun_out/r2_more
mkdir -p $O
timeout -k 10 300 python -u bench.py --fp8 > $O/l2_fp8_b64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --fp8 --batch 1 > $O/l2_fp8_b1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-8b > $O/l3_b64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-8b --batch 1 > $O/l3_b1.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model llama3-70b --fp8 --batch 1 --steps 16 --warmup 4 > $O/l70_fp8_b1.log 2>&1
