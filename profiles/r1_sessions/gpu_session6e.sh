set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_gpu_s6e.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 > gpurun_out/b1_mp256.log 2>&1 && \
MPAMD_ATTN_MIN_PART=64 timeout -k 10 300 python -u bench.py --batch 1 > gpurun_out/b1_mp64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-8b --batch 1 > gpurun_out/l3_b1_mp256.log 2>&1 && \
MPAMD_ATTN_MIN_PART=64 timeout -k 10 300 python -u bench.py --model llama3-8b --batch 1 > gpurun_out/l3_b1_mp64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-8b > gpurun_out/l3_b64_mp256.log 2>&1 && \
MPAMD_ATTN_MIN_PART=64 timeout -k 10 300 python -u bench.py --model llama3-8b > gpurun_out/l3_b64_mp64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 --prompt-len 2048 > gpurun_out/b1_long_mp256.log 2>&1 && \
MPAMD_ATTN_MIN_PART=64 timeout -k 10 300 python -u bench.py --batch 1 --prompt-len 2048 > gpurun_out/b1_long_mp64.log 2>&1
