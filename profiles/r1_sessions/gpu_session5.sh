set -o pipefail
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_gpu_all.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --batch 1 --steps 16 --warmup 4 > gpurun_out/mx_b1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 16 --warmup 4 > gpurun_out/mx_b64.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1
