set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k autotune > gpurun_out/pytest_autotune.log 2>&1 && \
timeout -k 10 500 python -u bench.py --model llama3-70b --fp8 --steps 16 --warmup 4 > gpurun_out/s6g_l70_fp8.log 2>&1
