set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "paged_attention" > gpurun_out/pytest_u8.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/s6m_u8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 --prompt-len 2048 > gpurun_out/s6m_u8_b1_long.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 128 > gpurun_out/s6m_u8_b128.log 2>&1
