set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "mfma_rope" > gpurun_out/pytest_mfma_rope_mha.log 2>&1 && \
MPAMD_ATTN_MFMA_DECODE=1 timeout -k 10 300 python -u bench.py > gpurun_out/s6i_mha_mfma.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/s6i_mha_simt.log 2>&1 && \
MPAMD_ATTN_MFMA_DECODE=1 timeout -k 10 300 python -u bench.py --batch 1 > gpurun_out/s6i_mha_mfma_b1.log 2>&1 && \
MPAMD_ATTN_MFMA_DECODE=1 timeout -k 10 300 python -u bench.py --batch 128 > gpurun_out/s6i_mha_mfma_b128.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 128 > gpurun_out/s6i_mha_simt_b128.log 2>&1
