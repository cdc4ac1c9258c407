set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "mfma" > gpurun_out/pytest_mfma_rope.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_gpu_s6h.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-8b > gpurun_out/s6h_l3_fuse.log 2>&1 && \
MPAMD_FUSE_ROPE=0 timeout -k 10 300 python -u bench.py --model llama3-8b > gpurun_out/s6h_l3_nofuse.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-8b --batch 1 > gpurun_out/s6h_l3_b1_fuse.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/s6h_default.log 2>&1
