set -o pipefail
# split-K ring GEMM with the half-grid ring kernel ("rwh") as an autotune candidate for the narrow projections
O=gpurun_out/r2_rwh
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_norm.py tests/test_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread -k "shared_a or fused or w8a16 or fp8_executor or rwk" > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/b64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 > $O/b1.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model llama3-70b --fp8 --steps 8 --warmup 2 > $O/b70.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run -- python3 bench.py --steps 16 --warmup 4 > $O/prof64.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof70 -o run -- python3 bench.py --model llama3-70b --fp8 --steps 6 --warmup 2 > $O/prof70.log 2>&1
