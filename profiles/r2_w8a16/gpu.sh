set -o pipefail
# W8A16 fused-norm decode path for fp8 stages vs the W8A8 path
O=gpurun_out/r2_w8a16
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread -k "w8a16 or fp8" > $O/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model llama3-70b --fp8 --steps 8 --warmup 2 > $O/b70_w8a16.log 2>&1 && \
MPAMD_FP8_MODE=w8a8 timeout -k 10 400 python -u bench.py --model llama3-70b --fp8 --steps 8 --warmup 2 > $O/b70_w8a8.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof70 -o run -- python3 bench.py --model llama3-70b --fp8 --steps 6 --warmup 2 > $O/prof70.log 2>&1
