set -o pipefail
# decode GEMMs skip the A-fragment loads of rows past M (batch 1: 1 of 16 rows is real)
O=gpurun_out/r2_amask
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_norm.py tests/test_executor_gpu.py tests/test_mixtral.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 > $O/b1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 8 > $O/b8.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/b64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-8b --batch 1 > $O/l3_b1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python3 bench.py --batch 1 --steps 16 --warmup 4 > $O/prof1.log 2>&1
