set -o pipefail
O=gpurun_out/r3_first
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_training_rpc.py tests/test_fused_norm.py -m gpu > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/b64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 > $O/b1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run -- python3 bench.py --steps 16 --warmup 4 > $O/prof64.log 2>&1
