set -o pipefail
O=gpurun_out/r3_b
mkdir -p $O
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 "$@" || { echo "STEP FAILED: $name rc=$?" >> $O/steps.log; exit 1; }; echo "ok $name" >> $O/steps.log; }
run tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_executor_gpu.py tests/test_engine_gpu.py tests/test_training_rpc.py tests/test_fused_norm.py tests/test_hf_parity.py -m gpu > $O/tests.log 2>&1
run b1 300 python -u bench.py --batch 1 > $O/b1.log 2>&1
run b128 300 python -u bench.py --batch 128 > $O/b128.log 2>&1
run b256 300 python -u bench.py --batch 256 --steps 16 --warmup 4 > $O/b256.log 2>&1
run b70 400 python -u bench.py --model llama3-70b --fp8 --steps 8 --warmup 2 > $O/b70.log 2>&1
run prof70 400 rocprofv3 --kernel-trace --stats -d $O/prof70 -o run -- python3 bench.py --model llama3-70b --fp8 --steps 6 --warmup 2 > $O/prof70.log 2>&1
