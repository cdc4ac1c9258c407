set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py tests/test_training_rpc.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_new.log; [ $rc -ne 0 ] && exit $rc
MPAMD_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/mprof -o bench -- python bench.py --steps 8 --warmup 2 > gpurun_out/mprof.log 2>&1
rc=$?; tail -3 gpurun_out/mprof.log; exit $rc
