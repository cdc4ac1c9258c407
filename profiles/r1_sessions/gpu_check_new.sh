# Quick GPU check of recently added tests (one process, each step time-limited).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_offload_gpu.py tests/test_executor_gpu.py}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_new.log; exit $rc
