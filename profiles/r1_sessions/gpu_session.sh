#!/bin/bash
# One GPU-box session: kernel/executor tests, 1-GPU bench, rocprofv3 kernel stats, HF baseline.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-tests bench prof hf}"

step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
    echo "stopping: $name exited $rc"; exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    bench) step bench1 600 python bench.py ;;
    benchgemm) step bench1_hipblaslt 600 python bench.py --gemm hipblaslt ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --steps 8 --warmup 2 ;;
    hf) step hf_baseline 600 python scripts/hf_baseline.py ;;
    kern) step bench_kernels 600 python scripts/bench_kernels.py ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "=== done"
