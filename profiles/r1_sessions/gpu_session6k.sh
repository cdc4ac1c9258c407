set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_gpu_s6k.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s6k.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/s6k_default.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-8b > gpurun_out/s6k_l3.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s6k -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 16 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/prof_s6k.log 2>&1
