set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_gpu_s6d.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s6d.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 > gpurun_out/bench_b1_s6d.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 128 > gpurun_out/bench_b128_s6d.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default_s6d.log 2>&1
