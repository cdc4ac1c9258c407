set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_gpu_s6f.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s6f.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/s6f_default.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-8b > gpurun_out/s6f_l3_b64.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model mixtral-8x7b --steps 16 --warmup 4 > gpurun_out/s6f_mx_b64.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model llama3-70b --fp8 --steps 16 --warmup 4 > gpurun_out/s6f_l70_fp8.log 2>&1
