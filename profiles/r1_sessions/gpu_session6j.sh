set -o pipefail
mkdir -p gpurun_out
for nt in 64 128; do
MPAMD_NORM_THREADS=$nt timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k rmsnorm > gpurun_out/pytest_norm_$nt.log 2>&1 || exit 1
done
for nt in 64 128 256 512; do
MPAMD_NORM_THREADS=$nt timeout -k 10 300 python -u bench.py > gpurun_out/s6j_norm_$nt.log 2>&1 || exit 1
done
