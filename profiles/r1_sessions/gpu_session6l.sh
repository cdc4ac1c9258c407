set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "paged_attention" > gpurun_out/pytest_pglds.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/s6l_a.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 > gpurun_out/s6l_b1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 --prompt-len 2048 > gpurun_out/s6l_b1_long.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s6l -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 16 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/prof_s6l.log 2>&1
