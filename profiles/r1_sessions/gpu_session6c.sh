set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_kern_6c.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_fuse.log 2>&1 && \
MPAMD_FUSE_ROPE=0 timeout -k 10 300 python -u bench.py > gpurun_out/bench_nofuse.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fuse2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 16 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/prof_fuse2.log 2>&1
