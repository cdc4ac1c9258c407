set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_b1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 1 --steps 16 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/prof_b1.log 2>&1
