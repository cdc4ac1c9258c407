#!/bin/bash
# Round 6: per-step kernel tables and inter-kernel gaps (rocprofv3 --kernel-trace) of the 64-session and
# batch-1 7B benches on the current tree.
set -o pipefail
O=gpurun_out/${1:-r6gaps}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for b in 64 1; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p$b -o run -- python3 bench.py --gpus 1 --batch $b --steps 20 --warmup 5 > $O/b${b}_prof.json 2> $O/b${b}_prof.err || exit 1
  DB=$(find $O/p$b -name "*.db" | head -1)
  python3 lab/tools/rocpd_steps.py $DB --steps 20 --seq 16 > $O/b${b}_kernels_per_step.txt || exit 1
  python3 lab/tools/prof_gaps.py $DB --steps 20 > $O/b${b}_gaps.txt && rm -rf $O/p$b || exit 1
  head -3 $O/b${b}_kernels_per_step.txt; head -14 $O/b${b}_gaps.txt
done
