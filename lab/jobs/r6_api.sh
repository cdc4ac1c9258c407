#!/bin/bash
# Round 6: which host call blocks at the decode step boundary - HIP API + kernel trace of the 64-session
# and batch-1 7B benches (no counters in this run).
set -o pipefail
O=gpurun_out/${1:-r6api}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for b in 64 1; do
  timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace -d $O/p$b -o run -- python3 bench.py --gpus 1 --batch $b --steps 20 --warmup 5 \
    > $O/b${b}.json 2> $O/b${b}.err || exit 1
  DB=$(find $O/p$b -name "*.db" | head -1)
  python3 lab/tools/prof_api.py $DB --steps 4 > $O/b${b}_api.txt && rm -rf $O/p$b || exit 1
  head -60 $O/b${b}_api.txt
done
