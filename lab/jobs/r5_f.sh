#!/bin/bash
# Round 5: host API timeline of the 64-session decode step (where the host blocks).
set -o pipefail
O=gpurun_out/${1:-r5f}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace -d $O/b64 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b64.json 2> $O/b64.err || exit 1
DB=$(find $O/b64 -name "*.db" | head -1)
python3 lab/tools/prof_host.py $DB --steps 20 > $O/host.txt
python3 lab/tools/prof_gaps.py $DB --steps 20 > $O/gaps.txt
cat $O/host.txt $O/gaps.txt
