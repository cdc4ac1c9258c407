#!/bin/bash
# Round 6 final tree: box-to-box spread of the default bench (64 sessions) and batch 1.
set -o pipefail
O=gpurun_out/${1:-r6spread}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 bench.py > $O/b64.json 2> $O/b64.err || exit 1
timeout -k 10 200 python3 bench.py --batch 1 > $O/b1.json 2> $O/b1.err || exit 1
for f in b64 b1; do python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], d['value'])" $O/$f.json; done
