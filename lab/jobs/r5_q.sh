#!/bin/bash
# Round 5: after the DPP reductions / sampler / GQA flat-load fixes: GPU suite, bench 64 / 1, kernel table.
set -o pipefail
O=gpurun_out/${1:-r5q}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 200 python3 bench.py > $O/b64.json 2> $O/b64.err || exit 1
timeout -k 10 200 python3 bench.py --batch 1 > $O/b1.json 2> $O/b1.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b64_prof.json 2> $O/b64_prof.err || exit 1
DB=$(find $O/prof -name "*.db" | head -1)
python3 lab/tools/rocpd_steps.py $DB --steps 20 > $O/b64_kernels_per_step.txt && rm -f $DB
for f in b64 b1; do python3 -c "
import json
r=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); print('$f', r['ms_per_step'], r['value'])"; done
cat $O/b64_kernels_per_step.txt
