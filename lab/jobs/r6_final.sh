#!/bin/bash
# Round 6 validation: GPU suite (-x, as the driver runs it), smoke, bench 64 / 1 / 256 sessions and
# 70B fp8, then the 70B fp8 per-step kernel table.
set -o pipefail
O=gpurun_out/${1:-r6final}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
tail -1 $O/smoke.txt
timeout -k 10 200 python3 bench.py > $O/b64.json 2> $O/b64.err || exit 1
timeout -k 10 200 python3 bench.py --batch 1 > $O/b1.json 2> $O/b1.err || exit 1
timeout -k 10 200 python3 bench.py --batch 256 > $O/b256.json 2> $O/b256.err || exit 1
timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70.json 2> $O/b70.err || exit 1
for f in b64 b1 b256 b70; do python3 -c "
import json
r=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); print('$f', r['ms_per_step'], r['value'])"; done
if [ "${KTAB70:-1}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p70 -o run -- python3 bench.py --model llama3-70b --fp8 --steps 10 --warmup 3 \
    > $O/b70_prof.json 2> $O/b70_prof.err || exit 1
  DB=$(find $O/p70 -name "*.db" | head -1)
  python3 lab/tools/rocpd_steps.py $DB --steps 10 --seq 12 > $O/b70_kernels_per_step.txt && rm -rf $O/p70 || exit 1
  head -20 $O/b70_kernels_per_step.txt
fi
if [ "${KTAB7:-1}" = 1 ]; then
  for b in 64 1; do
    timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p$b -o run -- python3 bench.py --batch $b --steps 20 --warmup 5 \
      > $O/b${b}_prof.json 2> $O/b${b}_prof.err || exit 1
    DB=$(find $O/p$b -name "*.db" | head -1)
    python3 lab/tools/rocpd_steps.py $DB --steps 20 --seq 16 > $O/b${b}_kernels_per_step.txt && rm -rf $O/p$b || exit 1
    head -12 $O/b${b}_kernels_per_step.txt
  done
fi
