#!/bin/bash
# Round 6: batch-1 gate/up entry (after M4 gate/up -> rw): rw vs rw+r vs pk on Llama-2-7B, and the
# same question for Llama-3-8B's gate/up.
set -o pipefail
O=gpurun_out/${1:-r6ab1b}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u lab/tools/table_ab.py --batch 1 --rounds 4 --steps 40 --var base \
  --var "M4:N22016xK4096e1=rw+r" --var "M4:N22016xK4096e1=pk" > $O/ab7.json 2> $O/ab7.err || { tail -20 $O/ab7.err; exit 1; }
timeout -k 10 300 python3 -u lab/tools/table_ab.py --model llama3-8b --batch 1 --rounds 4 --steps 40 --var base \
  --var "M4:N28672xK4096e1=rw" --var "M4:N28672xK4096e1=rw+r" > $O/ab8.json 2> $O/ab8.err || { tail -20 $O/ab8.err; exit 1; }
for f in ab7 ab8; do python3 -c "
import json; r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
for k,v in sorted(r['ab'].items(), key=lambda kv: kv[1]['mean_ms']): print('$f', f'{v[\"mean_ms\"]:.4f}', k, v['windows'])"; done
