#!/bin/bash
# Round 6: whole-step A/B of the Llama-3-70B fp8 (W8A16) 64-session table entries.
set -o pipefail
O=gpurun_out/${1:-r6ab70}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O3=M64:N8192xK8192e3; D3=M64:N8192xK28672e3; GU=M64:N57344xK8192e1; Q=M64:N10240xK8192e0
timeout -k 10 900 python3 -u lab/tools/table_ab.py --model llama3-70b --fp8 --batch 64 --rounds 2 --steps 10 --var base \
  --var "$O3=rwk" --var "$O3=rw+r" --var "$D3=rwk" --var "$D3=rw+r" --var "$GU=rw+r" --var "fold=0" \
  > $O/ab70.json 2> $O/ab70.err || { tail -20 $O/ab70.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$O/ab70.json').read().strip().splitlines()[-1])
for k,v in sorted(r['ab'].items(), key=lambda kv: kv[1]['mean_ms']): print(f'{v[\"mean_ms\"]:.4f}', k, v['windows'])"
