#!/bin/bash
# Round 6: whole-step A/B of the Llama-3-8B 64-session table entries it does not share with Llama-2-7B.
set -o pipefail
O=gpurun_out/${1:-r6ab8}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
Q=M64:N6144xK4096e0; GU=M64:N28672xK4096e1; D3=M64:N4096xK14336e3; LM=M64:N128256xK4096e0
timeout -k 10 900 python3 -u lab/tools/table_ab.py --model llama3-8b --batch 64 --rounds 3 --steps 20 --var base \
  --var "fold=0" --var "fold=0,$Q=rw" --var "$GU=rw" --var "$GU=rw+r" --var "$GU=lds42" --var "$D3=rwk+r" --var "$D3=rw" \
  --var "$LM=lds24+r" --var "$LM=rw" > $O/ab8.json 2> $O/ab8.err || { tail -20 $O/ab8.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$O/ab8.json').read().strip().splitlines()[-1])
for k,v in sorted(r['ab'].items(), key=lambda kv: kv[1]['mean_ms']): print(f'{v[\"mean_ms\"]:.4f}', k, v['windows'])"
