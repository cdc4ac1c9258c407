#!/bin/bash
# Round 6: whole-decode-step A/B of the 64-session kernel table entries (lab/tools/table_ab.py).
set -o pipefail
O=gpurun_out/${1:-r6ab}
mkdir -p $O
O3=M64:N4096xK4096e3; D3=M64:N4096xK11008e3; GU=M64:N22016xK4096e1; LM=M64:N32000xK4096e0; Q=M64:N12288xK4096e0
timeout -k 10 300 python3 -u lab/tools/table_ab.py --batch 64 --rounds 4 --var base \
  --var "$O3=rwr" --var "$O3=rwr+r" --var "$O3=rwk+r" --var "$O3=rwki" --var "$O3=pk" \
  --var "$D3=rwk" --var "$D3=rwki" --var "$D3=rwki+r" --var "$GU=rw+r" --var "fold=0" --var "fold=0,$Q=rw+r" \
  --var "$LM=rw" --var "$LM=sk" > $O/ab64.json 2> $O/ab64.err || { tail -20 $O/ab64.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$O/ab64.json').read().strip().splitlines()[-1])
for k,v in sorted(r['ab'].items(), key=lambda kv: kv[1]['mean_ms']): print(f'{v[\"mean_ms\"]:.4f}', k, v['windows'])"
