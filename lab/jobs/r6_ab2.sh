#!/bin/bash
# Round 6: whole-step A/B, second set: gate/up and qkv kernel forms at 64 sessions (sk = stream-K, which
# balances gate/up's 1376 column tiles over 256 CUs; lds = shared-A forms).
set -o pipefail
O=gpurun_out/${1:-r6ab2}
mkdir -p $O
GU=M64:N22016xK4096e1; Q=M64:N12288xK4096e0
timeout -k 10 300 python3 -u lab/tools/table_ab.py --batch 64 --rounds 4 --var base \
  --var "$GU=sk" --var "$GU=sk+r" --var "$GU=lds24" --var "$GU=lds42" --var "$GU=lds22" --var "$GU=pk" \
  --var "fold=0,$Q=sk" --var "fold=0,$Q=lds24" --var "fold=0" > $O/ab64.json 2> $O/ab64.err || { tail -20 $O/ab64.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$O/ab64.json').read().strip().splitlines()[-1])
for k,v in sorted(r['ab'].items(), key=lambda kv: kv[1]['mean_ms']): print(f'{v[\"mean_ms\"]:.4f}', k, v['windows'])"
