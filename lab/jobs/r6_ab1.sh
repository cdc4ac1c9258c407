#!/bin/bash
# Round 6: whole-step A/B of the batch-1 (M4 bucket) kernel table entries, Llama-2-7B.
set -o pipefail
O=gpurun_out/${1:-r6ab1}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O3=M4:N4096xK4096e3; D3=M4:N4096xK11008e3; GU=M4:N22016xK4096e1; LM=M4:N32000xK4096e0; Q=M4:N12288xK4096e0
timeout -k 10 400 python3 -u lab/tools/table_ab.py --batch 1 --rounds 4 --steps 40 --var base \
  --var "$O3=pk" --var "$O3=rw" --var "$O3=rw+r" --var "$O3=rwk" --var "$O3=rwk+r" \
  --var "$D3=pk" --var "$D3=rw+r" --var "$D3=rwk+r" --var "$GU=rw" --var "$GU=pk+r" --var "$Q=pk" --var "$Q=rw+r" \
  --var "$LM=rw" --var "$LM=pk" > $O/ab1.json 2> $O/ab1.err || { tail -20 $O/ab1.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$O/ab1.json').read().strip().splitlines()[-1])
for k,v in sorted(r['ab'].items(), key=lambda kv: kv[1]['mean_ms']): print(f'{v[\"mean_ms\"]:.4f}', k, v['windows'])"
