#!/bin/bash
# Round 6, after the nontemporal split-K slabs (r6nt): re-run the whole-step table A/B at 64 sessions
# (7B and 70B fp8) - the slab store form changes what a "+r" (reduce-launch) entry costs.
set -o pipefail
O=gpurun_out/${1:-r6abnt}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O3=M64:N4096xK4096e3; D3=M64:N4096xK11008e3; GU=M64:N22016xK4096e1; Q=M64:N12288xK4096e0
timeout -k 10 400 python3 -u lab/tools/table_ab.py --batch 64 --rounds 4 --var base \
  --var "$O3=rwr" --var "$O3=rwk+r" --var "$O3=rwki" --var "$O3=pk" \
  --var "$D3=rwk" --var "$D3=rwki" --var "$D3=rwk+r" --var "$GU=rw+r" --var "fold=0" \
  > $O/ab64.json 2> $O/ab64.err || { tail -20 $O/ab64.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$O/ab64.json').read().strip().splitlines()[-1])
for k,v in sorted(r['ab'].items(), key=lambda kv: kv[1]['mean_ms']): print(f'{v[\"mean_ms\"]:.4f}', k, v['windows'])"
O3=M64:N8192xK8192e3; D3=M64:N8192xK28672e3; GU=M64:N57344xK8192e1
timeout -k 10 600 python3 -u lab/tools/table_ab.py --model llama3-70b --fp8 --batch 64 --rounds 2 --steps 10 --var base \
  --var "$O3=rwk" --var "$O3=rw+r" --var "$D3=rwk" --var "$D3=rw+r" --var "$GU=rw+r" --var "fold=0" \
  > $O/ab70.json 2> $O/ab70.err || { tail -20 $O/ab70.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$O/ab70.json').read().strip().splitlines()[-1])
for k,v in sorted(r['ab'].items(), key=lambda kv: kv[1]['mean_ms']): print(f'{v[\"mean_ms\"]:.4f}', k, v['windows'])"
