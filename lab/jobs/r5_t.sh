#!/bin/bash
# Round 5: what the per-step host<->device copies cost a 64-session decode step (timing lab).
set -o pipefail
O=gpurun_out/${1:-r5t}
mkdir -p $O
for v in old new old2 new2 old3 new3; do
  case $v in old*) f="--old-ev";; new*) f="";; esac
  timeout -k 10 200 python3 lab/tools/copy_ab.py $f -- --steps 30 --warmup 5 > $O/$v.json 2> $O/$v.err || exit 1
  python3 -c "
import json
r=json.loads([l for l in open('$O/$v.json') if l.startswith('{')][-1]); print('$v', r['ms_per_step'], r['per_stage_ms'])"
done
