#!/bin/bash
# Round 6, after r6_ntld: 4 more interleaved rounds of 7B 64 sessions and batch 1, reduce slab loads
# nontemporal (ablation library -DMP_SKR_NTLOAD=1) vs the default.
set -o pipefail
O=gpurun_out/${1:-r6ntld2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2 3 4; do
  for v in ntld default; do
    if [ $v = default ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_ntld.so; fi
    for b in 64 1; do
      timeout -k 10 200 python3 bench.py --batch $b > $O/b${b}_${v}_$r.json 2> $O/b${b}_${v}_$r.err || { tail -5 $O/b${b}_${v}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/b${b}_${v}_$r.json
    done
  done
done
