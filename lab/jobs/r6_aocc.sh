#!/bin/bash
# Round 6: decode attention occupancy (launch-bounds minimum waves per SIMD 4 / 5 / 6; 5 and 6 spill
# 20 / 38 VGPRs): attention microbench (64 x 170 cold and warm, batch 1) and bench.py 64 sessions.
set -o pipefail
O=gpurun_out/${1:-r6aocc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in base aw5 aw6; do
    if [ $v = base ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_$v.so; fi
    timeout -k 10 120 python3 lab/tools/attn_decode_bench.py --batch 64 --ctx 170 --heads 32/32 --cold > $O/m_${v}_$r.txt 2>&1 || { tail -3 $O/m_${v}_$r.txt; exit 1; }
    timeout -k 10 200 python3 bench.py --steps 40 > $O/b64_${v}_$r.json 2> $O/b64_${v}_$r.err || { tail -5 $O/b64_${v}_$r.err; exit 1; }
    echo "$v r$r micro $(grep flash_decode $O/m_${v}_$r.txt | python3 -c 'import sys,json; print([json.loads(l)["us"] for l in sys.stdin])') bench $(python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['ms_per_step'])" $O/b64_${v}_$r.json)"
  done
done
