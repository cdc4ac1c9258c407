#!/bin/bash
# Round 6: deeper register rings for one-row-tile ring GEMMs (batch 1): ablation libraries
# (-DMP_RW_M1_DEPTH=3 / 4) vs the default, bench.py batch 1 and 16, interleaved.
set -o pipefail
O=gpurun_out/${1:-r6m1d}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in base d3 d4; do
    case $v in base) unset MPAMD_KERNEL_LIB;; d3) export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_m1d3.so;; d4) export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_m1d4.so;; esac
    for b in 1 16; do
      timeout -k 10 200 python3 bench.py --batch $b --steps 40 > $O/b${b}_${v}_$r.json 2> $O/b${b}_${v}_$r.err || { tail -5 $O/b${b}_${v}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/b${b}_${v}_$r.json
    done
  done
done
