#!/bin/bash
# Round 6: split-K ring geometry (column-group width NT x K splits S) of the 7B 64-session o / down
# projections and the qkv fold partials, whole decode step (lab/tools/table_ab.py base), one
# MPAMD_RWK_GEOM per process, interleaved.
set -o pipefail
O=gpurun_out/${1:-r6geom}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for g in base "256:2:2:0" "256:8:8:0" "768:8:2:0" "256:2:2:0,768:8:2:0"; do
    tag=$(echo "$g" | tr ':,' '_-')
    if [ "$g" = base ]; then unset MPAMD_RWK_GEOM; else export MPAMD_RWK_GEOM="$g"; fi
    timeout -k 10 300 python3 lab/tools/table_ab.py --batch 64 --rounds 2 --steps 20 > $O/${tag}_$r.json 2> $O/${tag}_$r.err || { tail -5 $O/${tag}_$r.err; exit 1; }
    echo "$g r$r $(tail -1 $O/${tag}_$r.json)"
  done
done
