#!/bin/bash
# Round 6: split-K ring geometry of the 7B 64-session o (K 4096) and down (K 11008) projections
# separately (MPAMD_RWK_GEOM with the K filter), whole decode step, interleaved.
set -o pipefail
O=gpurun_out/${1:-r6geom2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for g in base "256:2:2:0:128" "256:8:8:0:128" "256:2:2:0:344" "256:8:8:0:344"; do
    tag=$(echo "$g" | tr ':,' '_-')
    if [ "$g" = base ]; then unset MPAMD_RWK_GEOM; else export MPAMD_RWK_GEOM="$g"; fi
    timeout -k 10 300 python3 lab/tools/table_ab.py --batch 64 --rounds 2 --steps 20 > $O/${tag}_$r.json 2> $O/${tag}_$r.err || { tail -5 $O/${tag}_$r.err; exit 1; }
    echo "$g r$r $(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ab']['base']['mean_ms'])" $O/${tag}_$r.json)"
  done
done
