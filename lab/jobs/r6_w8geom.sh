#!/bin/bash
# Round 6: W8A16 split-K ring geometry (the MX form gained from 4-tile groups / half the splits):
# isolated projections under MPAMD_RWK_GEOM per process.
set -o pipefail
O=gpurun_out/${1:-r6w8geom}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for g in base "512:4:2:1,256:4:4:1" "512:2:1:1,256:2:2:1" "256:4:2:1"; do
  tag=$(echo "$g" | tr ':,' '_-')
  if [ "$g" = base ]; then unset MPAMD_RWK_GEOM; else export MPAMD_RWK_GEOM="$g"; fi
  timeout -k 10 300 python3 lab/tools/mx_ab.py --ms 64,32 --shapes 70b.o,70b.down,7b.o,7b.down > $O/$tag.jsonl 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  echo "== $g"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d['shape'], d['M'], 'w8a16', d['w8a16'], 'mx', d['mx'])" $O/$tag.jsonl
done
