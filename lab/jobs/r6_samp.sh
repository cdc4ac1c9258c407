#!/bin/bash
# Round 6: the split sampler (8K-id chunk workgroups + merge) for Llama-2's 32K vocabulary at 1 and 64
# sessions vs the single-workgroup sampler (MPAMD_SAMPLE_SPLIT_MIN=32000 vs default), interleaved.
set -o pipefail
O=gpurun_out/${1:-r6samp}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in base split; do
    if [ $v = split ]; then export MPAMD_SAMPLE_SPLIT_MIN=32000; else unset MPAMD_SAMPLE_SPLIT_MIN; fi
    for b in 1 64; do
      timeout -k 10 200 python3 bench.py --batch $b --steps 40 > $O/b${b}_${v}_$r.json 2> $O/b${b}_${v}_$r.err || { tail -5 $O/b${b}_${v}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/b${b}_${v}_$r.json
    done
  done
done
