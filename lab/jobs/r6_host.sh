#!/bin/bash
# Round 6: is a shallow stage (a pipeline stage of an 8-GPU Llama-2-7B run: 4 layers) host-bound?
# GPU ms per decode step vs host time per step, 4 / 8 / 32 layers, 64 sessions and batch 1.
set -o pipefail
O=gpurun_out/${1:-r6host}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for b in 64 1; do
  for l in 4 8 32; do
    timeout -k 10 200 python3 lab/tools/decode_host_probe.py --batch $b --layers $l --steps 60 > $O/b${b}_l$l.json 2> $O/b${b}_l$l.err || { tail -5 $O/b${b}_l$l.err; exit 1; }
    cat $O/b${b}_l$l.json
  done
done
