#!/bin/bash
# Round 6: batch-1 MHA decode attention vs its split-K slice floor (cold KV).
set -o pipefail
O=gpurun_out/${1:-r6b1attn}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for mp in 16 32 64 128 256; do
  timeout -k 10 120 python3 lab/tools/attn_decode_bench.py --batch 1 --ctx 150 170 300 1024 --heads 32/32 --cold --min-part $mp > $O/mp$mp.txt 2>&1 || { tail -5 $O/mp$mp.txt; exit 1; }
  echo "min-part $mp"; grep -v "^#" $O/mp$mp.txt | tail -4
done
