#!/bin/bash
# Round 6: decode projections with their weights cold (rotated over 1 GiB) vs resident in the 256 MB
# Infinity Cache (1-4 copies): what a weight prefetch into the MALL ahead of the consumer could buy.
set -o pipefail
O=gpurun_out/${1:-r6mall}
mkdir -p $O
for shape in "4096 4096 3" "12288 4096 0" "22016 4096 0" "4096 11008 3"; do
  set -- $shape
  for c in 0 4 1; do
    timeout -k 10 120 python3 lab/tools/o_probe.py --N $1 --K $2 --epi $3 --copies $c --ms 1,64 --iters 48 >> $O/mall.txt 2>&1 || { tail -5 $O/mall.txt; exit 1; }
  done
done
grep "us/launch" $O/mall.txt
