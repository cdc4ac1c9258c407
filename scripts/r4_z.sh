#!/bin/bash
# Timing experiment (not a serving mode): per-step host copies - seeds H2D skipped, sampler output written into the graph input.
set -o pipefail
OUT=gpurun_out/${1:-r4z}
mkdir -p $OUT
export TMPDIR=/tmp
for mode in base noseed xalias both; do
  unset MPAMD_EXP_NOSEED MPAMD_EXP_XALIAS
  [ $mode = noseed ] && export MPAMD_EXP_NOSEED=1
  [ $mode = xalias ] && export MPAMD_EXP_XALIAS=1
  [ $mode = both ] && export MPAMD_EXP_NOSEED=1 MPAMD_EXP_XALIAS=1
  timeout -k 10 300 python bench.py --gpus 1 --batch 1 > $OUT/b1_$mode.json 2> $OUT/b1_$mode.err || exit 1
  timeout -k 10 300 python bench.py --gpus 1 > $OUT/b64_$mode.json 2> $OUT/b64_$mode.err || exit 1
done
