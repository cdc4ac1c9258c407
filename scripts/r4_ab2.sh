#!/bin/bash
# Llama-3-70B fp8: 4 ring slots for the 14-tile W8A16 gate/up form (-DMP_F8_DEEP=2 ablation library) vs default, alternating.
set -o pipefail
OUT=gpurun_out/${1:-r4ab2}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_def$i.json 2> $OUT/b70_def$i.err || exit 1
  MPAMD_KERNEL_LIB=$PWD/ablation/_mpamd_kernels_f8deep2.so timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70_deep$i.json 2> $OUT/b70_deep$i.err || exit 1
done
