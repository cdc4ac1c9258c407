#!/bin/bash
# Round 6: decode attention waves per workgroup by grid size (default build: 2 for big grids, 8 for
# small ones, else 4) vs forced 4 / 2 / 8 (_build_ab/lib_nw*.so): attention tests on the default
# build, cold microbench per library, then 64-session and batch-1 benches (default vs nw4).
set -o pipefail
O=gpurun_out/${1:-r6attn2}
mkdir -p $O
timeout -k 10 300 python3 -m pytest tests/test_kernels_gpu.py -q -x -k "attention or attn" -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for lib in default nw4 nw2 nw8; do
  if [ $lib = default ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=_build_ab/lib_$lib.so; fi
  timeout -k 10 120 python3 lab/tools/attn_decode_bench.py --batch 64 16 1 --ctx 170 1024 --heads 32/32 --cold > $O/micro_$lib.txt 2>&1 || { tail -5 $O/micro_$lib.txt; exit 1; }
  echo "== $lib $(grep flash $O/micro_$lib.txt | python3 -c "
import sys, json
print(' | '.join(f\"{r['batch']}x{r['ctx']} {r['us']}us\" for r in map(json.loads, sys.stdin)))")"
done
for rep in 1 2; do for lib in default nw4; do for b in 64 1; do
  if [ $lib = default ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=_build_ab/lib_$lib.so; fi
  timeout -k 10 200 python3 bench.py --batch $b > $O/b${b}_${lib}_$rep.json 2> $O/b${b}_${lib}_$rep.err || { tail -5 $O/b${b}_${lib}_$rep.err; exit 1; }
  echo "b$b $lib rep$rep $(python3 -c "import json; print(json.loads(open('$O/b${b}_${lib}_$rep.json').read().strip().splitlines()[-1])['ms_per_step'])")"
done; done; done
