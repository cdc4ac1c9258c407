#!/bin/bash
# Round 6: decode attention on v_dot2c_f32_bf16 (+ ping-pong pipeline, native exp2) vs the round-5
# kernel: attention numerics tests on the new default build, then cold microbench and the 64-session
# bench per library (_build_ab/lib_*.so: base = round 5, pp0w4 / pp1w0 = ablations; default = new).
set -o pipefail
O=gpurun_out/${1:-r6attn}
mkdir -p $O
timeout -k 10 300 python3 -m pytest tests/test_kernels_gpu.py -q -x -k "attention or attn" -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for lib in base default pp0w4 pp1w0; do
  if [ $lib = default ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=_build_ab/lib_$lib.so; fi
  timeout -k 10 120 python3 lab/tools/attn_decode_bench.py --batch 64 1 --ctx 170 1024 --heads 32/32 --cold > $O/micro_$lib.txt 2>&1 || { tail -5 $O/micro_$lib.txt; exit 1; }
  echo "== $lib"; grep flash $O/micro_$lib.txt | python3 -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print(r['batch'], r['ctx'], r['us'], r['TBps'])"
done
for rep in 1 2; do for lib in base default pp0w4; do
  if [ $lib = default ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=_build_ab/lib_$lib.so; fi
  timeout -k 10 200 python3 bench.py > $O/b64_${lib}_$rep.json 2> $O/b64_${lib}_$rep.err || { tail -5 $O/b64_${lib}_$rep.err; exit 1; }
  echo "b64 $lib rep$rep $(python3 -c "import json; print(json.loads(open('$O/b64_${lib}_$rep.json').read().strip().splitlines()[-1])['ms_per_step'])")"
done; done
