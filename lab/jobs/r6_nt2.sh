#!/bin/bash
# Round 6, after r6_nt: the new default (reduce outputs sc1 on 4096-wide rows, nontemporal on wider)
# vs rednt (nontemporal on every width, -DMP_SKR_WT_MAXN=0) vs slabnt (split-K slabs nontemporal
# instead of sc1, -DMP_SLAB_SC1=2).  Tests on the default and on each library, then 7B 64 sessions,
# batch 1 and 70B fp8 interleaved.
set -o pipefail
O=gpurun_out/${1:-r6nt2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fused_norm.py tests/test_mx_gpu.py tests/test_executor_gpu.py > $O/tests_default.log 2>&1 || { tail -30 $O/tests_default.log; exit 1; }
tail -1 $O/tests_default.log
for v in rednt slabnt; do
  MPAMD_KERNEL_LIB=lab/_ab/_mpamd_$v.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fused_norm.py > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
for r in 1 2 3; do
  for v in default rednt slabnt; do
    if [ $v = default ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_$v.so; fi
    timeout -k 10 200 python3 bench.py > $O/b64_${v}_$r.json 2> $O/b64_${v}_$r.err || { tail -5 $O/b64_${v}_$r.err; exit 1; }
    if [ $v != rednt ]; then
      timeout -k 10 200 python3 bench.py --batch 1 > $O/b1_${v}_$r.json 2> $O/b1_${v}_$r.err || { tail -5 $O/b1_${v}_$r.err; exit 1; }
      timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70_${v}_$r.json 2> $O/b70_${v}_$r.err || { tail -5 $O/b70_${v}_$r.err; exit 1; }
    fi
    for f in b64 b1 b70; do [ -f $O/${f}_${v}_$r.json ] && python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/${f}_${v}_$r.json; done
  done
done
exit 0
