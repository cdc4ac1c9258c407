#!/bin/bash
# Round 6: nontemporal output stores (lab switch MP_NT_OUT): nt1 = SwiGLU epilogue stores, nt2 = the
# plain-form (8192-wide) split-K reduce row outputs, vs the default.  Tests on each library, then
# 7B 64 sessions and 70B fp8 interleaved.
set -o pipefail
O=gpurun_out/${1:-r6nt}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in nt1 nt2; do
  MPAMD_KERNEL_LIB=lab/_ab/_mpamd_$v.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fused_norm.py tests/test_mx_gpu.py > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
for r in 1 2 3; do
  for v in default nt1 nt2; do
    if [ $v = default ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_$v.so; fi
    if [ $v != nt2 ]; then
      timeout -k 10 200 python3 bench.py > $O/b64_${v}_$r.json 2> $O/b64_${v}_$r.err || { tail -5 $O/b64_${v}_$r.err; exit 1; }
    fi
    timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70_${v}_$r.json 2> $O/b70_${v}_$r.err || { tail -5 $O/b70_${v}_$r.err; exit 1; }
    for f in b64 b70; do [ -f $O/${f}_${v}_$r.json ] && python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/${f}_${v}_$r.json; done
  done
done
exit 0
