#!/bin/bash
# Round 6: SwiGLU epilogue with quad-transposed 8-byte packed stores (MP_EPI1_WIDE=1, default) vs the
# 2-byte stores (ablation library -DMP_EPI1_WIDE=0): GEMM / candidate / executor tests on the new
# default, then 7B 64 / 1 sessions and 70B fp8 interleaved.
set -o pipefail
O=gpurun_out/${1:-r6e1w}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_kernel_candidates_gpu.py tests/test_executor_gpu.py tests/test_fused_norm.py tests/test_mx_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in wide narrow; do
    if [ $v = wide ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_e1n.so; fi
    for b in 64 1; do
      timeout -k 10 200 python3 bench.py --batch $b > $O/b${b}_${v}_$r.json 2> $O/b${b}_${v}_$r.err || { tail -5 $O/b${b}_${v}_$r.err; exit 1; }
    done
    if [ $r -le 2 ]; then
      timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70_${v}_$r.json 2> $O/b70_${v}_$r.err || { tail -5 $O/b70_${v}_$r.err; exit 1; }
    fi
    for f in b64 b1 b70; do [ -f $O/${f}_${v}_$r.json ] && python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/${f}_${v}_$r.json; done
  done
done
exit 0
