#!/bin/bash
# Round 6: nontemporal split-K slab stores in the 129..256-row t2d GEMM (MP_T2D_SLAB_ST=2, default)
# vs plain stores (ablation library -DMP_T2D_SLAB_ST=0): GEMM tests, then 7B at 160 / 256 sessions
# interleaved.
set -o pipefail
O=gpurun_out/${1:-r6t2dnt}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_executor_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in nt plain; do
    if [ $v = nt ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_t2d0.so; fi
    for b in 256 160; do
      timeout -k 10 300 python3 bench.py --batch $b > $O/b${b}_${v}_$r.json 2> $O/b${b}_${v}_$r.err || { tail -5 $O/b${b}_${v}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/b${b}_${v}_$r.json
    done
  done
done
