#!/bin/bash
# Round 6: ring-tail loads to the L2-resident activation (MP_RING_TAIL_L2, default 1) vs the old tail
# (ablation library, -DMP_RING_TAIL_L2=0): GEMM oracle tests, then 7B 64 / 1 sessions and 70B fp8
# benches interleaved.
set -o pipefail
O=gpurun_out/${1:-r6tail}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fused_norm.py tests/test_mx_gpu.py tests/test_kernel_candidates_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_tail0.so; else unset MPAMD_KERNEL_LIB; fi
    for b in 64 1; do
      timeout -k 10 200 python3 bench.py --batch $b > $O/b${b}_${v}_$r.json 2> $O/b${b}_${v}_$r.err || { tail -5 $O/b${b}_${v}_$r.err; exit 1; }
    done
    timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70_${v}_$r.json 2> $O/b70_${v}_$r.err || { tail -5 $O/b70_${v}_$r.err; exit 1; }
    for f in b64 b1 b70; do python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/${f}_${v}_$r.json; done
  done
done
