#!/bin/bash
# Round 6: the split-K reduce's slab loads with the nontemporal hint (ablation library
# -DMP_SKR_NTLOAD=1) vs the default: fused-norm / executor / kernel tests on
# the variant, then 7B 64 sessions and 70B fp8 interleaved.
set -o pipefail
O=gpurun_out/${1:-r6ntld}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MPAMD_KERNEL_LIB=lab/_ab/_mpamd_ntld.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fused_norm.py tests/test_executor_gpu.py tests/test_qkv_fold_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in default ntld; do
    if [ $v = default ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_ntld.so; fi
    timeout -k 10 200 python3 bench.py > $O/b64_${v}_$r.json 2> $O/b64_${v}_$r.err || { tail -5 $O/b64_${v}_$r.err; exit 1; }
    timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70_${v}_$r.json 2> $O/b70_${v}_$r.err || { tail -5 $O/b70_${v}_$r.err; exit 1; }
    for f in b64 b70; do python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/${f}_${v}_$r.json; done
  done
done
