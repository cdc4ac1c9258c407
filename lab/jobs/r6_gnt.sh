#!/bin/bash
# Round 6: non-temporal K/V page loads in the GQA attention kernels (MP_GQA_KV_NT=1, default) vs the
# default cache policy (ablation library -DMP_GQA_KV_NT=0): attention / executor / MX tests, then
# Llama-3-8B bf16 and Llama-3-70B fp8 at 64 sessions interleaved.
set -o pipefail
O=gpurun_out/${1:-r6gnt}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_mx_gpu.py tests/test_qkv_fold_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in nt def; do
    if [ $v = nt ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_gkv0.so; fi
    timeout -k 10 200 python3 bench.py --model llama3-8b > $O/b8_${v}_$r.json 2> $O/b8_${v}_$r.err || { tail -5 $O/b8_${v}_$r.err; exit 1; }
    timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70_${v}_$r.json 2> $O/b70_${v}_$r.err || { tail -5 $O/b70_${v}_$r.err; exit 1; }
    for f in b8 b70; do python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/${f}_${v}_$r.json; done
  done
done
