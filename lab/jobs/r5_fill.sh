#!/bin/bash
# Lab A/B: fp8 split-K grids sized for one (default) vs two workgroups per CU, Llama-3-70B fp8 bench.
set -o pipefail
O=gpurun_out/${1:-r5fill}
mkdir -p $O
for v in 1 2 1 2; do
  MPAMD_RWK_F8_FILL=$v timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70_fill$v.json 2> $O/b70_fill$v.err || exit 1
  echo fill=$v $(grep -o '"ms_per_step": [0-9.]*' $O/b70_fill$v.json) $(grep -o '"qkv_fold_ab_ms": {[^}]*}' $O/b70_fill$v.json)
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MPAMD_RWK_F8_FILL=2 timeout -k 10 600 rocprofv3 --kernel-trace -d $O/p70 -o run -- python3 bench.py --model llama3-70b --fp8 --steps 10 --warmup 3 > $O/b70_prof.json 2> $O/b70_prof.err || exit 1
DB=$(find $O/p70 -name "*.db" | head -1)
python3 lab/tools/rocpd_steps.py $DB --steps 10 --marker embedding_kernel --seq 16 > $O/b70_kernels_per_step.txt && rm -rf $O/p70 || exit 1
cat $O/b70_kernels_per_step.txt
