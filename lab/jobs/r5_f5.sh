#!/bin/bash
# Round 5: kernel-level A/B of two builds of the GQA decode attention (fold forced on), 70B fp8.
set -o pipefail
O=gpurun_out/${1:-r5f5}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in new old; do
  L=""; [ $v = old ] && L="--lib labbin/_mpamd_kernels_old.so"
  timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p_$v -o run -- python3 lab/tools/fold_ab.py --fold on $L -- --model llama3-70b --fp8 --steps 10 --warmup 3 > $O/b70_$v.json 2> $O/b70_$v.err || exit 1
  DB=$(find $O/p_$v -name "*.db" | head -1)
  echo "== $v"; python3 lab/tools/rocpd_steps.py $DB --steps 10 | head -6; rm -rf $O/p_$v
done
