#!/bin/bash
# Round 6, after r6_nt2: split-K slabs sc1 (default) vs nontemporal (slabnt), 4 interleaved rounds of
# 7B 64 sessions and 70B fp8.
set -o pipefail
O=gpurun_out/${1:-r6nt3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2 3 4; do
  for v in default slabnt; do
    if [ $v = default ]; then unset MPAMD_KERNEL_LIB; else export MPAMD_KERNEL_LIB=lab/_ab/_mpamd_$v.so; fi
    timeout -k 10 200 python3 bench.py > $O/b64_${v}_$r.json 2> $O/b64_${v}_$r.err || { tail -5 $O/b64_${v}_$r.err; exit 1; }
    timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70_${v}_$r.json 2> $O/b70_${v}_$r.err || { tail -5 $O/b70_${v}_$r.err; exit 1; }
    for f in b64 b70; do python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'])" $O/${f}_${v}_$r.json; done
  done
done
