#!/bin/bash
# Fold decided end to end at warm-up (7B MHA, 70B fp8 GQA) + a kernel trace of the 64 x 128 prefill.
set -o pipefail
OUT=gpurun_out/${1:-r4c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/b64.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --model llama3-70b --fp8 --steps 8 --warmup 2 > $OUT/b70.log 2>&1 || exit 1
MPAMD_QKV_FOLD=0 timeout -k 10 400 python bench.py --model llama3-70b --fp8 --steps 8 --warmup 2 > $OUT/b70_nofold.log 2>&1 || exit 1
timeout -k 10 150 python scripts/prefill_bench.py --batch 64 --prompt-len 128 --repeats 3 > $OUT/prefill.log 2>&1 || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/profp -o run -- python3 $GRAFT_REPO_ROOT/scripts/prefill_bench.py --batch 64 --prompt-len 128 --repeats 2 > $GRAFT_REPO_ROOT/$OUT/prof_prefill.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
DB=$(find /tmp/profp -name "*.db" | head -1)
python scripts/prof_db_summary.py "$DB" 0.33 > $OUT/kernels_prefill.txt 2>&1
