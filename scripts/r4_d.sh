#!/bin/bash
# 129..256-row decode kernels (tests + 128 / 256-session benches), fold decided at warm-up, 70B fp8,
# and a kernel trace of the 64 x 128 prefill.
set -o pipefail
OUT=gpurun_out/${1:-r4d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_norm.py tests/test_qkv_fold_gpu.py > $OUT/pytest_wide.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention_fa or fa_blocks" > $OUT/pytest_fa.log 2>&1 || exit 1
timeout -k 10 200 python scripts/attn_bench.py --seqs 1x2048 2x2048 1x4096 64x128 --heads 32/32 32/8 --kernels fa4:n fa4:z fa8:n fa8:z > $OUT/attn_pair.jsonl 2>&1 || exit 1
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/b64.log 2>&1 || exit 1
timeout -k 10 120 python scripts/attn_decode_bench.py --batch 64 256 --ctx 170 --heads 32/32 32/8 > $OUT/attn_dec_u4.jsonl 2>&1 || exit 1
MPAMD_ATTN_U=8 timeout -k 10 120 python scripts/attn_decode_bench.py --batch 64 256 --ctx 170 --heads 32/32 32/8 > $OUT/attn_dec_u8.jsonl 2>&1 || exit 1
timeout -k 10 200 python bench.py --batch 128 --steps 16 --warmup 4 > $OUT/b128.log 2>&1 || exit 1
timeout -k 10 250 python bench.py --batch 256 --steps 12 --warmup 4 > $OUT/b256.log 2>&1 || exit 1
cd /tmp && timeout -k 10 250 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof256 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 256 --steps 8 --warmup 3 > $GRAFT_REPO_ROOT/$OUT/prof256.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python scripts/prof_db_summary.py "$(find /tmp/prof256 -name '*.db' | head -1)" 40ms > $OUT/kernels_b256.txt 2>&1
timeout -k 10 400 python bench.py --model llama3-70b --fp8 --steps 8 --warmup 2 > $OUT/b70.log 2>&1 || exit 1
timeout -k 10 150 python scripts/prefill_bench.py --batch 64 --prompt-len 128 --repeats 3 > $OUT/prefill.log 2>&1 || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/profp -o run -- python3 $GRAFT_REPO_ROOT/scripts/prefill_bench.py --batch 64 --prompt-len 128 --repeats 2 > $GRAFT_REPO_ROOT/$OUT/prof_prefill.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python scripts/prof_db_summary.py "$(find /tmp/profp -name '*.db' | head -1)" 0.33 > $OUT/kernels_prefill.txt 2>&1
