#!/bin/bash
# Full GPU test suite + smoke on this tree, then the driver-config benches (64 sessions, 70B fp8) with the confirmed-fold policy.
set -o pipefail
OUT=gpurun_out/${1:-r4h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 150 python bench.py > $OUT/bench_default.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --model llama3-70b --fp8 --steps 8 --warmup 2 > $OUT/b70.log 2>&1 || exit 1
for mp in 256 128 64; do
  timeout -k 10 120 python scripts/attn_decode_bench.py --batch 64 --ctx 170 512 --heads 64/8 32/8 --min-part $mp > $OUT/gqa_mp$mp.jsonl 2>&1 || exit 1
done
