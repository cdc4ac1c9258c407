#!/bin/bash
# Replay-cache GPU test; the 16-wave attention threshold (MPAMD_ATTN_WIDE_WGS) at small batches.
set -o pipefail
OUT=gpurun_out/${1:-r4o}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_replay_cache.py > $OUT/pytest_replay.log 2>&1 || exit 1
for w in 512 256 0; do
  MPAMD_ATTN_WIDE_WGS=$w timeout -k 10 120 python scripts/attn_decode_bench.py --batch 1 2 4 8 16 --ctx 170 1024 --heads 32/32 > $OUT/wide_wgs$w.jsonl 2>&1 || exit 1
done
