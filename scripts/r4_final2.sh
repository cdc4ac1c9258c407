#!/bin/bash
# Verification on the late-round tree (4-wave decode attention default): full GPU suite, smoke,
# driver-config bench, and the README configs (batch 1, batch 1 x prompt 2048, 128 / 256 sessions,
# Llama-3-8B, Llama-3-70B fp8).
set -o pipefail
OUT=gpurun_out/${1:-r4final2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 200 python bench.py --batch 1 --steps 40 --warmup 8 > $OUT/b1.json 2> $OUT/b1.err || exit 1
timeout -k 10 200 python bench.py --batch 1 --prompt-len 2048 --steps 40 --warmup 8 > $OUT/b1_p2048.json 2> $OUT/b1_p2048.err || exit 1
timeout -k 10 200 python bench.py --batch 128 > $OUT/b128.json 2> $OUT/b128.err || exit 1
timeout -k 10 250 python bench.py --batch 256 > $OUT/b256.json 2> $OUT/b256.err || exit 1
timeout -k 10 200 python bench.py --model llama3-8b > $OUT/l3.json 2> $OUT/l3.err || exit 1
timeout -k 10 400 python bench.py --model llama3-70b --fp8 > $OUT/b70.json 2> $OUT/b70.err || exit 1
