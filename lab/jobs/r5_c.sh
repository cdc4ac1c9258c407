#!/bin/bash
# Round 5: GPU suite + 1-GPU bench (driver command) on the pruned tree.
set -o pipefail
O=gpurun_out/${1:-r5c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b64.json 2> $O/b64.err && cat $O/b64.json
