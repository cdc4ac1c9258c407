#!/bin/bash
# End-of-round verification on the final tree: full GPU suite, smoke, driver-config bench, batch 1.
set -o pipefail
OUT=gpurun_out/${1:-r4final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --batch 1 --steps 40 --warmup 8 > $OUT/b1.log 2>&1 || exit 1
