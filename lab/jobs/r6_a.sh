#!/bin/bash
# Round 6: write the decode-kernel table on this box, then run the GPU suite and the 64-session bench
# from it (the same tree the driver will run).
set -o pipefail
O=gpurun_out/${1:-r6a}
mkdir -p $O
T=global_capstone_design_distributed-inference-of-llms-over-the-internet_amd/ops/tuned/decode_kernels_gfx950.json
timeout -k 10 900 python3 -u -m src.ops.tune --out $O/decode_kernels_gfx950.json > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
cp $O/decode_kernels_gfx950.json $T
tail -3 $O/tune.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 200 python3 bench.py > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
tail -1 $O/b64.json
