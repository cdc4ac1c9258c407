#!/bin/bash
# Round 5: graph-input receive target + the bench second phase on one GPU (2 ranks on the card,
# gloo-staged: RCCL refuses two ranks per device): phase 2 over gloo (both phases run, same tokens)
# and phase 2 over RCCL (set-up refused on one device -> reported, headline kept, exit 0).
set -o pipefail
O=gpurun_out/${1:-r5d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_graph_input_gpu.py \
    tests/test_rccl_gpu.py tests/test_engine_gpu.py tests/test_qkv_fold_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
export MPAMD_DIST_BACKEND=gloo MPAMD_CHANNEL_DATA=gloo MPAMD_KV_GB=12
timeout -k 10 400 python bench.py --gpus 2 --steps 8 --warmup 2 --phase2 gloo > $O/p2_gloo.json 2> $O/p2_gloo.err || { tail -30 $O/p2_gloo.err; exit 1; }
cat $O/p2_gloo.json
timeout -k 10 400 python bench.py --gpus 2 --steps 8 --warmup 2 --phase2 rccl --phase2-hop-timeout 30 > $O/p2_rccl.json 2> $O/p2_rccl.err || { tail -30 $O/p2_rccl.err; exit 1; }
cat $O/p2_rccl.json
