#!/bin/bash
# Round 5: (1) stage-local recovery (--replay_cache) on the GPU path, one MI355X: client + 3 stage
# servers on the card, the tail SIGKILLed mid-decode, its spare rebuilds by one prefill;
# (2) BASELINE config 5 at its own shape: Llama-3-70B fp8 (W8A16), 2 replicas x 4 stages = 8 ranks
# on the one card (gloo-staged payloads: RCCL refuses two ranks per device), stage rank 5 SIGKILLed
# after 20 micro-batch steps, its replica's sessions re-placed on the survivor.
set -o pipefail
O=gpurun_out/${1:-r5b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
    tests/test_stage_local_recovery.py -k one_gpu > $O/stage_local_gpu.log 2>&1 || exit 1
MPAMD_DIST_BACKEND=gloo MPAMD_CHANNEL_DATA=gloo MPAMD_KV_GB=4 MPAMD_DRILL_TIMEOUT=240 \
    timeout -k 10 1000 python bench.py --gpus 8 --replicas 2 --model llama3-70b --fp8 --batch 16 --steps 24 \
    --kill 5@20 --dump-tokens $O/drill70_tokens.json > $O/drill70.json 2> $O/drill70.log
