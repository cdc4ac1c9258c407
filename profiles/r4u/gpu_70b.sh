#!/bin/bash
# Llama-3-70B fp8 (W8A16) pp8 on ONE GPU (gloo data plane, 8 ranks time-share the card): the 8-stage
# code path with this round's per-stage warm-up / fold A/B / balanced splits, as in profiles/r2_rehearsal2.
set -o pipefail
OUT=gpurun_out/${1:-r4ae}
mkdir -p $OUT
export TMPDIR=/tmp MPAMD_DIST_BACKEND=gloo MPAMD_CHANNEL_DATA=gloo
MPAMD_KV_GB=8 timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29615 bench.py --gpus 8 --model llama3-70b --fp8 --batch 16 --steps 3 --warmup 1 > $OUT/reh_70b_pp8.log 2>&1 || exit 1
