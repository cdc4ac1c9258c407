set -o pipefail
# multi-rank bench layouts on ONE GPU (gloo: RCCL refuses two ranks per device), after this
# session's kernel / engine changes: pp2, pp8, 4 stages x 2 replicas, 70B fp8 pp8 (W8A16)
O=gpurun_out/r2_rehearsal2
mkdir -p $O
export MPAMD_DIST_BACKEND=gloo MPAMD_CHANNEL_DATA=gloo
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
MPAMD_KV_GB=12 timeout -k 10 400 $R --nproc-per-node 2 --master-port 29611 bench.py --gpus 2 --steps 4 --warmup 2 > $O/reh_pp2.log 2>&1 && \
MPAMD_KV_GB=8 timeout -k 10 500 $R --nproc-per-node 8 --master-port 29612 bench.py --gpus 8 --steps 4 --warmup 2 > $O/reh_pp8.log 2>&1 && \
MPAMD_KV_GB=8 timeout -k 10 500 $R --nproc-per-node 8 --master-port 29613 bench.py --gpus 8 --replicas 2 --steps 4 --warmup 2 > $O/reh_pp4dp2.log 2>&1 && \
MPAMD_KV_GB=8 timeout -k 10 600 $R --nproc-per-node 8 --master-port 29614 bench.py --gpus 8 --model llama3-70b --fp8 --batch 16 --steps 3 --warmup 1 > $O/reh_70b_pp8.log 2>&1
