set -o pipefail
# multi-rank bench layouts on ONE GPU with the round-4 tree (gloo default group and device channel:
# RCCL refuses two ranks per device): the driver's torchrun launch at pp2 / pp4 / pp8, and the
# self-spawned launch (no torchrun) at pp4.  Step times are meaningless (ranks time-share one GPU,
# hops staged through host memory); what is checked is that every layout completes and prints its line.
O=gpurun_out/r4u
mkdir -p $O
export MPAMD_DIST_BACKEND=gloo MPAMD_CHANNEL_DATA=gloo
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
MPAMD_KV_GB=12 timeout -k 10 400 $R --nproc-per-node 2 --master-port 29611 bench.py --gpus 2 --steps 4 --warmup 2 > $O/reh_pp2.log 2>&1 && \
MPAMD_KV_GB=10 timeout -k 10 450 $R --nproc-per-node 4 --master-port 29612 bench.py --gpus 4 --steps 4 --warmup 2 > $O/reh_pp4.log 2>&1 && \
MPAMD_KV_GB=8 timeout -k 10 500 $R --nproc-per-node 8 --master-port 29613 bench.py --gpus 8 --steps 4 --warmup 2 > $O/reh_pp8.log 2>&1 && \
MPAMD_KV_GB=10 timeout -k 10 450 python bench.py --gpus 4 --steps 4 --warmup 2 > $O/reh_pp4_selfspawn.log 2>&1
