# One-GPU rehearsal of the multi-stage RCCL pipeline: 2 ranks share cuda:0 (KV pool capped).
set -o pipefail
mkdir -p gpurun_out
export MPAMD_KV_GB=16
timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 8 --warmup 2 > gpurun_out/pp2_rehearsal.log 2>&1
