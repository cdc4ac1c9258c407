#!/bin/bash
# Round 5: phase 2 rehearsed at world 8 on one GPU (8 gloo-staged ranks: RCCL refuses two ranks per
# device), Llama-2-7B pp8 and Llama-3-70B fp8 pp8; both phases must draw identical tokens.
set -o pipefail
O=gpurun_out/${1:-r5l}
mkdir -p $O
export MPAMD_DIST_BACKEND=gloo MPAMD_CHANNEL_DATA=gloo
MPAMD_KV_GB=2 timeout -k 10 400 python3 bench.py --gpus 8 --steps 8 --warmup 2 --phase2 gloo > $O/p2_pp8.json 2> $O/p2_pp8.err || { tail -20 $O/p2_pp8.err; exit 1; }
MPAMD_KV_GB=3 timeout -k 10 500 python3 bench.py --gpus 8 --model llama3-70b --fp8 --batch 16 --steps 6 --warmup 2 --phase2 gloo > $O/p2_70b_pp8.json 2> $O/p2_70b_pp8.err || { tail -20 $O/p2_70b_pp8.err; exit 1; }
for f in p2_pp8 p2_70b_pp8; do python3 -c "
import json
r=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); print('$f', r['config']['parallelism'], r['ms_per_step'], r['data_plane'], json.dumps(r.get('phase2')))"; done
