#!/bin/bash
# Round 6: world-8 rehearsal on one GPU (8 gloo-staged ranks share the card: RCCL refuses two ranks per
# device).  Headline: every decode hop received straight into the receiver's decode-graph input
# (host-staged copy into it); phase 2: the same sessions through the receive slab + copy path.  The two
# must draw identical tokens.  Llama-2-7B pp8 and Llama-3-70B fp8 pp8.
set -o pipefail
O=gpurun_out/${1:-r6l}
mkdir -p $O
export MPAMD_DIST_BACKEND=gloo MPAMD_CHANNEL_DATA=gloo
MPAMD_KV_GB=2 timeout -k 10 400 python3 bench.py --gpus 8 --steps 8 --warmup 2 --phase2 gloo --phase2-recv-into off > $O/pp8.json 2> $O/pp8.err || { tail -20 $O/pp8.err; exit 1; }
MPAMD_KV_GB=3 timeout -k 10 500 python3 bench.py --gpus 8 --model llama3-70b --fp8 --batch 16 --steps 6 --warmup 2 --phase2 gloo --phase2-recv-into off > $O/pp8_70b.json 2> $O/pp8_70b.err || { tail -20 $O/pp8_70b.err; exit 1; }
for f in pp8 pp8_70b; do python3 -c "
import json
r=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); print('$f', r['config']['parallelism'], r['ms_per_step'], r['data_plane'], 'into', r['hop_recv_into_graph_per_rank'], json.dumps(r.get('phase2')))"; done
