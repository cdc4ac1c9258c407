#!/bin/bash
# Round 5: Llama-3-70B fp8 GQA decode attention A/B (MFMA kernel vs pipelined flash-decoding kernel), 64 sessions.
set -o pipefail
O=gpurun_out/${1:-r5h}
mkdir -p $O
timeout -k 10 500 python3 lab/tools/gqa_decode_ab.py --valu -- --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/valu.json 2> $O/valu.err || exit 1
timeout -k 10 500 python3 lab/tools/gqa_decode_ab.py -- --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/mfma.json 2> $O/mfma.err || exit 1
python3 -c "
import json
for n in ('valu','mfma'):
    r=json.loads([l for l in open('$O/'+n+'.json') if l.startswith('{')][-1]); print(n, r['ms_per_step'], r['value'])
"
