#!/bin/bash
# Round 6 final tree: the README's other rows (batch 1, 256 sessions, Llama-3-8B, Llama-2-7B fp8).
set -o pipefail
O=gpurun_out/${1:-r6rows}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { local n=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], d['value'])" $O/$n.json; }
run b1 --batch 1
run b256 --batch 256
run l3b64 --model llama3-8b
run l3b1 --model llama3-8b --batch 1
run f8b64 --fp8
run f8b1 --fp8 --batch 1
