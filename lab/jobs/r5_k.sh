#!/bin/bash
# Round 5 mid-round check: full GPU suite, smoke, and the bench at 64 (driver default) / 1 / 128 / 256 sessions + 70B fp8.
set -o pipefail
O=gpurun_out/${1:-r5k}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 200 python3 bench.py > $O/b64.json 2> $O/b64.err || exit 1
timeout -k 10 200 python3 bench.py --batch 1 > $O/b1.json 2> $O/b1.err || exit 1
timeout -k 10 200 python3 bench.py --batch 128 > $O/b128.json 2> $O/b128.err || exit 1
timeout -k 10 200 python3 bench.py --batch 256 > $O/b256.json 2> $O/b256.err || exit 1
timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70.json 2> $O/b70.err || exit 1
for f in b64 b1 b128 b256 b70; do python3 -c "
import json,sys
r=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); print('$f', r['ms_per_step'], r['value'])"; done
