#!/bin/bash
# Round 6: GPU suite + benches from the committed kernel table, then a kernel-trace profile.
set -o pipefail
O=gpurun_out/${1:-r6b}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread --durations=15 > $O/pytest.txt 2>&1 || { tail -80 $O/pytest.txt; exit 1; }
tail -20 $O/pytest.txt
timeout -k 10 200 python3 bench.py > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
tail -1 $O/b64.json
timeout -k 10 200 python3 bench.py --batch 1 > $O/b1.json 2> $O/b1.err || { tail -20 $O/b1.err; exit 1; }
tail -1 $O/b1.json
