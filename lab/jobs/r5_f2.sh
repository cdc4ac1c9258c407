#!/bin/bash
# Round 5: GQA decode attention with the fold's loads issued ahead of the K / V stream - GPU
# tests, 70B bench, and the 70B per-kernel trace.
set -o pipefail
O=gpurun_out/${1:-r5f2}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_qkv_fold_gpu.py \
  tests/test_kernels_gpu.py -k "fold or mfma or gqa or attention" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70.json 2> $O/b70.err || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/b70.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p70 -o run -- python3 bench.py --model llama3-70b --fp8 --steps 10 --warmup 3 > $O/b70_prof.json 2> $O/b70_prof.err || exit 1
F=$(find $O/p70 -name "*kernel_stats.csv" | head -1)
python3 - "$F" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{float(r["AverageNs"])/1000:8.2f} us avg  {int(r["Calls"]):6d} calls  {r["Name"][:70]}')
PY
