#!/bin/bash
# Round 6 final tree: the driver's sequence (GPU suite with -x, smoke, default bench) plus a
# rocprofv3 --stats profile of the default bench and the 70B fp8 bench in both fp8 modes.
set -o pipefail
O=gpurun_out/${1:-r6final}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
tail -1 $O/smoke.txt
timeout -k 10 200 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
tail -1 $O/bench_default.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \; && rm -rf $O/prof
head -12 $O/kernel_stats.csv | cut -c1-150
for m in w8a16 mx; do
  MPAMD_FP8_MODE=$m timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70_$m.json 2> $O/b70_$m.err || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], d['dtype'][:30])" $O/b70_$m.json
done
