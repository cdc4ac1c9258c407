#!/bin/bash
# Round 6 final tree: rocprofv3 --kernel-trace --stats of the default bench (csv summary).
set -o pipefail
O=gpurun_out/${1:-r6final}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" $O/kernel_stats.csv
rm -rf $O/prof
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/kernel_stats.csv')))[:14]: print(r['Name'][:70], r['Calls'], r['TotalDurationNs'], r['Percentage'])"
