#!/bin/bash
# Round 6: why the W8A8-MX split-K kernel is not faster than W8A16 on the 70B o projection (M = 64):
# kernel trace + one rocprofv3 --pmc pass per counter block.
set -o pipefail
O=gpurun_out/${1:-r6mxpmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PROG="python3 lab/tools/mx_ab.py --shapes ${SHAPE:-70b.o} --ms 64 --iters 24"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $PROG > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- $PROG > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if "gemm" not in name and "reduce" not in name and "quant" not in name:
            continue
        key = name.split("(")[0].replace("void ", "")[:70]
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(f"{O}/summary.txt", "w") as out:
    for k, d in acc.items():
        line = k + " " + str({c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
        print(line)
        out.write(line + "\n")
PY
rm -rf $O/p[0-9]*/ $O/kt
python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats.csv')): print(r['Name'][:80], r['Calls'], r['AverageNs'])"
