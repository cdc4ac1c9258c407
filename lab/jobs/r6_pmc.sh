#!/bin/bash
# Round 6: what limits the 64-row o projection (N 4096 x K 4096, fused-norm producer
# epilogue) against its M = 1 run - one rocprofv3 --pmc pass per counter block (<= 8 SQ, 4 TCC, 4 TCP,
# 2 TA, 2 TD, 2 GRBM), plus the plain timing of both.
set -o pipefail
O=gpurun_out/${1:-r6pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PROG="python3 lab/tools/o_probe.py --N 4096 --K 4096 --epi 3 --ms 1,64 --iters 24"
timeout -k 10 120 $PROG > $O/timing.txt 2>&1 || { cat $O/timing.txt; exit 1; }
cat $O/timing.txt
i=0
for set in "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum" \
           "TCC_EA0_RDREQ_LEVEL_sum TCC_LATENCY_FIFO_FULL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUBBLE_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum" \
           "TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
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
        if "gemm" not in name and "reduce" not in name:
            continue
        key = name.split("(")[0].replace("void ", "")[:60] + f" grid={r.get('Grid_Size', '?')}"
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(f"{O}/summary.txt", "w") as out:
    for k, d in acc.items():
        line = k + " " + str({c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
        print(line)
        out.write(line + "\n")
PY
rm -rf $O/p[0-9]*/
