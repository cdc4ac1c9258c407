#!/bin/bash
# Round 6 (after the dot2 rewrite): what limits the 64-session MHA decode attention (paged_attn1, 64 x 170, cold):
# VALU vs memory - rocprofv3 --pmc passes over lab/tools/attn_decode_bench.py.
set -o pipefail
O=gpurun_out/${1:-r6apmc2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PROG="python3 lab/tools/attn_decode_bench.py --batch 64 --ctx 170 --heads 32/32 --cold"
timeout -k 10 120 $PROG > $O/timing.txt 2>&1 || { cat $O/timing.txt; exit 1; }
cat $O/timing.txt
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_LEVEL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_avr TD_TD_BUSY_sum" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
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
        if "attn" not in name:
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
