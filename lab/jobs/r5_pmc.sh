#!/bin/bash
# Round 5: counters behind the per-CU intake limit - the tiled kernel (qkv, 256 rows) and the
# 64-row ring (qkv), each its own rocprofv3 --pmc pass (<= 8 SQ / 4 TCC / 2 TA / 2 GRBM counters).
set -o pipefail
O=gpurun_out/${1:-r5pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -oE "Counter_Name +:\s+(SQ|TCC|TA|TCP|GRBM|TD)_[A-Za-z0-9_]+" $O/avail.txt | awk '{print $NF}' | sort -u > $O/avail_names.txt || true
wc -l < $O/avail_names.txt
PROG="python3 lab/tools/t2d_bench.py --m 256 64 --splits 0 --shapes qkv --iters 10 --ring"
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"; do
  ok=1; for c in $set; do b=${c%_sum}; b=${b%_avr}; grep -qx "$b" $O/avail_names.txt || grep -qx "$c" $O/avail_names.txt || { echo "skip $c"; ok=0; }; done
  [ $ok = 1 ] || continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- $PROG > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for f in sorted(glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        key = "t2d" if "t2d" in name else ("rwk" if "rwk" in name else ("reduce" if "reduce" in name else ("blas" if "Cijk" in name else None)))
        if key is None:
            continue
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", f.split("/")[-3] if "/" in f else f)
    for k, d in acc.items():
        print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
