#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-kernel time over the last third of the run (decode steady state)."""
import collections
import csv
import sys

path = sys.argv[1]
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.33
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-int(len(rows) * frac):]
d = collections.defaultdict(list)
for r in tail:
    n = r["Kernel_Name"].split("(")[0][:70]
    d[(n, r.get("Grid_Size_X", ""))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in d.values())
span = int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])
print(f"{'total_us':>10} {'n':>5} {'avg_us':>8} {'%':>5}  kernel [grid]")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v)/1e3:10.1f} {len(v):5d} {sum(v)/len(v)/1e3:8.2f} {100*sum(v)/tot:5.1f}  {k[0]} [{k[1]}]")
print(f"kernel time {tot/1e6:.2f} ms over a {span/1e6:.2f} ms window ({100*tot/span:.0f}% busy)")
