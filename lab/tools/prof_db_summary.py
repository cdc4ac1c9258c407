#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite (rocpd) kernel trace: per-kernel time over the last third of the
dispatches (decode steady state).  Usage: prof_db_summary.py run_results.db [fraction | <N>ms]
(``40ms``: the kernels that start in the trace's last 40 ms instead of a fraction of them)"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
arg = sys.argv[2] if len(sys.argv) > 2 else "0.33"
rows = db.execute("select name, grid_x, grid_y, grid_z, start, end, vgpr_count from kernels order by start").fetchall()
if arg.endswith("ms"):
    t_end = max(r[5] for r in rows)
    tail = [r for r in rows if r[4] >= t_end - float(arg[:-2]) * 1e6]
else:
    tail = rows[-int(len(rows) * float(arg)):]
d = collections.defaultdict(list)
for name, gx, gy, gz, s, e, vg in tail:
    d[(name.split("(")[0][:60], f"{gx}x{gy}x{gz}", vg)].append(e - s)
tot = sum(sum(v) for v in d.values())
span = tail[-1][5] - tail[0][4]
print(f"{'total_us':>10} {'n':>5} {'avg_us':>8} {'%':>5} {'vgpr':>4}  kernel [grid]")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v)/1e3:10.1f} {len(v):5d} {sum(v)/len(v)/1e3:8.2f} {100*sum(v)/tot:5.1f} {k[2]:4d}  {k[0]} [{k[1]}]")
print(f"kernel time {tot/1e6:.2f} ms over a {span/1e6:.2f} ms window ({100*tot/span:.0f}% busy)")
