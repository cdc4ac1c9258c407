#!/usr/bin/env python3
"""Per-kernel breakdown of ONE decode step from a rocprofv3 SQLite trace: the kernels between the
last two sampler launches (the step boundary), grouped by kernel, plus the inter-kernel gaps.
Usage: prof_step.py run_results.db [step_from_end=1]"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = db.execute("select name, grid_x, start, end from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if r[0].startswith("mp::sample_kernel")]
a, b = idx[-1 - back], idx[-back]
step = rows[a + 1:b + 1]
span = (step[-1][3] - step[0][2]) / 1e3
d = collections.defaultdict(list)
for r in step:
    d[(r[0].split("(")[0][:60], r[1])].append((r[3] - r[2]) / 1e3)
busy = sum(sum(v) for v in d.values())
print(f"{len(step)} kernels, step span {span:.1f} us, kernel time {busy:.1f} us ({100 * busy / span:.0f}% busy)")
print(f"{'total_us':>9} {'n':>4} {'avg':>7} {'min':>7} {'max':>7}  kernel [grid]")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v):9.1f} {len(v):4d} {sum(v) / len(v):7.2f} {min(v):7.2f} {max(v):7.2f}  {k[0]} [{k[1]}]")
first = [(r[0].split("(")[0][:48], (r[3] - r[2]) / 1e3) for r in step[:24]]
print("first kernels of the step:", ", ".join(f"{n} {t:.1f}" for n, t in first))
