#!/usr/bin/env python3
"""Per-kernel PMC summary of a rocprofv3 --pmc run (rocpd SQLite): mean counter value and mean
duration per kernel name over the last ``fraction`` of dispatches.
Usage: prof_pmc_summary.py run_results.db [fraction]"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
rows = db.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection "
                  "order by dispatch_id").fetchall()
disp = sorted({r[0] for r in rows})
keep = set(disp[-int(len(disp) * frac):])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for d, name, cn, v, du in rows:
    if d not in keep:
        continue
    n = name.split("(")[0][:64]
    agg[n][cn].append(float(v))
    dur[n][d] = du
for n in sorted(agg, key=lambda k: -sum(dur[k].values())):
    cs = "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(agg[n].items()))
    ds = list(dur[n].values())
    print(f"{n:64s} n={len(ds):4d} dur_us={sum(ds) / len(ds) / 1e3:8.2f}  {cs}")
