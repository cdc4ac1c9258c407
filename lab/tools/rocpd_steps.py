"""Per-step kernel breakdown from a rocprofv3 (rocpd SQLite) database.

The last ``--steps`` occurrences of a once-per-step marker kernel bound the timed decode steps;
every dispatch between the first and last marker is grouped by short kernel name and
divided by the number of step intervals.  Usage:
    python scripts/rocpd_steps.py gpurun_out/r4q/b64/run_results.db --steps 20 --marker sample
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    n = re.sub(r"^void ", "", n)
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--marker", default="sample")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--seq", type=int, default=0,
                    help="also print the mean duration of the first SEQ dispatches of a step, in order "
                         "(tells apart projections that share one kernel instantiation)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in short(r[0])]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker dispatches")
    lo, hi = marks[-a.steps - 1], marks[-1]
    n = a.steps
    span = (rows[hi][1] - rows[lo][1]) / 1e3 / n
    agg = defaultdict(lambda: [0, 0.0])
    for name, s, e in rows[lo:hi]:
        k = short(name)
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
    busy = sum(v[1] for v in agg.values()) / n
    print(f"steps={n} wall_us/step={span:.1f} busy_us/step={busy:.1f} idle_us/step={span - busy:.1f}")
    for k, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{t / n:9.1f} us {cnt / n:6.1f}x  {k}")
    if a.seq:
        steps = [rows[marks[i]:marks[i + 1]] for i in range(len(marks) - n - 1, len(marks) - 1)]
        width = min(len(st) for st in steps)
        if any(len(st) != width for st in steps):
            print("# steps differ in dispatch count; per-position means use the shortest")
        print(f"# first {min(a.seq, width)} dispatches of a step (mean us over {n} steps)")
        for j in range(min(a.seq, width)):
            d = sum((st[j][2] - st[j][1]) / 1e3 for st in steps) / n
            print(f"{j:4d} {d:9.1f} us  {short(steps[0][j][0])}")


if __name__ == "__main__":
    main()
