#!/usr/bin/env python3
"""Idle time between the kernels of the last decode steps of a rocprofv3 (rocpd SQLite) trace:
steps are bounded by the once-per-step sampler kernel; every inter-kernel gap is attributed to the
(previous kernel -> next kernel) pair, summed per step.  Answers "where does the GPU wait" (host
launch gaps, graph boundaries, copies) next to rocpd_steps.py's "where does it compute".
Usage: prof_gaps.py run_results.db [--steps 20] [--top 25]"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name.split("(")[0])
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--marker", default="sample_kernel")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    lo, hi = marks[-a.steps - 1], marks[-1]
    gaps = defaultdict(lambda: [0, 0.0])
    hist = defaultdict(int)
    total = 0.0
    for i in range(lo, hi):
        g = (rows[i + 1][1] - rows[i][2]) / 1e3
        if g <= 0:
            continue
        total += g
        key = (short(rows[i][0]), short(rows[i + 1][0]))
        gaps[key][0] += 1
        gaps[key][1] += g
        hist[min(int(g), 20)] += 1
    n = a.steps
    print(f"steps={n} gap_us/step={total / n:.1f}")
    print("gap histogram (us bucket: count/step):", {k: round(v / n, 1) for k, v in sorted(hist.items())})
    for (p, q), (cnt, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{t / n:8.1f} us {cnt / n:6.1f}x  {p}  ->  {q}")


if __name__ == "__main__":
    main()
