#!/usr/bin/env python3
"""Host-side view of the last decode steps of a rocprofv3 trace taken with --hip-trace
(--kernel-trace too): HIP API calls of the timed window grouped by name (calls and host time per
step), the long ones listed with what the GPU was doing meanwhile.  Finds the host waits that
leave the GPU idle (synchronous copies, event / stream synchronisation).
Usage: prof_host.py run_results.db [--steps 20] [--min-us 15]"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--marker", default="sample_kernel")
    ap.add_argument("--min-us", type=float, default=15.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [r for r in ks if a.marker in r[0]]
    t0, t1 = marks[-a.steps - 1][1], marks[-1][1]
    regs = c.execute("select name, start, end, tid from regions where start >= ? and start < ? order by start",
                     (t0, t1)).fetchall()
    agg = defaultdict(lambda: [0, 0.0])
    for name, s, e, tid in regs:
        agg[name][0] += 1
        agg[name][1] += (e - s) / 1e3
    n = a.steps
    print(f"window {(t1 - t0) / 1e3 / n:.1f} us/step, {len(regs) / n:.0f} API calls/step")
    for name, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"{t / n:9.1f} us {cnt / n:7.1f}x  {name}")
    print(f"\ncalls >= {a.min_us} us (last 2 steps):")
    t2 = marks[-3][1]
    for name, s, e, tid in regs:
        if s >= t2 and (e - s) / 1e3 >= a.min_us:
            busy = [k[0].split("(")[0][:40] for k in ks if k[1] < e and k[2] > s]
            print(f"  +{(s - t2) / 1e3:8.1f} us  {name}  {(e - s) / 1e3:.1f} us  tid {tid}  gpu: {busy[:3]}")


if __name__ == "__main__":
    main()
