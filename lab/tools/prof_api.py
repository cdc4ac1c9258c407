#!/usr/bin/env python3
"""HIP API calls of a rocprofv3 --hip-trace run (rocpd SQLite): the calls that BLOCK the host.

Prints the database's views (schema probe), the API calls by total host time, and the long calls
(>= --min-us) of the last --steps decode steps (steps delimited by the sampler kernel), each with
the kernel that was running on the GPU when it returned - to find the host wait that leaves the
GPU idle at the decode step boundary."""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--min-us", type=float, default=20.0)
    ap.add_argument("--marker", default="sample_kernel")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    views = [r[0] for r in c.execute("select name from sqlite_master where type in ('view','table')")]
    print("views:", ", ".join(sorted(v for v in views if not v.startswith("rocpd_info"))))
    cols = [r[1] for r in c.execute("pragma table_info(regions)")]
    print("regions columns:", cols)
    regs = c.execute("select name, start, end from regions order by start").fetchall()
    ks = c.execute("select name, start, end from kernels order by start").fetchall()
    tot = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for n, s, e in regs:
        t = tot[n]
        t[0] += 1
        t[1] += (e - s) / 1e3
        t[2] = max(t[2], (e - s) / 1e3)
    print("\nAPI by total host us (count, total, max):")
    for n, (k, s, m) in sorted(tot.items(), key=lambda x: -x[1][1])[:25]:
        print(f"{s:12.1f} {k:8d} {m:10.1f}  {n}")
    marks = [k for k in ks if a.marker in k[0]]
    if len(marks) < a.steps + 1:
        return
    t0, t1 = marks[-a.steps - 1][1], marks[-1][1]
    print(f"\nlong calls ({a.min_us} us+) over the last {a.steps} steps ({(t1 - t0) / 1e3 / a.steps:.1f} us/step):")
    for n, s, e in regs:
        if s < t0 or s > t1 or (e - s) / 1e3 < a.min_us:
            continue
        running = [k[0].split("(")[0][-40:] for k in ks if k[1] <= e <= k[2]]
        print(f"{(s - t0) / 1e3:10.1f} us  {(e - s) / 1e3:8.1f} us  {n[:40]:40s}  gpu at return: {running[:1]}")


if __name__ == "__main__":
    main()
