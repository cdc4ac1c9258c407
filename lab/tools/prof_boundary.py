#!/usr/bin/env python3
"""The kernels around the last step boundaries of a rocprofv3 (rocpd SQLite) trace: name, start
relative to the marker, duration, gap before - to see what sits between two decode graph replays."""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="sample_kernel")
    ap.add_argument("--before", type=int, default=6)
    ap.add_argument("--after", type=int, default=8)
    ap.add_argument("--n", type=int, default=2)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    for m in marks[-a.n - 1:-1]:
        t0 = rows[m][1]
        print(f"--- boundary at {m}")
        for i in range(max(0, m - a.before), min(len(rows), m + a.after)):
            gap = (rows[i][1] - rows[i - 1][2]) / 1e3 if i else 0.0
            print(f"{(rows[i][1] - t0) / 1e3:9.1f} us  dur {(rows[i][2] - rows[i][1]) / 1e3:7.1f}  gap {gap:7.1f}  "
                  f"{re.sub(r'^void ', '', rows[i][0].split('(')[0])[:60]}")


if __name__ == "__main__":
    main()
