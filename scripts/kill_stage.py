#!/usr/bin/env python3
"""Fault injection: terminate the stage server(s) serving ``--stage N`` (reference scripts/kill_stage.py).

Unlike the reference (``ps aux`` grep + interactive confirm), the process is matched on
its exact argv (``src.main`` with ``--stage N``), only processes owned by the current user
are considered, and ``--dry_run`` lists them without sending anything.
"""
from __future__ import annotations

import argparse
import os
import signal
import sys


def find_stage_pids(stage: int):
    me = os.getuid()
    out = []
    for pid in os.listdir("/proc"):
        if not pid.isdigit() or int(pid) == os.getpid():
            continue
        try:
            if os.stat(f"/proc/{pid}").st_uid != me:
                continue
            argv = open(f"/proc/{pid}/cmdline", "rb").read().split(b"\0")
        except OSError:
            continue
        args = [x.decode(errors="replace") for x in argv if x]
        if "src.main" not in args:
            continue
        if "--stage" in args and args.index("--stage") + 1 < len(args) and args[args.index("--stage") + 1] == str(stage):
            out.append((int(pid), " ".join(args)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stage", type=int)
    ap.add_argument("--signal", default="TERM", choices=["TERM", "KILL", "INT"])
    ap.add_argument("--dry_run", action="store_true")
    a = ap.parse_args()
    pids = find_stage_pids(a.stage)
    if not pids:
        print(f"no stage {a.stage} server found")
        return 1
    for pid, cmd in pids:
        print(f"{'would send' if a.dry_run else 'sending'} SIG{a.signal} to {pid}: {cmd}")
        if not a.dry_run:
            os.kill(pid, getattr(signal, f"SIG{a.signal}"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
