#!/usr/bin/env python3
"""Load-balanced swarm on ONE host (reference scripts/elice_test_load_balancing.sh: 4 servers
all started as ``--stage 1 --use_load_balancing --num_blocks 8 --total_blocks 32`` plus a
client).  Each server picks its own span with ``choose_best_blocks``; the script prints the
spans they selected ("Selected blocks" log lines) and runs one client generation over
module routing.

    python scripts/lb_swarm.py --model tiny-llama --servers 3 --num_blocks 2 --splits 1
    python scripts/lb_swarm.py --model llama3-8b --servers 4 --num_blocks 8 --splits 8 --gpus
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from run_all import MADDR_RE, READY_RE, wait_log  # noqa: E402

SEL_RE = re.compile(r"Selected blocks \[(\d+), (\d+)\)")
ANN_RE = re.compile(r"Announced blocks \[(\d+), (\d+)\)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="tiny-llama")
    ap.add_argument("--splits", default="1", help="first cut = the client's span end (min_block)")
    ap.add_argument("--servers", type=int, default=3)
    ap.add_argument("--num_blocks", type=int, default=2)
    ap.add_argument("--base_port", type=int, default=29900)
    ap.add_argument("--max_new_tokens", type=int, default=8)
    ap.add_argument("--gpus", action="store_true")
    ap.add_argument("--log_dir", default=os.path.join(ROOT, "gpurun_out", "lb_swarm"))
    a = ap.parse_args()
    os.makedirs(a.log_dir, exist_ok=True)
    procs, first = [], None
    try:
        for k in range(a.servers):
            dev = f"cuda:{k}" if a.gpus else "cpu"
            cmd = [sys.executable, "-m", "src.main", "--model", a.model, "--splits", a.splits, "--stage", "1",
                   "--use_load_balancing", "--num_blocks", str(a.num_blocks), "--host", "127.0.0.1",
                   "--dht_port", str(a.base_port + 2 * k), "--rpc_port", str(a.base_port + 2 * k + 1),
                   "--device", dev, "--mean_balance_check_period", "1000"]
            if first:
                cmd += ["--dht_initial_peers", first]
            log = os.path.join(a.log_dir, f"server{k}.log")
            procs.append(subprocess.Popen(cmd, cwd=ROOT, stdout=open(log, "w"), stderr=subprocess.STDOUT))
            m = wait_log(log, MADDR_RE, 300, procs[-1])
            first = first or m.group(1)
            wait_log(log, READY_RE, 600, procs[-1])
            sel = wait_log(log, SEL_RE, 60, procs[-1])
            print(f"server {k}: Selected blocks [{sel.group(1)}, {sel.group(2)})", flush=True)
            # the next server chooses only once this one's span (with its measured throughput)
            # is in the registry: a fixed sleep raced the throughput probe on a loaded host
            wait_log(log, ANN_RE, 300, procs[-1])
            time.sleep(0.5)
        cmd = [sys.executable, "-m", "src.main", "--model", a.model, "--splits", a.splits, "--stage", "0",
               "--use_load_balancing", "--dht_initial_peers", first, "--max_new_tokens", str(a.max_new_tokens),
               "--temperature", "0", "--device", "cuda:0" if a.gpus else "cpu"]
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900)
        print(r.stdout[-2500:] + r.stderr[-2500:])
        return r.returncode
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()


if __name__ == "__main__":
    sys.exit(main())
