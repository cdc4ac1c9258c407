#!/usr/bin/env python3
"""Launch a whole swarm on ONE host: stage servers 1..N (in order), then the stage-0 client.

Reference: scripts/run_all.py (stages on ports base+0/+2/+4/+6, DHT multiaddr scraped from
stage 1's log, readiness from the "handlers registered" log line, logs to stage{N}.log).
Same procedure here, generalised to any number of cut points; the defaults actually work
(the reference defaults to ``--model gpt2 --splits 10,20,30``, which its own loader
rejects).  Each stage is its own OS process; on a multi-GPU host stage k uses GPU k-1
(``--gpus``), otherwise CPU.

    python scripts/run_all.py --model gpt2 --splits 6 --max_new_tokens 16
    python scripts/run_all.py --model llama2-7b --splits 8,16,24 --gpus
    # one GPU, 4 stage processes sharing it, 8 concurrent sessions, TCP path vs device channel:
    python scripts/run_all.py --model llama2-7b --splits 8,16,24 --gpus --extra "--kv_cache_gb 8" \
        --client_extra "--num_sessions 8 --device_channel off"
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MADDR_RE = re.compile(r"DHT visible multiaddrs: \['([^']+)'")
READY_RE = re.compile(r"handlers registered")


def wait_log(path: str, pattern: re.Pattern, timeout: float, proc: subprocess.Popen):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise RuntimeError(f"{path}: process exited with {proc.returncode}")
        if os.path.exists(path):
            with open(path, errors="replace") as f:
                m = pattern.search(f.read())
            if m:
                return m
        time.sleep(0.2)
    raise TimeoutError(f"{path}: no match for {pattern.pattern!r} within {timeout}s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--splits", default="6")
    ap.add_argument("--base_port", type=int, default=29800)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--max_new_tokens", type=int, default=16)
    ap.add_argument("--prompt", default="Hello, how are you?")
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--gpus", action="store_true",
                    help="stage k on cuda:(k-1) mod #GPUs, client on cuda:N mod #GPUs (one GPU: all share cuda:0)")
    ap.add_argument("--client_extra", default="", help="extra args for the stage-0 client only")
    ap.add_argument("--log_dir", default=os.path.join(ROOT, "gpurun_out", "run_all"))
    ap.add_argument("--extra", default="", help="extra args for every stage")
    a = ap.parse_args()
    os.makedirs(a.log_dir, exist_ok=True)
    sys.path.insert(0, ROOT)
    from src.models.config import resolve_model
    from src.partition import parse_splits

    n_servers = len(parse_splits(a.splits, resolve_model(a.model).num_hidden_layers))
    n_gpu = 1
    if a.gpus:
        import torch

        n_gpu = max(1, torch.cuda.device_count())  # does not initialise the GPU in this process
    procs = []
    first_maddr = None
    env = dict(os.environ)
    try:
        for k in range(1, n_servers + 1):
            dev = f"cuda:{(k - 1) % n_gpu}" if a.gpus else "cpu"
            cmd = [sys.executable, "-m", "src.main", "--model", a.model, "--splits", a.splits, "--stage", str(k),
                   "--host", a.host, "--dht_port", str(a.base_port + 2 * k), "--rpc_port", str(a.base_port + 2 * k + 1),
                   "--device", dev] + a.extra.split()
            if first_maddr:
                cmd += ["--dht_initial_peers", first_maddr]
            log = os.path.join(a.log_dir, f"stage{k}.log")
            procs.append(subprocess.Popen(cmd, cwd=ROOT, stdout=open(log, "w"), stderr=subprocess.STDOUT, env=env))
            m = wait_log(log, MADDR_RE, 300, procs[-1])
            if first_maddr is None:
                first_maddr = m.group(1)
            wait_log(log, READY_RE, 600, procs[-1])
            print(f"stage {k} ready ({log})", flush=True)
        dev = f"cuda:{n_servers % n_gpu}" if a.gpus else "cpu"
        cmd = [sys.executable, "-m", "src.main", "--model", a.model, "--splits", a.splits, "--stage", "0",
               "--dht_initial_peers", first_maddr, "--max_new_tokens", str(a.max_new_tokens), "--prompt", a.prompt,
               "--temperature", str(a.temperature), "--device", dev] + a.extra.split() + a.client_extra.split()
        log = os.path.join(a.log_dir, "stage0.log")
        with open(log, "w") as f:
            rc = subprocess.call(cmd, cwd=ROOT, stdout=f, stderr=subprocess.STDOUT, env=env)
        print(open(log).read()[-3000:])
        return rc
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
