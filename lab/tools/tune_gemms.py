#!/usr/bin/env python3
"""Regenerate ops/tuned/gemm_gfx950.csv: the hipBLASLt / rocBLAS solution per row-major GEMM
shape (prefill steps and decode steps above 128 rows, which the hand-written decode kernels do
not take), chosen by PyTorch TunableOp on this GPU.

Runs the workloads whose shapes matter as child processes with tuning on (each writes its own
TunableOp file), then merges every tuned row into the shipped table (later runs win on equal
shapes).  Run on a MI355X box:

    python scripts/tune_gemms.py [--model llama2-7b] [--out .../ops/tuned/gemm_gfx950.csv]

The executor loads the table read-only (ops.use_tuned_gemms): shapes missing from it keep the
library heuristic.  Measured effect (profiles/r3_g): 256 sessions 9.92 -> 9.62 ms/step, 8K-token
prefill 101.5 -> 100.0 ms.
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_OUT = os.path.join(ROOT, "global_capstone_design_distributed-inference-of-llms-over-the-internet_amd", "ops",
                           "tuned", "gemm_gfx950.csv")


def workloads(model: str):
    # decode above 128 rows runs at the hipGraph batch buckets (192, 256); prefill shapes of the
    # bench (256 x 128 tokens) and of single long prompts
    yield [sys.executable, "bench.py", "--model", model, "--batch", "256", "--steps", "2", "--warmup", "1"]
    yield [sys.executable, "bench.py", "--model", model, "--batch", "192", "--steps", "2", "--warmup", "1"]
    for n in (512, 2048, 8192):
        yield [sys.executable, "scripts/prefill_bench.py", "--model", model, "--prompt-len", str(n), "--repeats", "1"]


def merge(files, out):
    validators, rows = {}, {}
    for f in files:
        with open(f) as fh:
            for line in fh:
                parts = line.strip().split(",")
                if len(parts) < 3:
                    continue
                if parts[0] == "Validator":
                    validators[parts[1]] = line.strip()
                else:
                    rows[(parts[0], parts[1])] = line.strip()
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as fh:
        for v in validators.values():
            fh.write(v + "\n")
        for k in sorted(rows):
            fh.write(rows[k] + "\n")
    return len(rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--out", default=DEFAULT_OUT)
    ap.add_argument("--max-tuning-ms", type=int, default=20)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="mpamd_tune_")
    files = [a.out] if os.path.exists(a.out) else []
    for i, cmd in enumerate(workloads(a.model)):
        f = os.path.join(tmp, f"run{i}.csv")
        env = dict(os.environ, PYTORCH_TUNABLEOP_ENABLED="1", PYTORCH_TUNABLEOP_TUNING="1",
                   PYTORCH_TUNABLEOP_FILENAME=f, PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=str(a.max_tuning_ms),
                   MPAMD_TUNED_GEMMS="0")
        print("tuning:", " ".join(cmd[1:]), flush=True)
        r = subprocess.run(cmd, cwd=ROOT, env=env)
        if r.returncode != 0:
            raise SystemExit(f"workload failed ({r.returncode}): {' '.join(cmd)}")
        files += sorted(glob.glob(os.path.join(tmp, f"run{i}*.csv")))
    n = merge(files, a.out)
    print(f"{n} tuned shapes -> {a.out}")


if __name__ == "__main__":
    main()
