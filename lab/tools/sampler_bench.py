#!/usr/bin/env python3
"""The decode sampler alone (csrc/sampling.hip), HIP-event timed inside a captured hipGraph (so
launch gaps are excluded), at the bench's 64 rows x 32000 vocab, split by what it does:

  greedy       temperature 0: fp32 copy of the row + argmax only
  topk         top-k 50 / top-p 0.92, no repetition penalty
  full         + repetition penalty 1.5 over a history of ``--hist`` generated ids
  full_update  + the in-kernel history append (the serving loop's form)

    python scripts/sampler_bench.py --rows 64 --vocab 32000 --hist 10 50
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from src import ops  # noqa: E402


def timed(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        fn()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[64])
    ap.add_argument("--vocab", type=int, nargs="+", default=[32000])
    ap.add_argument("--hist", type=int, nargs="+", default=[10, 50])
    a = ap.parse_args()
    dev = "cuda"
    for R in a.rows:
        for V in a.vocab:
            logits = (torch.randn(R, V, device=dev) * 3).to(torch.bfloat16)
            ws = torch.empty(R * V, dtype=torch.float32, device=dev)
            out = torch.empty(R, dtype=torch.long, device=dev)
            seeds = torch.arange(R, dtype=torch.long, device=dev)
            for H in a.hist:
                cap = 50
                recent = torch.randint(0, V, (R, cap), dtype=torch.int32, device=dev)
                rlen0 = torch.full((R,), H, dtype=torch.int32, device=dev)
                rlen = rlen0.clone()
                cases = {
                    "greedy": (0.0, 0.92, 50, 1.0, False),
                    "topk": (1.0, 0.92, 50, 1.0, False),
                    "full": (1.0, 0.92, 50, 1.5, False),
                    "full_update": (1.0, 0.92, 50, 1.5, True),
                }
                for name, (t, p, k, rp, upd) in cases.items():
                    temps = torch.full((R,), t, device=dev)
                    tps = torch.full((R,), p, device=dev)
                    tks = torch.full((R,), k, dtype=torch.int32, device=dev)
                    rps = torch.full((R,), rp, device=dev)

                    def fn():
                        if upd:  # keep the history length fixed across replays
                            rlen.copy_(rlen0)
                        ops.sample(logits, temps, tps, tks, rps, recent, rlen, seeds, workspace=ws, out=out,
                                   update_history=upd)

                    us = timed(fn)
                    print(json.dumps({"rows": R, "vocab": V, "hist": H, "case": name, "us": round(us, 2)}),
                          flush=True)


if __name__ == "__main__":
    main()
