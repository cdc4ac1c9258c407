#!/usr/bin/env python3
"""129..256-row decode GEMMs on the Llama-2-7B layer shapes (one MI355X): the two-dimensionally
tiled kernel (csrc/gemm_t2d.h) against hipBLASLt and the ring kernels, each with the epilogue the
fused-norm decode path runs (qkv / gate-up: row-scaled consumer; o / down: the residual-stream
producer).  hipBLASLt is timed bare (no norm / SwiGLU / residual kernels), i.e. favourably.

Weights rotate over a 1 GiB pool (a decode step never finds them in the 256 MB Infinity Cache).
One JSON line per (M, shape, kernel): us and weight-stream TB/s.

    python scripts/t2d_bench.py [--m 256 192] [--iters 30] [--splits 0 1 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from src import ops  # noqa: E402

SHAPES = [("qkv", 12288, 4096, 0), ("o", 4096, 4096, 3), ("gate_up", 22016, 4096, 1), ("down", 4096, 11008, 3)]


def timed(fn, iters):
    for i in range(3):
        fn(i)
    best = float("inf")
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(iters):
            fn(i)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1000)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[256, 192])
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--splits", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--shapes", nargs="+", default=[s[0] for s in SHAPES])
    ap.add_argument("--ring", action="store_true", help="also time the 12 / 16-row-tile ring kernels")
    ap.add_argument("--gl", action="store_true", help="also time the LDS-DMA staging form")
    a = ap.parse_args()
    dev = torch.device("cuda")
    ws_buf = ops.gemm_workspace(dev)
    print(json.dumps({"tuned_hipblaslt_table": ops.use_tuned_gemms()}), flush=True)
    pool = (torch.randn((1 << 30) // 2, device=dev) * 0.02).to(torch.bfloat16)
    ss = ops.norm_stats_buffer(dev, 3)
    for M in a.m:
        for name, N, K, epi in SHAPES:
            if name not in a.shapes:
                continue
            n = N * K
            nw = min(16, pool.numel() // n)
            wrm = [pool[i * n:(i + 1) * n].view(N, K) for i in range(nw)]
            wps = [pool[i * n:(i + 1) * n].view(N // 16, K // 32, 64, 8) for i in range(nw)]
            xa = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
            us = timed(lambda i: torch.nn.functional.linear(xa, wrm[i % nw]), a.iters)
            print(json.dumps({"M": M, "shape": name, "kernel": "hipblaslt", "us": round(us, 2),
                              "TBps": round(n * 2 / us / 1e6, 2)}), flush=True)
            xp = ops.pack_act(xa)
            ncols = N // 2 if epi == 1 else N
            res = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            apo = torch.zeros(ops.packed_numel(M, N), dtype=torch.bfloat16, device=dev)
            out = (torch.empty(ops.packed_numel(M, ncols), dtype=torch.bfloat16, device=dev) if epi == 1
                   else (res if epi == 3 else torch.empty(M, ncols, dtype=torch.bfloat16, device=dev)))
            ss_in = ss[2] if epi in (0, 1) else None
            flags0 = 1 | (2 if epi == 1 else 0)
            cands = [("t2d" + (f"/S{s}" if s else ""), flags0 | 32768 | (s << 16)) for s in a.splits]
            if a.gl:
                cands += [("t2d-gl" + (f"/S{s}" if s else ""), flags0 | 32768 | 262144 | (s << 16)) for s in a.splits]
            if a.ring:
                ring = 256 if (epi != 1 and N % 2048 == 0) else 128
                cands.append(("ring", flags0 | ring))
            for kname, flags in cands:
                def run(i, flags=flags):
                    torch.ops.mpamd.gemm(xp, wps[i % nw], out, res if epi == 3 else None, epi, M, flags, ws_buf, None,
                                         apo if epi == 3 else None, ss[0] if epi == 3 else None,
                                         ss[1] if epi == 3 else None, ss_in, 1.0 / K, 1e-5)
                try:
                    us = timed(run, a.iters)
                except RuntimeError as e:  # shape / split not covered
                    print(json.dumps({"M": M, "shape": name, "kernel": kname, "error": str(e)[:120]}), flush=True)
                    continue
                print(json.dumps({"M": M, "shape": name, "kernel": kname, "us": round(us, 2),
                                  "TBps": round(n * 2 / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
