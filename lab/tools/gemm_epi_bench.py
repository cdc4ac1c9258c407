#!/usr/bin/env python3
"""Decode-GEMM kernel x epilogue matrix on the Llama-2-7B layer shapes (one MI355X).

Every applicable kernel family (pk / sk / lds*) is timed for the plain epilogues and for the
fused-norm ones (consumer row scale ``ss_in``, producer epilogue 3), with weights rotated over a
1 GiB pool like the autotuner (the 256 MB Infinity Cache never serves a decode step's weights).
Prints one JSON line per (shape, epilogue, kernel): us and weight-stream TB/s.

    python scripts/gemm_epi_bench.py [--m 64] [--iters 30]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from src import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[64])
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda")
    ops.gemm_workspace(dev)
    pool = (torch.randn((1 << 30) // 2, device=dev) * 0.02).to(torch.bfloat16)
    shapes = [("qkv", 12288, 4096, 0, False), ("qkv+rs", 12288, 4096, 0, True), ("o", 4096, 4096, 0, False),
              ("o+res3", 4096, 4096, 3, False), ("gate_up", 22016, 4096, 1, False),
              ("gate_up+rs", 22016, 4096, 1, True), ("down", 4096, 11008, 0, False),
              ("down+res3", 4096, 11008, 3, False), ("o+res3-noatomic", 4096, 4096, 3, None),
              ("down+res3-noatomic", 4096, 11008, 3, None)]
    for M in a.m:
        # library baseline: hipBLASLt through torch (row-major bf16 weight, same rotation)
        for name, N, K in (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008)):
            ws = [pool[i * N * K:(i + 1) * N * K].view(N, K) for i in range(min(16, pool.numel() // (N * K)))]
            xa = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
            for i in range(3):
                torch.nn.functional.linear(xa, ws[i % len(ws)])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.iters):
                torch.nn.functional.linear(xa, ws[i % len(ws)])
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1000
            print(json.dumps({"M": M, "shape": name, "N": N, "K": K, "kernel": "hipblaslt", "us": round(us, 2),
                              "TBps": round(N * K * 2 / us / 1e6, 2)}), flush=True)
        ss = ops.norm_stats_buffer(dev, 3)
        for name, N, K, epi, rs in shapes:
            n = N * K
            wps = [pool[i * n:(i + 1) * n].view(N // 16, K // 32, 64, 8) for i in range(min(16, pool.numel() // n))]
            xp = ops.pack_act((torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16))
            ncols = N // 2 if epi == 1 else N
            res = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            apo = torch.zeros(ops.packed_numel(M, N), dtype=torch.bfloat16, device=dev)
            out = (torch.empty(ops.packed_numel(M, ncols), dtype=torch.bfloat16, device=dev) if epi == 1
                   else (res if epi == 3 else torch.empty(M, ncols, dtype=torch.bfloat16, device=dev)))
            kw = dict(out=out, epilogue=epi, a_rows=M, out_packed=epi == 1)
            if epi == 3:
                kw.update(residual=res, ap_out=apo, ss_out=ss[0] if rs is not None else None, ss_zero=ss[1])
            if rs:
                kw.update(ss_in=ss[2], eps=1e-5)
            for kern in ops._KERNEL_FLAGS:
                if not ops._covered(kern, M, N, K, epi):
                    continue
                ops.set_gemm_sk(kern)
                try:
                    for i in range(3):
                        ops.linear(xp, None, wp=wps[i % len(wps)], **kw)
                    best = float("inf")
                    for _ in range(3):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for i in range(a.iters):
                            ops.linear(xp, None, wp=wps[i % len(wps)], **kw)
                        e1.record()
                        e1.synchronize()
                        best = min(best, e0.elapsed_time(e1) / a.iters)
                finally:
                    ops.set_gemm_sk("auto")
                us = best * 1000
                print(json.dumps({"M": M, "shape": name, "N": N, "K": K, "epi": epi, "row_scale": rs, "kernel": kern,
                                  "us": round(us, 2), "TBps": round(N * K * 2 / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
