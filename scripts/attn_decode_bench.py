#!/usr/bin/env python3
"""Decode attention alone (one new token per session, paged KV), HIP-event timed: the
flash-decoding kernel with RoPE + KV write folded in (the executor's MHA decode launch) and
the MFMA GQA kernel, at the bench's batch / context sizes.  Reports achieved KV bandwidth.

    python scripts/attn_decode_bench.py --batch 1 64 256 --ctx 170 1024 --heads 32/32 32/8
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src import ops  # noqa: E402


def timeit(fn, iters=20, rounds=3):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 64, 256])
    ap.add_argument("--ctx", type=int, nargs="+", default=[170, 1024])
    ap.add_argument("--heads", nargs="+", default=["32/32", "32/8"])
    a = ap.parse_args()
    dev, D, ps = "cuda", 128, 64
    for hs in a.heads:
        nh, nkv = (int(x) for x in hs.split("/"))
        for B in a.batch:
            for ctx in a.ctx:
                npg = math.ceil(ctx / ps)
                kc = (torch.randn(B * npg + 1, nkv, ps, D, device=dev) * 0.5).to(torch.bfloat16)
                vc = torch.randn_like(kc)
                bt = torch.randperm(B * npg, device=dev).to(torch.int32).view(B, npg)
                q = (torch.randn(B, (nh + 2 * nkv) * D, device=dev) * 0.5).to(torch.bfloat16)
                q_seq = torch.arange(B, dtype=torch.int32, device=dev)
                q_ctx = torch.full((B,), ctx, dtype=torch.int32, device=dev)
                pos = (q_ctx - 1).long()
                slots = (bt[:, (ctx - 1) // ps].long() * ps + (ctx - 1) % ps)
                cos, sin = ops.rope_cos_sin(D, 4096, 10000.0, dev)
                scale = 1 / math.sqrt(D)
                nrep = nh // nkv
                part = ops.attention_partition(B, nkv, ctx, min_part=256 if nrep >= 4 else 64)
                out = torch.empty(B, nh * D, dtype=torch.bfloat16, device=dev)
                ws = ops.attention_workspace(B, nh, D, part[1], dev)
                if nrep >= 4:
                    qb = torch.from_numpy(__import__("numpy").stack([__import__("numpy").arange(B),
                                                                     __import__("numpy").ones(B)]).astype("int32")).to(dev)
                    ps2 = 128 * math.ceil(part[0] / 128)
                    np2 = max(1, math.ceil(part[0] * part[1] / ps2))
                    fn = lambda: ops.attention_mfma_rope(q, kc, vc, bt, q_seq, q_ctx, qb, pos, cos, sin, slots,  # noqa
                                                         nh, nkv, scale, out=out, workspace=ws, part_size=ps2,
                                                         num_parts=np2)
                    kind = "mfma_gqa_rope"
                else:
                    fn = lambda: ops.paged_attention_rope(q, kc, vc, bt, q_seq, q_ctx, pos, cos, sin, slots, nh,  # noqa
                                                          nkv, scale, out=out, workspace=ws, part_size=part[0],
                                                          num_parts=part[1])
                    kind = "flash_decode_rope"
                us = timeit(fn)
                kv = B * ctx * nkv * D * 2 * 2
                print(json.dumps({"heads": hs, "batch": B, "ctx": ctx, "kernel": kind, "part": list(part),
                                  "us": round(us, 2), "kv_MB": round(kv / 1e6, 1),
                                  "TBps": round(kv / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
