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

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from src import ops  # noqa: E402

COLD = False


_FLUSH = None


def timeit_cold(fn, iters=10):
    """Each call after a 1 GiB write (evicts L2 and the 256 MB Infinity Cache), timed alone:
    the KV stream comes from HBM as in a decode step, where the layer's weights run between
    two reads of its KV."""
    global _FLUSH
    if _FLUSH is None:
        _FLUSH = torch.ones(1 << 29, dtype=torch.int16, device="cuda")
    fn()
    ts = []
    for i in range(iters):
        # a 1 GiB READ (a write would leave ~256 MB of dirty lines to be written back during
        # the timed kernel): the decode step's weight stream leaves clean lines behind too
        _FLUSH.sum(dtype=torch.int32)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2] * 1000.0


def timeit(fn, iters=20, rounds=3):
    if COLD:
        return timeit_cold(fn)
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
    ap.add_argument("--cold", action="store_true", help="evict L2 / Infinity Cache before every timed call")
    ap.add_argument("--min-part", type=int, default=None, help="override the split-K slice floor")
    ap.add_argument("--kernel", default="auto", choices=["auto", "simt"],
                    help="simt: the flash-decoding (VALU) kernel for GQA too")
    a = ap.parse_args()
    global COLD
    COLD = a.cold
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
                mp_ = a.min_part or (256 if nrep >= 4 else 64)
                part = ops.attention_partition(B, nkv, ctx, min_part=mp_)
                out = torch.empty(B, nh * D, dtype=torch.bfloat16, device=dev)
                ws = ops.attention_workspace(B, nh, D, part[1], dev)
                if nrep >= 4 and a.kernel == "auto":
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
                if COLD:  # reference: a plain device copy of the same pages (read + write)
                    dst = torch.empty_like(kc)
                    cu = timeit(lambda: dst.copy_(kc))
                    print(json.dumps({"heads": hs, "batch": B, "ctx": ctx, "kernel": "copy_of_k_pages", "cold": True,
                                      "us": round(cu, 2), "TBps_rw": round(2 * kc.numel() * 2 / cu / 1e6, 2)}),
                          flush=True)
                print(json.dumps({"heads": hs, "batch": B, "ctx": ctx, "kernel": kind, "part": list(part), "cold": COLD,
                                  "us": round(us, 2), "kv_MB": round(kv / 1e6, 1),
                                  "TBps": round(kv / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
