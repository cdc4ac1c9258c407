#!/usr/bin/env python3
"""Prefill attention kernels alone (causal, paged KV, Llama shapes): the FA2 kernel
(csrc/attention_fa.hip, 4 / 8 waves) vs the 16x16 grouped kernel (csrc/attention_mfma.hip),
HIP-event timed, TFLOP/s over the causal FLOPs (4 * heads * D * sum over rows of ctx).

    python scripts/attn_bench.py --seqs 1x2048 1x8192 8x2048 --heads 32/32 32/8
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


def timeit(fn, iters=10, rounds=3):
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
    ap.add_argument("--seqs", nargs="+", default=["1x2048", "1x8192", "8x2048", "64x128"])
    ap.add_argument("--heads", nargs="+", default=["32/32", "32/8"])
    ap.add_argument("--kernels", nargs="+", default=["grp", "fa4", "fa8"])
    a = ap.parse_args()
    dev = "cuda"
    D, ps = 128, 64
    for hs in a.heads:
        nh, nkv = (int(x) for x in hs.split("/"))
        for sq in a.seqs:
            B, L = (int(x) for x in sq.split("x"))
            npg = math.ceil(L / ps)
            kc = (torch.randn(B * npg + 2, nkv, ps, D, device=dev) * 0.5).to(torch.bfloat16)
            vc = torch.randn_like(kc)
            bt = torch.arange(B * npg, dtype=torch.int32, device=dev).view(B, npg)
            T = B * L
            q = (torch.randn(T, (nh + 2 * nkv) * D, device=dev) * 0.5).to(torch.bfloat16)
            ntoks = [L] * B
            q_seq = torch.arange(B, dtype=torch.int32, device=dev).repeat_interleave(L)
            q_ctx = torch.arange(1, L + 1, dtype=torch.int32, device=dev).repeat(B)
            flops = 4.0 * nh * D * B * L * (L + 1) / 2
            scale = 1 / math.sqrt(D)
            out = torch.empty(T, nh * D, dtype=torch.bfloat16, device=dev)
            res = {}
            ref_out = None
            for k in a.kernels:
                if k == "grp":
                    qb = torch.from_numpy(ops.query_blocks(ntoks, nh // nkv)).to(dev)
                    sb = torch.from_numpy(ops.query_superblocks(ntoks, nh // nkv)).to(dev)
                    fn = lambda: ops.attention_mfma(q, kc, vc, bt, q_seq, q_ctx, qb, nh, nkv, scale, out=out,  # noqa
                                                    max_ctx=L, superblocks=sb)
                else:  # fa<waves>[:p<parts>][:z|:n] (parts: explicit context split; z / n: causal block
                    #       pairing forced on / off, default the library's rule)
                    name, *opts = k.split(":")
                    w = int(name[2:])
                    nparts = next((int(o[1:]) for o in opts if o.startswith("p")), None)
                    pair = True if "z" in opts else (False if "n" in opts else None)
                    fb = torch.from_numpy(ops.fa_blocks(ntoks, nh // nkv, w)).to(dev)
                    fn = lambda: ops.attention_fa(q, kc, vc, bt, q_seq, q_ctx, fb, nh, nkv, scale, out=out,  # noqa
                                                  max_ctx=L, waves=w, num_parts=nparts, pair=pair)
                us = timeit(fn)
                o = out.float().clone()
                if ref_out is None:
                    ref_out = o
                err = float((o - ref_out).abs().max())
                res[k] = dict(us=round(us, 1), tflops=round(flops / us / 1e6, 1), maxdiff=round(err, 4))
            print(json.dumps({"heads": hs, "seqs": sq, **res}), flush=True)


if __name__ == "__main__":
    main()
