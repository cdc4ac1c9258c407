#!/usr/bin/env python3
"""Per-kernel microbenchmarks on the decode shapes of Llama-2-7B (and 70B/8-stage shapes).

Times each HIP kernel with HIP events over many back-to-back launches (random data) and
reports achieved bandwidth; for GEMMs the native fragment-packed kernel is compared with
hipBLASLt (torch.nn.functional.linear) in the same process (interleaved rounds).
"""
from __future__ import annotations

import argparse
import json
import math

import torch
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from src import ops


def timeit(fn, iters=50, rounds=3):
    for _ in range(3):
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
    return best * 1000.0  # us


def gemm_rows(Ms, shapes):
    out = []
    for (name, N, K, epi) in shapes:
        w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        wp = ops.pack_weight(w)
        for M in Ms:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            xp = ops.pack_act(x)  # decode path: activations arrive packed from their producer
            y = torch.empty(M, N // 2 if epi == 1 else N, device="cuda", dtype=torch.bfloat16)
            ops.set_gemm_sk("off")
            t_nat = timeit(lambda: ops.linear(xp, None, out=y, epilogue=epi, wp=wp, a_rows=M))
            ops.set_gemm_sk("on")
            t_sk = timeit(lambda: ops.linear(xp, None, out=y, epilogue=epi, wp=wp, a_rows=M))
            ops.set_gemm_sk("off")
            t_lib = timeit(lambda: ops.linear(x, w, out=y, epilogue=epi, policy="hipblaslt"))
            byts = N * K * 2
            out.append(dict(kernel="gemm", name=name, M=M, N=N, K=K, native_us=round(t_nat, 2),
                            streamk_us=round(t_sk, 2), hipblaslt_us=round(t_lib, 2),
                            native_TBps=round(byts / t_nat / 1e6, 2), streamk_TBps=round(byts / t_sk / 1e6, 2),
                            hipblaslt_TBps=round(byts / t_lib / 1e6, 2)))
            print(json.dumps(out[-1]), flush=True)
    return out


def attn_rows(cases):
    for (B, ctx, nh, nkv) in cases:
        D, ps = 128, 64
        pages_per = math.ceil((ctx + 1) / ps)
        P = B * pages_per
        kc = torch.randn(P, nkv, ps, D, device="cuda").to(torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.randperm(P, device="cuda").view(B, pages_per).to(torch.int32)
        q = torch.randn(B, (nh + 2 * nkv) * D, device="cuda").to(torch.bfloat16)
        q_seq = torch.arange(B, dtype=torch.int32, device="cuda")
        q_ctx = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        part = ops.attention_partition(B, nkv, ctx)
        out = torch.empty(B, nh * D, device="cuda", dtype=torch.bfloat16)
        ws = ops.attention_workspace(B, nh, D, part[1], "cuda")
        t = timeit(lambda: ops.paged_attention(q, kc, vc, bt, q_seq, q_ctx, nh, nkv, 0.088, out=out, workspace=ws,
                                               part_size=part[0], num_parts=part[1]))
        byts = B * ctx * nkv * D * 2 * 2
        qb = torch.from_numpy(ops.query_blocks([1] * B, nh // nkv)).cuda()
        wsm = ops.attention_workspace(B, nh, D, 16, "cuda")
        tm = timeit(lambda: ops.attention_mfma(q, kc, vc, bt, q_seq, q_ctx, qb, nh, nkv, 0.088, out=out, workspace=wsm,
                                               max_ctx=ctx))
        print(json.dumps(dict(kernel="paged_attention", B=B, ctx=ctx, nh=nh, nkv=nkv, part=part, us=round(t, 2),
                              TBps=round(byts / t / 1e6, 2), mfma_us=round(tm, 2),
                              mfma_TBps=round(byts / tm / 1e6, 2))), flush=True)
    # prefill: B sequences x L prompt tokens, causal, all queries at once
    for (B, L, nh, nkv) in [(64, 128, 32, 32), (4, 2048, 32, 32), (8, 1024, 64, 8)]:
        D, ps = 128, 64
        pages_per = math.ceil(L / ps)
        P = B * pages_per
        kc = torch.randn(P, nkv, ps, D, device="cuda").to(torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.randperm(P, device="cuda").view(B, pages_per).to(torch.int32)
        T = B * L
        q = torch.randn(T, (nh + 2 * nkv) * D, device="cuda").to(torch.bfloat16)
        q_seq = torch.arange(B, dtype=torch.int32, device="cuda").repeat_interleave(L)
        q_ctx = torch.arange(1, L + 1, dtype=torch.int32, device="cuda").repeat(B)
        out = torch.empty(T, nh * D, device="cuda", dtype=torch.bfloat16)
        qb = torch.from_numpy(ops.query_blocks([L] * B, nh // nkv)).cuda()
        t = timeit(lambda: ops.paged_attention(q, kc, vc, bt, q_seq, q_ctx, nh, nkv, 0.088, out=out, max_ctx=L),
                   iters=5)
        tm = timeit(lambda: ops.attention_mfma(q, kc, vc, bt, q_seq, q_ctx, qb, nh, nkv, 0.088, out=out, max_ctx=L),
                    iters=5)
        flops = 4 * B * nh * D * L * L / 2
        print(json.dumps(dict(kernel="prefill_attention", B=B, L=L, nh=nh, nkv=nkv, valu_us=round(t, 1),
                              mfma_us=round(tm, 1), mfma_TFLOPs=round(flops / tm / 1e6, 1))), flush=True)


def misc_rows(B=64):
    H, F, V = 4096, 11008, 32000
    x = torch.randn(B, H, device="cuda").to(torch.bfloat16)
    r = torch.randn_like(x)
    w = torch.ones(H, device="cuda", dtype=torch.bfloat16)
    y = torch.empty_like(x)
    t = timeit(lambda: ops.rmsnorm(x, w, 1e-5, out=y, residual=r, mode=1))
    print(json.dumps(dict(kernel="add_rmsnorm", B=B, us=round(t, 2))), flush=True)
    logits = torch.randn(B, V, device="cuda").to(torch.bfloat16)
    R = B
    kw = dict(top_ps=torch.full((R,), 0.92, device="cuda"), top_ks=torch.full((R,), 50, dtype=torch.int32, device="cuda"),
              rep_pens=torch.full((R,), 1.5, device="cuda"),
              recent=torch.randint(0, V, (R, 50), dtype=torch.int32, device="cuda"),
              recent_len=torch.full((R,), 50, dtype=torch.int32, device="cuda"),
              seeds=torch.arange(R, device="cuda"))
    temps = torch.ones(R, device="cuda")
    ws = torch.empty(R * V, device="cuda")
    outt = torch.empty(R, dtype=torch.long, device="cuda")
    t = timeit(lambda: ops.sample(logits, temps, workspace=ws, out=outt, **kw))
    print(json.dumps(dict(kernel="sample", R=R, V=V, us=round(t, 2))), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="gemm,attn,misc")
    a = ap.parse_args()
    assert ops.load_library()
    what = a.what.split(",")
    if "gemm" in what:
        shapes = [("qkv", 12288, 4096, 0), ("o", 4096, 4096, 0), ("gate_up+swiglu", 22016, 4096, 1),
                  ("down", 4096, 11008, 0), ("lm_head", 32000, 4096, 0)]
        gemm_rows([1, 16, 32, 64], shapes)
    if "attn" in what:
        attn_rows([(64, 256, 32, 32), (64, 1024, 32, 32), (1, 4096, 32, 32), (64, 1024, 64, 8), (8, 8192, 32, 8)])
    if "misc" in what:
        misc_rows()


if __name__ == "__main__":
    main()
