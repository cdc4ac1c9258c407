#!/usr/bin/env python3
"""Measured per-stage decode GPU time of a pipeline layout (validates ``partition.balanced_splits``).

Builds each stage of the layout in turn on ONE GPU (its blocks; the embedding on stage 0; final
norm + lm_head on the last), prefills ``--batch`` sessions of ``--prompt-len`` tokens, then times
``--steps`` decode steps of the stage (hipGraph replay, as serving runs them; the last stage also
runs the sampler at batch rows) with HIP events.  Prints one JSON line: cuts, per-stage ms,
measured max/mean, and the cost model's per-stage estimate and max/mean for comparison.

    python scripts/stage_balance.py --model llama2-7b --stages 8
    python scripts/stage_balance.py --model llama3-70b --fp8 --stages 8
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--stages", type=int, default=8)
    ap.add_argument("--splits", default="auto", help="auto (balanced_splits), even, or explicit cuts")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--fp8", action="store_true")
    a = ap.parse_args()

    from src import ops
    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.partition import balanced_splits, even_splits, parse_splits, stage_ranges, stage_times
    from src.runtime.executor import StageExecutor
    from src.runtime.sampler import RECENT

    dev = torch.device("cuda:0")
    cfg = resolve_model(a.model)
    L, S, B, P = cfg.num_hidden_layers, a.stages, a.batch, a.prompt_len
    ctx = P + a.steps // 2 + 1
    if a.splits == "auto":
        cuts = balanced_splits(cfg, S, batch=B, ctx=ctx, fp8=a.fp8)
    elif a.splits == "even":
        cuts = even_splits(L, S)
    else:
        cuts = parse_splits(a.splits, L)
    model_s = stage_times(cfg, cuts, batch=B, ctx=ctx, fp8=a.fp8)
    ms = []
    for st, (lo, hi) in enumerate(stage_ranges(cuts, L)):
        first, last = st == 0, st == S - 1
        w = random_stage_weights(cfg, lo, hi, has_embed=first, has_head=last, device=dev, dtype=torch.bfloat16,
                                 fp8=a.fp8)
        ex = StageExecutor(w.cfg, w, dev, max_sessions=B + 8, max_seq_len=256, graph_max_batch=B,
                           max_tokens_per_step=B * P, kv_cache_bytes=8 << 30)
        sids = [(f"s{i}", P) for i in range(B)]
        g = torch.Generator(device=dev).manual_seed(st)

        def inp(n):
            if first:
                return torch.randint(0, cfg.vocab_size, (n,), device=dev, generator=g)
            return (0.1 * torch.randn(n, cfg.hidden_size, device=dev, generator=g)).to(torch.bfloat16)

        with torch.inference_mode():
            ex.forward(sids, inp(B * P), reset=[True] * B)
            dec = [(s, 1) for s, _ in sids]
            n = B
            samp = None
            if last:
                V = cfg.vocab_size
                samp = dict(t=torch.ones(n, device=dev), p=torch.full((n,), 0.92, device=dev),
                            k=torch.full((n,), 50, dtype=torch.int32, device=dev), r=torch.full((n,), 1.5, device=dev),
                            h=torch.zeros(n, RECENT, dtype=torch.int32, device=dev),
                            hl=torch.zeros(n, dtype=torch.int32, device=dev),
                            sd=torch.arange(n, dtype=torch.int64, device=dev),
                            ws=torch.empty(max(n, 64) * V, dtype=torch.float32, device=dev))

            def step():
                out = ex.forward(dec, inp(n))
                if samp is not None:
                    ops.sample(out, samp["t"], samp["p"], samp["k"], samp["r"], samp["h"], samp["hl"], samp["sd"],
                               workspace=samp["ws"], update_history=True)

            for _ in range(3):
                step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                step()
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1) / a.steps)
        print(f"stage {st}: blocks [{lo}, {hi}) {ms[-1]:.3f} ms (model {1000 * model_s[st]:.3f})", file=sys.stderr,
              flush=True)
        del ex, w
        gc.collect()
        torch.cuda.empty_cache()
    mean = sum(ms) / len(ms)
    mmean = sum(model_s) / len(model_s)
    print(json.dumps({"model": a.model, "fp8": a.fp8, "stages": S, "batch": B, "ctx": ctx, "cuts": cuts,
                      "stage_ms": [round(v, 3) for v in ms], "max_over_mean": round(max(ms) / mean, 3),
                      "model_stage_ms": [round(1000 * v, 3) for v in model_s],
                      "model_max_over_mean": round(max(model_s) / mmean, 3)}), flush=True)


if __name__ == "__main__":
    main()
