#!/usr/bin/env python3
"""End-to-end A/B of decode-kernel table entries: the whole graph-replayed decode step of a
full-depth stage (random-init weights), one kernel choice changed per variant.

The autotuner times each GEMM alone, back to back; inside the decode step the same kernel sits
between other launches (its ramp / tail, the split-K reduce launch, caches left by its neighbours),
so the isolated winner is not always the step's winner.  Every window re-prefills the sessions
(same prompts), captures, warms, then times ``--steps`` decode steps; windows of all variants are
interleaved over ``--rounds`` rounds and each variant keeps its mean.

    python lab/tools/table_ab.py --batch 64 --var base --var "M64:N4096xK4096e3=rwr"
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from src import ops  # noqa: E402
from src.models.config import resolve_model  # noqa: E402
from src.models.weights import random_stage_weights  # noqa: E402
from src.runtime.executor import StageExecutor  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--var", action="append", default=[],
                    help="'base' or 'KEY=KERNEL[,KEY=KERNEL...]' (KEY as in the table, e.g. M64:N4096xK4096e3; "
                         "'fold=0/1' sets the bucket's qkv fold)")
    a = ap.parse_args()
    cfg = resolve_model(a.model)
    B = a.batch
    dev = a.device
    w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device=dev, seed=0,
                             fp8=a.fp8)
    ex = StageExecutor(cfg, w, dev, max_sessions=B + 8, max_seq_len=a.prompt + a.steps + 16,
                       kv_cache_bytes=16 << 30, graph_max_batch=B, max_tokens_per_step=B * a.prompt, warmup=False)
    ex.warmup_serving(B, a.prompt)
    base_gemm, base_w8 = dict(ops._SK_CHOICE), dict(ops._W8_CHOICE)
    Bb = ex._bucket(B)
    base_fold = ex.qkv_fold_by_bucket.get(Bb, False)
    g = torch.Generator(device=dev).manual_seed(7)
    prompts = torch.randint(0, cfg.vocab_size, (B * a.prompt,), device=dev, generator=g)
    toks = torch.randint(0, cfg.vocab_size, (a.steps + 4, B), device=dev, generator=g)
    variants = a.var or ["base"]

    def apply(v):
        ops._SK_CHOICE.clear()
        ops._SK_CHOICE.update(base_gemm)
        ops._W8_CHOICE.clear()
        ops._W8_CHOICE.update(base_w8)
        ex.qkv_fold_by_bucket[Bb] = base_fold
        if v != "base":
            for item in v.split(","):
                k, kern = item.split("=")
                if k == "fold":
                    ex.qkv_fold_by_bucket[Bb] = kern == "1"
                    continue
                key = ops._parse_key(k)
                (ops._W8_CHOICE if a.fp8 else ops._SK_CHOICE)[key] = kern
        ex.clear_graphs()

    sids = [f"ab{i}" for i in range(B)]
    res = {v: [] for v in variants}
    for r in range(a.rounds):
        order = variants if r % 2 == 0 else variants[::-1]
        for v in order:
            apply(v)
            ex.forward([(s, a.prompt) for s in sids], prompts, reset=[True] * B)
            for t in range(4):
                ex.forward([(s, 1) for s in sids], toks[t])
            if dev == "cuda":
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            else:
                import time
                t0 = time.perf_counter()
            for t in range(a.steps):
                ex.forward([(s, 1) for s in sids], toks[4 + t])
            if dev == "cuda":
                e1.record()
                e1.synchronize()
                res[v].append(e0.elapsed_time(e1) / a.steps)
            else:
                res[v].append(1000 * (time.perf_counter() - t0) / a.steps)
            for s in sids:
                ex.sessions.close(s)
    out = {v: {"mean_ms": round(sum(res[v]) / len(res[v]), 4), "windows": [round(t, 4) for t in res[v]]}
           for v in variants}
    print(json.dumps({"model": a.model, "batch": B, "fp8": a.fp8, "ab": out}), flush=True)


if __name__ == "__main__":
    with torch.no_grad():
        main()
