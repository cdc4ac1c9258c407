#!/usr/bin/env python3
"""Prefill throughput of one stage executor (cold first call vs warm repeats).

``bench.py``'s prefill round is the first forward of its shape (hipBLASLt heuristics, first
kernel loads, KV page reservation); this times the same ragged prefill step again on warm
state: B sessions x L prompt tokens through all blocks + the head (last-token logits).

    python scripts/prefill_bench.py --batch 1 --prompt-len 2048
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--prompt-len", type=int, default=2048)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--fp8", action="store_true")
    a = ap.parse_args()

    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor

    dev = torch.device("cuda:0")
    cfg = resolve_model(a.model)
    L = cfg.num_hidden_layers
    w = random_stage_weights(cfg, 0, L, has_embed=True, has_head=True, device=dev, fp8=a.fp8)
    T = a.batch * a.prompt_len
    ex = StageExecutor(cfg, w, dev, max_sessions=a.batch + 4, max_seq_len=a.prompt_len + 64,
                       kv_cache_bytes=16 << 30, max_tokens_per_step=T)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (T,), generator=g).to(dev)
    seqs = [(f"s{i}", a.prompt_len) for i in range(a.batch)]
    times = []
    for r in range(1 + a.repeats):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ex.forward(seqs, ids, reset=[True] * a.batch)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    warm = min(times[1:])
    # 2 FLOPs per weight per token (projections + lm_head on the last tokens only) + causal attention
    H, F = cfg.hidden_size, cfg.intermediate_size
    proj = L * (H * (cfg.q_dim + 2 * cfg.kv_dim) + cfg.q_dim * H + 3 * H * F)
    attn = L * 2 * a.batch * cfg.num_attention_heads * cfg.head_dim * a.prompt_len * (a.prompt_len + 1)
    flops = 2 * proj * T + attn + 2 * H * cfg.vocab_size * a.batch
    print(json.dumps({"model": a.model, "batch": a.batch, "prompt_len": a.prompt_len, "tokens": T,
                      "cold_s": round(times[0], 4), "warm_s": round(warm, 4),
                      "warm_tokens_per_s": round(T / warm, 1), "warm_tflops": round(flops / warm / 1e12, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
