#!/usr/bin/env python3
"""Single-device reference run: the whole model in ONE StageExecutor (no partitioning).

The reference's correctness/perf oracle (scripts/single_gpu_check.py:183-315) runs HF
generate-style code on one GPU and prints top-5 logits, TTFT, decode tokens/s and total
throughput; distributed outputs are compared against it by hand.  Same report here, on the
framework's own engine (HIP kernels + hipGraph decode on a GPU, torch path on CPU), plus an
optional ``--check`` against the dense fp32 oracle.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.models.config import resolve_model  # noqa: E402
from src.models.reference_model import reference_forward  # noqa: E402
from src.models.tokenizer import load_tokenizer  # noqa: E402
from src.models.weights import build_stage_weights  # noqa: E402
from src.ops.reference import sample_row  # noqa: E402
from src.runtime.executor import StageExecutor  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--prompt", default="Hello, how are you?")
    ap.add_argument("--max_new_tokens", type=int, default=32)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--top_p", type=float, default=0.92)
    ap.add_argument("--top_k", type=int, default=50)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--check", action="store_true", help="compare every step's logits with the fp32 oracle")
    a = ap.parse_args()
    dev = torch.device(a.device)
    cfg = resolve_model(a.model)
    dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
    w = build_stage_weights(cfg, a.model, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device=dev, dtype=dt)
    ex = StageExecutor(cfg, w, dev, dtype=dt, max_sessions=2, max_seq_len=1024,
                       kv_cache_bytes=None if dev.type == "cuda" else 64 << 20)
    tok = load_tokenizer(a.model, cfg)
    ids = torch.tensor(tok.encode(a.prompt) if hasattr(tok, "encode") else tok(a.prompt).input_ids[0])
    sync = (lambda: torch.cuda.synchronize()) if dev.type == "cuda" else (lambda: None)
    t0 = time.perf_counter()
    logits = ex.forward([("s", len(ids))], ids.to(dev))
    sync()
    ttft = time.perf_counter() - t0
    v, i = logits[0].float().topk(5)
    print(f"Top5 ids: {i.tolist()}  logits: {[round(x, 2) for x in v.tolist()]}")
    gen = []
    seq = ids.clone()
    t1 = time.perf_counter()
    for step in range(a.max_new_tokens):
        nxt = sample_row(logits[0], a.temperature, a.top_p, a.top_k, 1.0, gen)
        gen.append(nxt)
        if a.check:
            seq = torch.cat([seq, torch.tensor([nxt])])
        if step == a.max_new_tokens - 1:
            break
        logits = ex.forward([("s", 1)], torch.tensor([nxt], device=dev))
        if a.check:
            ref = reference_forward([w], seq.to(dev))[-1]
            err = (logits[0].float() - ref).abs().max().item()
            print(f"step {step}: max |logit - fp32 oracle| = {err:.4f}")
    sync()
    dec = time.perf_counter() - t1
    print(f"Generated: {tok.decode(gen)!r}")
    print(f"TTFT: {ttft:.3f}s  decode: {dec:.3f}s  ({(len(gen) - 1) / max(dec, 1e-9):.2f} tokens/s)  "
          f"throughput: {len(gen) / (ttft + dec):.2f} tokens/s")


if __name__ == "__main__":
    main()
