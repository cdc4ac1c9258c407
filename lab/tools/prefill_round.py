#!/usr/bin/env python3
"""Where the bench's first (prefill) round goes: a one-stage Llama serving engine, warmed as
``bench.py`` warms it, then B requests of L prompt tokens admitted and ONE round run - timed on
the host (cProfile, top cumulative entries) and on the GPU (HIP events around every executor
forward) - followed by a second, identical round on fresh requests (the warm reference).

    python scripts/prefill_round.py --batch 64 --prompt-len 128
"""
from __future__ import annotations

import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--profile", action="store_true", help="cProfile the cold round (inflates its time)")
    a = ap.parse_args()

    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.parallel.engine import PipelineServingEngine, Request
    from src.runtime.executor import StageExecutor
    from src.runtime.sampler import SamplingParams

    dev = torch.device("cuda:0")
    cfg = resolve_model(a.model)
    L, B, P = cfg.num_hidden_layers, a.batch, a.prompt_len
    w = random_stage_weights(cfg, 0, L, has_embed=True, has_head=True, device=dev, dtype=torch.bfloat16)
    ex = StageExecutor(cfg, w, dev, max_sessions=2 * B + 8, max_seq_len=256, graph_max_batch=B,
                       max_tokens_per_step=B * P)
    t0 = time.perf_counter()
    eng = PipelineServingEngine(ex, None, n_slots=1, batch=B, name="pr")
    eng.freeze_heap = True
    eng._settle_heap()  # as bench.py / the CLI do before their first round
    t_init = time.perf_counter() - t0
    gpu = []
    orig = ex.forward

    def timed_forward(*args, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = orig(*args, **kw)
        e1.record()
        gpu.append((e0, e1))
        return out

    ex.forward = timed_forward
    sp = SamplingParams(1.0, 0.92, 50, 1.5)
    gen = torch.Generator().manual_seed(0)
    rec = {"model": a.model, "batch": B, "prompt_len": P, "engine_init_s": round(t_init, 3)}
    for tag in ("cold", "warm"):
        for i in range(B):
            prompt = torch.randint(0, cfg.vocab_size, (P,), generator=gen).tolist()
            eng.submit(Request(prompt, max_new_tokens=4, params=sp, stop_on_repeat=0, seed=i, rid=f"{tag}{i}"))
        gpu.clear()
        torch.cuda.synchronize()
        prof = cProfile.Profile() if tag == "cold" and a.profile else None
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        eng.run_rounds(1)
        torch.cuda.synchronize()
        if prof:
            prof.disable()
        dt = time.perf_counter() - t0
        rec[f"{tag}_round_s"] = round(dt, 4)
        rec[f"{tag}_forward_gpu_ms"] = [round(e0.elapsed_time(e1), 2) for e0, e1 in gpu]
        if prof:
            s = io.StringIO()
            pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(25)
            print(s.getvalue(), file=sys.stderr)
        eng.run_until_idle()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
