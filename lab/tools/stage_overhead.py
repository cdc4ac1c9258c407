#!/usr/bin/env python3
"""Host overhead of one pipeline stage's decode step (diagnostic, not the benchmark).

At pp8 a Llama-2-7B stage holds 4 blocks: its GPU step is ~8x shorter than the 1-stage step,
so the host side of a micro-batch step (engine bookkeeping, Plan metadata, hipGraph replay,
channel calls) must stay below it or the pipeline goes host-bound.  This runs the serving
engine on ONE GPU over a stage of ``--layers`` blocks (embedding + head included, so it is the
heaviest stage shape) and prints wall ms per step, the GPU time of the stage compute
(hipEvents) and the host time spent inside the engine step.

    python scripts/stage_overhead.py --layers 4 --batch 64
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
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    a = ap.parse_args()

    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.parallel.engine import PipelineServingEngine, Request
    from src.runtime.executor import StageExecutor
    from src.runtime.sampler import SamplingParams

    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    cfg = resolve_model(a.model)
    w = random_stage_weights(cfg, 0, a.layers, has_embed=True, has_head=True, device=dev)
    max_len = 64 * ((a.prompt_len + a.steps + a.warmup + 80) // 64)
    ex = StageExecutor(cfg, w, dev, max_sessions=a.batch + 8, max_seq_len=max_len, kv_cache_bytes=(8 << 30) if dev.type == "cuda" else (64 << 20),
                       graph_max_batch=a.batch, max_tokens_per_step=a.batch * a.prompt_len)
    eng = PipelineServingEngine(ex, None, n_slots=1, batch=a.batch, max_step_tokens=a.batch * a.prompt_len)
    sp = SamplingParams(1.0, 0.92, 50, 1.5)
    g = torch.Generator().manual_seed(0)
    for i in range(a.batch):
        eng.submit(Request(torch.randint(0, cfg.vocab_size, (a.prompt_len,), generator=g).tolist(),
                           max_new_tokens=a.steps + a.warmup + 16, params=sp, stop_on_repeat=0, seed=i, rid=f"s{i}"))
    eng.run_rounds(2 + a.warmup)
    sync()
    host = []
    eng.timing = True
    t0 = time.perf_counter()
    for _ in range(a.steps):
        h0 = time.perf_counter()
        eng.run_rounds(1)
        host.append(time.perf_counter() - h0)
    sync()
    wall = (time.perf_counter() - t0) / a.steps
    gpu = eng.stage_ms() or 0.0
    host.sort()
    print(json.dumps({"layers": a.layers, "batch": a.batch, "wall_ms_per_step": round(1e3 * wall, 4),
                      "gpu_ms_per_step": round(gpu, 4), "host_ms_per_step_median": round(1e3 * host[len(host) // 2], 4),
                      "host_ms_per_step_p90": round(1e3 * host[int(len(host) * 0.9)], 4)}), flush=True)
    eng.drain()


if __name__ == "__main__":
    main()
