#!/usr/bin/env python3
"""How long does the host sit inside ``hipGraphLaunch`` of the full-depth decode graph, and what does
the decode step cost end to end?  (The HIP trace showed the launch of the 7B 64-session graph blocking
the host for ~85% of the GPU step, leaving the host too little time for the next step's work.)  Run it
once per HIP runtime setting (they are read at HIP initialisation), e.g.

    ROC_SIGNAL_POOL_SIZE=1024 python lab/tools/decode_host_probe.py --batch 64
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from src.models.config import resolve_model  # noqa: E402
from src.models.weights import random_stage_weights  # noqa: E402
from src.runtime.executor import StageExecutor  # noqa: E402

KNOBS = ("ROC_SIGNAL_POOL_SIZE", "ROC_AQL_QUEUE_SIZE", "DEBUG_HIP_GRAPH_BATCH_SIZE", "DEBUG_CLR_MAX_BATCH_SIZE",
         "DEBUG_CLR_GRAPH_PACKET_CAPTURE", "DEBUG_HIP_FORCE_GRAPH_QUEUES", "HIP_FORCE_DEV_KERNARG",
         "DEBUG_HIP_KERNARG_COPY_OPT", "ROC_USE_FGS_KERNARG", "DEBUG_CLR_BATCH_CPU_SYNC_SIZE")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--layers", type=int, default=0, help="stage depth (0: the whole model)")
    a = ap.parse_args()
    cfg = resolve_model(a.model)
    if a.layers:
        import dataclasses
        cfg = dataclasses.replace(cfg, num_hidden_layers=a.layers)
    B, dev = a.batch, "cuda"
    w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device=dev, seed=0)
    ex = StageExecutor(cfg, w, dev, max_sessions=B + 8, max_seq_len=a.prompt + a.steps + 16,
                       kv_cache_bytes=16 << 30, graph_max_batch=B, max_tokens_per_step=B * a.prompt, warmup=False)
    ex.warmup_serving(B, a.prompt)
    inside = []
    orig = torch.cuda.CUDAGraph.replay

    def timed(self):
        t = time.perf_counter()
        orig(self)
        inside.append(time.perf_counter() - t)

    torch.cuda.CUDAGraph.replay = timed
    g = torch.Generator(device=dev).manual_seed(7)
    prompts = torch.randint(0, cfg.vocab_size, (B * a.prompt,), device=dev, generator=g)
    toks = torch.randint(0, cfg.vocab_size, (a.steps + 4, B), device=dev, generator=g)
    sids = [f"p{i}" for i in range(B)]
    ex.forward([(s, a.prompt) for s in sids], prompts, reset=[True] * B)
    for t in range(4):
        ex.forward([(s, 1) for s in sids], toks[t])
    torch.cuda.synchronize()
    inside.clear()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host = []
    cpu0 = time.process_time()
    e0.record()
    t0 = time.perf_counter()
    for t in range(a.steps):
        h = time.perf_counter()
        ex.forward([(s, 1) for s in sids], toks[4 + t])
        host.append(time.perf_counter() - h)
    e1.record()
    t_issue = time.perf_counter() - t0
    cpu = time.process_time() - cpu0
    e1.synchronize()
    gpu_ms = e0.elapsed_time(e1) / a.steps
    n = max(1, len(inside))
    print(json.dumps({"batch": B, "knobs": {k: os.environ[k] for k in KNOBS if k in os.environ},
                      "ms_per_step": round(gpu_ms, 4), "host_forward_ms": round(1e3 * sum(host) / len(host), 4),
                      "host_in_graph_launch_ms": round(1e3 * sum(inside) / n, 4), "replays": len(inside),
                      "host_issue_ms_per_step": round(1e3 * t_issue / a.steps, 4),
                      "host_cpu_ms_per_step": round(1e3 * cpu / a.steps, 4), "layers": cfg.num_hidden_layers}), flush=True)


if __name__ == "__main__":
    with torch.no_grad():
        main()
