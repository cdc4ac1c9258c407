"""Host time of the decode graph's launch call in the real executor (Llama-2-7B shapes, 64 rows,
N layers): profiles/r5f shows hipGraphLaunch holding the host ~4 ms per 64-session step, while a
plain captured chain of 1024 torch kernels launches in < 1 ms (graph_launch_probe2.py)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from src.models.config import resolve_model  # noqa: E402
from src.models.weights import random_stage_weights  # noqa: E402
from src.runtime import executor as exmod  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cfg = resolve_model("llama2-7b")
w = random_stage_weights(cfg, 0, L, has_embed=True, has_head=True, device="cuda")
ex = exmod.StageExecutor(cfg, w, "cuda", kv_cache_bytes=(L * 1) << 29, max_sessions=80, max_seq_len=512, graph_max_batch=64)
B = 64
ids = torch.randint(0, cfg.vocab_size, (B * 128,), device="cuda")
seqs = [(f"s{i}", 128) for i in range(B)]
ex.forward(seqs, ids, reset=[True] * B)
times = []
orig = exmod._DecodeGraph.replay


def timed(self, plan, x):
    g = self.graph
    real = g.replay

    def rp():
        a = time.perf_counter()
        real()
        times.append(time.perf_counter() - a)
    g.replay = rp
    try:
        return orig(self, plan, x)
    finally:
        g.replay = real


exmod._DecodeGraph.replay = timed
tok = torch.randint(0, cfg.vocab_size, (B,), device="cuda")
for step in range(12):
    ex.forward([(s, 1) for s, _ in seqs], tok)
torch.cuda.synchronize()
t0 = time.perf_counter()
for step in range(10):
    ex.forward([(s, 1) for s, _ in seqs], tok)
issued = time.perf_counter() - t0
torch.cuda.synchronize()
tot = time.perf_counter() - t0
print(f"{L} layers: graph launch host time {1e3 * sum(times[-10:]) / 10:.3f} ms/step, 10 steps issued after "
      f"{1e3 * issued:.2f} ms, done after {1e3 * tot:.2f} ms", flush=True)
