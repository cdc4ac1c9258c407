import os, sys, traceback
sys.path.insert(0, os.getcwd())
import torch
from src.models.config import resolve_model
from src.models.weights import random_stage_weights
from src.runtime.executor import StageExecutor
cfg = resolve_model("small-llama")
print("cfg", cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim, cfg.vocab_size, flush=True)
w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cuda", seed=5)
ex = StageExecutor(cfg, w, "cuda", kv_cache_bytes=256 << 20, max_sessions=32, max_seq_len=512, use_graphs=True,
                   graph_max_batch=16, max_tokens_per_step=1024)
print("executor ok", flush=True)
try:
    print("warm", ex.warmup_serving(8, 25), flush=True)
except Exception:
    traceback.print_exc()
torch.cuda.synchronize()
print("done", flush=True)
