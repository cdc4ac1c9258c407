"""Where does the GPU executor leave the bf16 envelope?  Per-step logit error vs the fp32 oracle
(computed on the CPU and on the GPU) for the executor variants: default (fused norm + graphs),
eager, no fused norm, hipBLASLt GEMMs; plus the CPU bf16 executor as the expected bf16 distance,
and the stage's hidden state (no head) after its layers."""
import dataclasses
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from src import ops  # noqa: E402
from src.models.config import resolve_model  # noqa: E402
from src.models.reference_model import llama_forward, reference_forward  # noqa: E402
from src.models.weights import random_stage_weights  # noqa: E402
from src.runtime.executor import StageExecutor  # noqa: E402


def run(cfg, dev, dtype, seqs, head=True, **kw):
    w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=head, device="cuda", seed=11)
    if dev == "cpu":
        import copy
        w = copy.deepcopy(w)
        for lay in w.layers:
            for f in dataclasses.fields(lay):
                t = getattr(lay, f.name)
                if isinstance(t, torch.Tensor):
                    setattr(lay, f.name, t.cpu())
        for n in ("embed", "final_norm", "lm_head"):
            if getattr(w, n) is not None:
                setattr(w, n, getattr(w, n).cpu())
    ex = StageExecutor(cfg, w, dev, dtype=dtype, kv_cache_bytes=256 << 20, max_sessions=8, max_seq_len=256,
                       max_tokens_per_step=1024, warmup=False, **kw)
    B = seqs.shape[0]
    s = seqs.to(dev)
    out = [ex.forward([(f"s{i}", 8) for i in range(B)], s[:, :8].reshape(-1), reset=[True] * B).clone()]
    if not head:
        return w, out[0].float().cpu().view(B, 8, -1)
    for t in range(2):
        out.append(ex.forward([(f"s{i}", 1) for i in range(B)], s[:, 8 + t].contiguous()).clone())
    return w, torch.stack([o.float().cpu() for o in out], 1)


def err(a, b):
    return [round(float((a[:, k] - b[:, k]).norm() / b[:, k].norm()), 4) for k in range(a.shape[1])]


def main():
    for name in sys.argv[1:] or ["small-llama", "llama2-7b"]:
        cfg = resolve_model(name)
        if cfg.num_hidden_layers > 8:
            cfg = dataclasses.replace(cfg, num_hidden_layers=2)
        g = torch.Generator().manual_seed(3)
        seqs = torch.randint(0, cfg.vocab_size, (3, 10), generator=g)
        w, got = run(cfg, "cuda", torch.bfloat16, seqs)
        ref_gpu = torch.stack([reference_forward([w], seqs[i].cuda())[7:].float().cpu() for i in range(3)])
        wc = w
        print(name, "default vs fp32-oracle(gpu)", err(got, ref_gpu), flush=True)
        _, e = run(cfg, "cuda", torch.bfloat16, seqs, use_graphs=False)
        print(name, "eager", err(e, ref_gpu), flush=True)
        os.environ["MPAMD_FUSED_NORM"] = "0"
        _, e = run(cfg, "cuda", torch.bfloat16, seqs)
        print(name, "no fused norm", err(e, ref_gpu), flush=True)
        os.environ.pop("MPAMD_FUSED_NORM")
        ops.set_gemm_policy("hipblaslt")
        _, e = run(cfg, "cuda", torch.bfloat16, seqs)
        print(name, "hipblaslt gemms", err(e, ref_gpu), flush=True)
        ops.set_gemm_policy("auto")
        _, c = run(cfg, "cpu", torch.bfloat16, seqs)
        print(name, "cpu bf16 executor", err(c, ref_gpu), flush=True)
        print(name, "gpu default vs cpu bf16", err(got, c), flush=True)
        _, h = run(cfg, "cuda", torch.bfloat16, seqs, head=False)
        hr = torch.stack([llama_forward([wc], seqs[i, :8].cuda(), return_hidden=True).float().cpu() for i in range(3)])
        print(name, "hidden after the stage (prefill rows)", [round(float((h[:, k] - hr[:, k]).norm() / hr[:, k].norm()), 4)
                                                            for k in range(8)], flush=True)


if __name__ == "__main__":
    with torch.no_grad():
        main()
