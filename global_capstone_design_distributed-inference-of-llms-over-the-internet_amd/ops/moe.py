"""Mixtral sparse-MoE MLP: top-k softmax routing and the expert combine.

The reference accepts ``model_type == "mixtral"`` (src/llama_partition.py:81-83) and runs
HF ``MixtralSparseMoeBlock`` on the host; this module gives the same math to this
framework's engine:

* routing (HF semantics): ``softmax(router(h))`` over all E experts in fp32, keep the top-k,
  renormalise the kept weights to sum to 1;
* expert j: ``down_j(silu(gate_j h) * up_j h)``; token output = sum_j w_j * expert_j(h).

MI355X execution strategy (runtime/executor.py ``_moe_mlp``):

* decode steps (T <= 64 rows) run EVERY expert on the whole (tiny) batch through the packed
  weight-streaming GEMMs and combine with a dense [T, E] weight matrix whose unrouted
  entries are zero.  A decode step is HBM-bound: at batch 64 with top-2 of 8 experts every
  expert is routed to by some token (P(unused) = (6/8 * 5/7)^64 ~ 1e-10), so the bytes read
  equal the sparse schedule's, the extra MFMA work is free at M <= 64, and the step has no
  data-dependent shapes - it stays inside the hipGraph;
* prefill (T > 64) groups tokens by expert (one host sync per layer, outside any graph),
  runs each expert's GEMMs on its gathered rows and scatter-adds the weighted result.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn.functional as F

from .reference import GU_BLOCK


def route(logits: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Router logits [T, E] -> (weights fp32 [T, k] summing to 1, expert ids [T, k])."""
    p = torch.softmax(logits.float(), dim=-1)
    w, idx = torch.topk(p, k, dim=-1)
    return w / w.sum(-1, keepdim=True), idx


def dense_weights(w: torch.Tensor, idx: torch.Tensor, E: int, out: torch.Tensor = None) -> torch.Tensor:
    """Top-k (w, idx) -> dense combine matrix [T, E] (zeros for unrouted experts)."""
    if out is None:
        out = torch.zeros(w.shape[0], E, dtype=torch.float32, device=w.device)
    else:
        out.zero_()
    return out.scatter_(1, idx, w)


def _split(gu: torch.Tensor):
    F2, H = gu.shape
    v = gu.view(F2 // (2 * GU_BLOCK), 2, GU_BLOCK, H)
    return v[:, 0].reshape(F2 // 2, H), v[:, 1].reshape(F2 // 2, H)


def moe_mlp_torch(h: torch.Tensor, router: torch.Tensor, gate_up: torch.Tensor, down: torch.Tensor,
                  k: int) -> torch.Tensor:
    """Differentiable plain-PyTorch MoE MLP in ``h``'s dtype (oracle + stateless autograd stage).

    h [..., H]; router [E, H]; gate_up [E, 2F, H] (16-row interleaved); down [E, H, F]."""
    shp = h.shape
    x = h.reshape(-1, shp[-1])
    w, idx = route(x @ router.t(), k)
    out = torch.zeros_like(x, dtype=torch.float32)
    for e in range(router.shape[0]):
        tok, slot = (idx == e).nonzero(as_tuple=True)
        if tok.numel() == 0:
            continue
        g, u = _split(gate_up[e])
        xe = x[tok]
        y = (F.silu(xe @ g.t()) * (xe @ u.t())) @ down[e].t()
        out = out.index_add(0, tok, y.float() * w[tok, slot].unsqueeze(1))
    return out.to(h.dtype).reshape(shp)
