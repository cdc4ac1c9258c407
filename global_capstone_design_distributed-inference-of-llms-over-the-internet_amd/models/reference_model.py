"""Dense fp32 reference forward (no paging, no fusion) used as the correctness oracle.

Plays the role of the reference's single-GPU check (reference scripts/single_gpu_check.py:183-277):
the same weights run without any partitioning, cache paging or kernel fusion, with a
causal mask, in fp32.  Pipeline/executor outputs are compared against it.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.nn.functional as F

from ..ops.moe import moe_mlp_torch
from ..ops.reference import rope_cos_sin
from .weights import StageWeights, split_gate_up


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def llama_forward(weights: List[StageWeights], ids: torch.Tensor, return_hidden: bool = False) -> torch.Tensor:
    """ids [L] -> logits [L, V] in fp32 through all stages' layers (causal)."""
    cfg = weights[0].cfg
    H, nh, nkv, D = cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    L = ids.numel()
    dev = ids.device
    x = weights[0].embed.float()[ids.long()]
    cos, sin = rope_cos_sin(D, max(L, 1), cfg.rope_theta, dev, cfg.rope_scaling)
    mask = torch.full((L, L), float("-inf"), device=dev).triu(1)
    for sw in weights:
        for lay in sw.layers:
            h = _rms(x, lay.input_norm.float(), cfg.rms_norm_eps)
            qkv = h @ lay.qkv.float().t()
            q = qkv[:, : nh * D].view(L, nh, D)
            k = qkv[:, nh * D: (nh + nkv) * D].view(L, nkv, D)
            v = qkv[:, (nh + nkv) * D:].view(L, nkv, D)

            def rot(t):
                t1, t2 = t[..., : D // 2], t[..., D // 2:]
                c, s = cos[:L].unsqueeze(1), sin[:L].unsqueeze(1)
                return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], -1)

            q, k = rot(q), rot(k)
            rep = nh // nkv
            k = k.repeat_interleave(rep, 1)
            v = v.repeat_interleave(rep, 1)
            s = torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(D) + mask
            p = torch.softmax(s, -1)
            a = torch.einsum("hqk,khd->qhd", p, v).reshape(L, nh * D)
            x = x + a @ lay.o.float().t()
            h = _rms(x, lay.post_norm.float(), cfg.rms_norm_eps)
            if lay.router is not None:
                x = x + moe_mlp_torch(h, lay.router.float(), lay.gate_up.float(), lay.down.float(),
                                      cfg.num_experts_per_tok)
                continue
            g, u = split_gate_up(lay.gate_up.float())
            x = x + (F.silu(h @ g.t()) * (h @ u.t())) @ lay.down.float().t()
    if return_hidden:
        return x
    last = weights[-1]
    x = _rms(x, last.final_norm.float(), cfg.rms_norm_eps)
    return x @ last.lm_head.float().t()


def gpt2_forward(weights: List[StageWeights], ids: torch.Tensor) -> torch.Tensor:
    cfg = weights[0].cfg
    H, nh, D = cfg.hidden_size, cfg.num_attention_heads, cfg.head_dim
    L = ids.numel()
    dev = ids.device
    x = weights[0].embed.float()[ids.long()] + weights[0].pos_embed.float()[:L]
    mask = torch.full((L, L), float("-inf"), device=dev).triu(1)
    for sw in weights:
        for lay in sw.layers:
            a = F.layer_norm(x, (H,), lay.ln1_w.float(), lay.ln1_b.float(), cfg.layer_norm_eps)
            qkv = a @ lay.attn_w.float().t() + lay.attn_b.float()
            q, k, v = [t.view(L, nh, D) for t in qkv.split(H, 1)]
            s = torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(D) + mask
            o = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), v).reshape(L, H)
            x = x + o @ lay.proj_w.float().t() + lay.proj_b.float()
            m = F.layer_norm(x, (H,), lay.ln2_w.float(), lay.ln2_b.float(), cfg.layer_norm_eps)
            m = F.gelu(m @ lay.fc_w.float().t() + lay.fc_b.float(), approximate="tanh")
            x = x + m @ lay.fc2_w.float().t() + lay.fc2_b.float()
    last = weights[-1]
    x = F.layer_norm(x, (H,), last.final_norm.float(), last.final_norm_b.float(), cfg.layer_norm_eps)
    return x @ last.lm_head.float().t()


def reference_forward(weights: List[StageWeights], ids: torch.Tensor) -> torch.Tensor:
    if weights[0].cfg.model_type == "gpt2":
        return gpt2_forward(weights, ids)
    return llama_forward(weights, ids)


def greedy_generate(weights: List[StageWeights], prompt: torch.Tensor, n_new: int) -> List[int]:
    ids = prompt.clone()
    out = []
    for _ in range(n_new):
        logits = reference_forward(weights, ids)
        nxt = int(torch.argmax(logits[-1]))
        out.append(nxt)
        ids = torch.cat([ids, torch.tensor([nxt], device=ids.device, dtype=ids.dtype)])
    return out
