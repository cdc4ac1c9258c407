"""Stateless, differentiable stage forward/backward: the fine-tuning half of the Petals server.

Reference (vendored upstream server):
* ``run_rpc_forward`` (petals/server/block_functions.py:32-81) runs the span's blocks on a
  ``[B, T, H]`` hidden state with optional *deep prompts* ``[n_blocks, B, P, H]``. Before block i,
  ``hidden[:, :P] += prompts[i]``. No KV cache is involved.
* ``run_rpc_backward`` (:84-141) recomputes that forward with autograd and returns the gradient
  w.r.t. the input hidden state and w.r.t. the prompts. For block i, the prompt gradient is
  the gradient flowing into ``hidden[:, :P]`` at its input.
* handler endpoints ``rpc_forward(_stream)`` / ``rpc_backward(_stream)``
  (petals/server/handler.py:352-488). Server weights are frozen. Clients train prompts or
  adapters on their side.

The inference hot path (paged KV, HIP kernels, hipGraphs) is not differentiable and does not
need to be. This module is the training-time path: plain PyTorch ops on the stage's resident
weights (the same tensors the executor uses; no copies).
* GEMMs go through rocBLAS / hipBLASLt.
* Attention is an explicit causal softmax in fp32.
* Backward = recompute forward + ``torch.autograd.grad``, as upstream, so no activations are
  held between the two RPCs.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from ..models.weights import split_gate_up
from ..ops.moe import moe_mlp_torch
from ..ops.reference import rope_cos_sin


def _rms(x, w, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype) * w


class AutogradStage:
    """Differentiable view of a stage's blocks (LLaMA-family and GPT-2)."""

    def __init__(self, cfg, weights, device, dtype=None):
        self.cfg = cfg
        self.w = weights
        self.device = torch.device(device)
        self.dtype = dtype or (weights.layers[0].input_norm.dtype if cfg.model_type != "gpt2"
                               else weights.layers[0].ln1_w.dtype)
        self._cache = {}  # per-layer (gate, up) views, made once

    @property
    def n_blocks(self) -> int:
        return len(self.w.layers)

    # ------------------------------------------------------------------ blocks
    def _attn(self, q, k, v):
        """q [B,T,nh,D], k/v [B,T,nkv,D] -> [B,T,nh*D], causal, fp32 softmax."""
        B, T, nh, D = q.shape
        rep = nh // k.shape[2]
        k = k.repeat_interleave(rep, 2) if rep > 1 else k
        v = v.repeat_interleave(rep, 2) if rep > 1 else v
        s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) / math.sqrt(D)
        mask = torch.ones(T, T, dtype=torch.bool, device=q.device).triu(1)
        p = torch.softmax(s.masked_fill(mask, float("-inf")), -1)
        return torch.einsum("bhqk,bkhd->bqhd", p, v.float()).to(q.dtype).reshape(B, T, nh * D)

    def _llama_block(self, i, x, cos, sin):
        cfg, lay = self.cfg, self.w.layers[i]
        nh, nkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        B, T, _ = x.shape
        h = _rms(x, lay.input_norm, cfg.rms_norm_eps)
        qkv = h @ lay.qkv.t()
        q = qkv[..., : nh * D].view(B, T, nh, D)
        k = qkv[..., nh * D: (nh + nkv) * D].view(B, T, nkv, D)
        v = qkv[..., (nh + nkv) * D:].view(B, T, nkv, D)
        c, s = cos[:T].view(1, T, 1, D // 2).to(x.dtype), sin[:T].view(1, T, 1, D // 2).to(x.dtype)

        def rot(t):
            t1, t2 = t[..., : D // 2], t[..., D // 2:]
            return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], -1)

        x = x + self._attn(rot(q), rot(k), v) @ lay.o.t()
        h = _rms(x, lay.post_norm, cfg.rms_norm_eps)
        if lay.router is not None:
            return x + moe_mlp_torch(h, lay.router, lay.gate_up, lay.down, cfg.num_experts_per_tok)
        if i not in self._cache:
            self._cache[i] = split_gate_up(lay.gate_up)
        g, u = self._cache[i]
        return x + (F.silu(h @ g.t()) * (h @ u.t())) @ lay.down.t()

    def _gpt2_block(self, i, x):
        cfg, lay = self.cfg, self.w.layers[i]
        H, nh, D = cfg.hidden_size, cfg.num_attention_heads, cfg.head_dim
        B, T, _ = x.shape
        a = F.layer_norm(x, (H,), lay.ln1_w, lay.ln1_b, cfg.layer_norm_eps)
        q, k, v = [t.reshape(B, T, nh, D) for t in (a @ lay.attn_w.t() + lay.attn_b).split(H, -1)]
        x = x + self._attn(q, k, v) @ lay.proj_w.t() + lay.proj_b
        m = F.layer_norm(x, (H,), lay.ln2_w, lay.ln2_b, cfg.layer_norm_eps)
        m = F.gelu(m @ lay.fc_w.t() + lay.fc_b, approximate="tanh")
        return x + m @ lay.fc2_w.t() + lay.fc2_b

    # ------------------------------------------------------------------ public API
    def forward(self, hidden: torch.Tensor, prompts: Optional[torch.Tensor] = None) -> torch.Tensor:
        """hidden [B, T, H]; prompts None or [n_blocks, B|1, P, H] (P <= T). Returns [B, T, H]."""
        x = hidden.to(self.device, self.dtype)
        if prompts is not None:
            prompts = prompts.to(self.device, self.dtype)
            if prompts.dim() != 4 or prompts.shape[0] != self.n_blocks or prompts.shape[2] > x.shape[1]:
                raise ValueError(f"prompts must be [{self.n_blocks}, B, P<=T, H], got {tuple(prompts.shape)}")
        T = x.shape[1]
        cos = sin = None
        if self.cfg.model_type != "gpt2":
            cos, sin = rope_cos_sin(self.cfg.head_dim, T, self.cfg.rope_theta, self.device, self.cfg.rope_scaling)
        for i in range(self.n_blocks):
            if prompts is not None:
                P = prompts.shape[2]
                x = torch.cat([x[:, :P] + prompts[i], x[:, P:]], 1)
            x = self._gpt2_block(i, x) if self.cfg.model_type == "gpt2" else self._llama_block(i, x, cos, sin)
        return x

    def backward(self, hidden: torch.Tensor, grad_output: torch.Tensor,
                 prompts: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """Recompute the forward with autograd and return (grad_hidden, grad_prompts)."""
        with torch.enable_grad():
            x = hidden.detach().to(self.device, self.dtype).requires_grad_(True)
            p = None
            if prompts is not None:
                p = prompts.detach().to(self.device, self.dtype).requires_grad_(True)
            out = self.forward(x, p)
            inputs = [x] if p is None else [x, p]
            grads = torch.autograd.grad(out, inputs, grad_output.to(self.device, out.dtype), allow_unused=True)
        gp = None
        if p is not None:
            gp = grads[1] if grads[1] is not None else torch.zeros_like(p)
        return grads[0], gp
