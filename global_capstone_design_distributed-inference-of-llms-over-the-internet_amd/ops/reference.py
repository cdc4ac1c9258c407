"""Plain-PyTorch reference implementations of every HIP op.

Two uses:
* the CPU data path (tests, the GPT-2 plumbing config, any host without a GPU);
* numerics oracles for the GPU kernel tests (computed in fp32 from the same inputs).

Rounding points mirror the kernels (and HF): values are rounded to the activation
dtype where the HF LLaMA modules round them (reference petals/llama/block.py).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

GU_BLOCK = 16  # gate/up weights are interleaved in blocks of 16 rows: [g16 u16 g16 u16 ...]


def pack_act(x, out=None):
    """Row-major [M, K] -> flat packed decode activation Ap[K/32][ceil(M/16)][64][8] (see csrc/common.h)."""
    M, K = x.shape
    MT = (M + 15) // 16
    xp = torch.zeros(MT * 16, K, dtype=x.dtype, device=x.device)
    xp[:M] = x
    # [MT, 16(c), K/32, 4(q), 8(j)] -> [K/32, MT, 4(q), 16(c), 8(j)]
    y = xp.view(MT, 16, K // 32, 4, 8).permute(2, 0, 3, 1, 4).reshape(-1)
    if out is not None:
        out[: y.numel()].copy_(y)
        return out
    return y


def unpack_act(ap, M, K):
    MT = (M + 15) // 16
    x = ap[: MT * 16 * K].view(K // 32, MT, 4, 16, 8).permute(1, 3, 0, 2, 4).reshape(MT * 16, K)
    return x[:M]


SS_SHARDS, SS_ROWS, SS_FX = 32, 256, float(1 << 20)


def fx_sumsq(x):
    """Per-row sum of round(x^2 * 2^20) as exact int64 (gemm.hip fused-norm row statistics)."""
    return torch.round(x.float().pow(2).double() * SS_FX).to(torch.int64).sum(-1)


def rmsnorm(x, w, eps, out=None, residual=None, mode=0, rows=None, ss=None):
    dt = x.dtype
    if mode == 3:  # fused-norm stage entry: residual = x, y = raw x, ss = fixed-point sum(x^2) per row
        residual.copy_(x)
        ss.view(SS_SHARDS, SS_ROWS).zero_()
        ss.view(SS_SHARDS, SS_ROWS)[0, : x.shape[0]] = fx_sumsq(x)
        if out is not None:
            out[: x.shape[0]].copy_(x)
            return out
        return x.clone()
    if mode == 1:
        residual.copy_((residual.float() + x.float()).to(dt))
        src = residual
    elif mode == 2:
        residual.copy_(x)
        src = x
    else:
        src = x
    if rows is not None:
        src = src.index_select(0, rows.long())
    xf = src.float()
    n = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(dt)
    y = (n.float() * w.float()).to(dt)
    if out is not None:
        out[: y.shape[0]].copy_(y)
        return out
    return y


def rope_cos_sin(head_dim: int, max_pos: int, theta: float, device=None, scaling: Optional[dict] = None):
    """fp32 cos/sin tables [max_pos, head_dim/2] (HF LlamaRotaryEmbedding, incl. llama3 scaling)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling.get("factor", 8.0)
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        smooth = (old / wl - lo) / (hi - lo)
        mid = (1 - smooth) * scaled / factor + smooth * scaled
        is_mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv = torch.where(is_mid, mid, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def _rotate(x, cos, sin):
    half = x.shape[-1] // 2
    x1, x2 = x[..., :half].float(), x[..., half:].float()
    c, s = cos.unsqueeze(-2), sin.unsqueeze(-2)
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)


def _scatter_cache(cache, slots, rows):
    """rows [T, nkv, D] -> cache[page, :, off, :] for slots >= 0."""
    P, nkv, ps, D = cache.shape
    valid = slots >= 0
    if not bool(valid.any()):
        return
    s = slots[valid]
    page, off = s // ps, s % ps
    cache[page, :, off, :] = rows[valid].to(cache.dtype)


def rope_kv_write(qkv, positions, cos, sin, k_cache, v_cache, slots, nh, nkv):
    T = qkv.shape[0]
    D = k_cache.shape[-1]
    view = qkv[:, : (nh + 2 * nkv) * D].view(T, nh + 2 * nkv, D)
    c, s = cos[positions.long()], sin[positions.long()]
    q = _rotate(view[:, :nh], c, s).to(qkv.dtype)
    k = _rotate(view[:, nh : nh + nkv], c, s).to(qkv.dtype)
    v = view[:, nh + nkv :]
    view[:, :nh] = q
    _scatter_cache(k_cache, slots, k)
    _scatter_cache(v_cache, slots, v)


def kv_write(k, v, k_cache, v_cache, slots):
    nkv, D = k_cache.shape[1], k_cache.shape[3]
    _scatter_cache(k_cache, slots, k.reshape(k.shape[0], nkv, D))
    _scatter_cache(v_cache, slots, v.reshape(v.shape[0], nkv, D))


def paged_attention(q, k_cache, v_cache, block_tables, q_seq, q_ctx, nh, nkv, scale, out=None):
    """softmax(q k^T * scale) v over the first q_ctx[t] cached tokens of sequence q_seq[t]."""
    T = q.shape[0]
    D = k_cache.shape[-1]
    ps = k_cache.shape[2]
    rep = nh // nkv
    res = torch.zeros(T, nh, D, dtype=torch.float32, device=q.device)
    qv = q[:, : nh * D].reshape(T, nh, D).float()
    for t in range(T):
        n = int(q_ctx[t])
        if n <= 0:
            continue
        pages = block_tables[int(q_seq[t])][: (n + ps - 1) // ps].long()
        k = k_cache[pages].permute(1, 0, 2, 3).reshape(nkv, -1, D)[:, :n].float()
        v = v_cache[pages].permute(1, 0, 2, 3).reshape(nkv, -1, D)[:, :n].float()
        k = k.repeat_interleave(rep, 0)
        v = v.repeat_interleave(rep, 0)
        s = torch.einsum("hd,hnd->hn", qv[t], k) * scale
        p = torch.softmax(s, -1)
        res[t] = torch.einsum("hn,hnd->hd", p, v)
    y = res.reshape(T, nh * D).to(q.dtype)
    if out is not None:
        out.view(T, nh * D).copy_(y)
        return out
    return y


def embedding(ids, table, out=None):
    y = table[ids.long()]
    if out is not None:
        out.copy_(y.view_as(out))
        return out
    return y


def swiglu(gu, out=None):
    """gu [T, 2F] with 16-row interleaved gate/up blocks -> silu(g) * u, HF rounding."""
    T, F2 = gu.shape
    F = F2 // 2
    v = gu.view(T, F // GU_BLOCK, 2, GU_BLOCK)
    g, u = v[:, :, 0].reshape(T, F), v[:, :, 1].reshape(T, F)
    a = torch.nn.functional.silu(g.float()).to(gu.dtype)
    y = (a.float() * u.float()).to(gu.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def add(a, b, out=None):
    y = (a.float() + b.float()).to(a.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def argmax(logits, out=None):
    y = torch.argmax(logits.float(), dim=-1)
    if out is not None:
        out.copy_(y)
        return out
    return y


def linear(x, w, out=None, epilogue=0, residual=None, ss_in=None, inv_k=0.0, eps=0.0, ap_out=None, ss_out=None,
           ss_zero=None):
    """``ss_in``: scale row r of x @ w^T by rsqrt(ss_in[r] * inv_k + eps) (fused-norm consumer);
    epilogue 3: r = bf16(bf16(y) + residual) -> residual (in place) and ``ap_out`` (packed),
    ``ss_out[r] += sum(r^2)`` (fused-norm producer)."""
    if ss_zero is not None:
        ss_zero.zero_()
    y = torch.nn.functional.linear(x, w) if x.dtype == w.dtype else torch.nn.functional.linear(x.to(w.dtype), w)
    if ss_in is not None:
        tot = ss_in.view(SS_SHARDS, SS_ROWS).sum(0)[: y.shape[0]].double() / SS_FX
        y = y.float() * torch.rsqrt(tot.float() * inv_k + eps)[:, None]
    y = y.to(x.dtype)
    if epilogue == 3:
        o = add(y, residual)
        residual.copy_(o)
        pack_act(o, out=ap_out)
        ss_out.view(SS_SHARDS, SS_ROWS)[0, : o.shape[0]] += fx_sumsq(o)
        return residual
    if epilogue == 1:
        y = swiglu(y)
    elif epilogue == 2:
        y = add(y, residual)
    if out is not None:
        out.copy_(y)
        return out
    return y


def sample_row(logits_row: torch.Tensor, temperature: float, top_p: float, top_k: int,
               repetition_penalty: float = 1.5, generated_tokens=None, generator=None) -> int:
    """One-row sampler with the reference semantics (reference src/rpc_handler.py:327-403)."""
    logits = logits_row.detach().float().clone().view(1, -1)
    if temperature <= 0.0:
        return int(torch.argmax(logits, dim=-1).item())
    temp = max(temperature, 1e-5)
    V = logits.shape[-1]
    if repetition_penalty != 1.0 and generated_tokens:
        recent = list(generated_tokens[-50:])
        counts = {}
        for tok in recent:
            counts[tok] = counts.get(tok, 0) + 1
        for tok, cnt in counts.items():
            if 0 <= tok < V:
                pen = repetition_penalty ** cnt
                if logits[0, tok] > 0:
                    logits[0, tok] /= pen
                else:
                    logits[0, tok] *= pen
        if len(generated_tokens) >= 3:
            last3 = list(generated_tokens[-3:])
            if len(set(last3)) == 1 and 0 <= last3[0] < V:
                pen = repetition_penalty ** 3
                if logits[0, last3[0]] > 0:
                    logits[0, last3[0]] /= pen
                else:
                    logits[0, last3[0]] *= pen
    probs = torch.softmax(logits / temp, dim=-1)
    if 0 < top_k < V:
        tv, ti = torch.topk(probs, top_k, dim=-1)
        probs = torch.zeros_like(probs).scatter(-1, ti, tv)
    if 0.0 < top_p < 1.0:
        sp, si = torch.sort(probs, descending=True, dim=-1)
        cum = torch.cumsum(sp, dim=-1)
        keep = cum <= top_p
        keep[..., 0] = True
        filt = sp * keep
        filt = filt / filt.sum(dim=-1, keepdim=True)
        probs = torch.zeros_like(probs).scatter(-1, si, filt)
    probs = probs / probs.sum(dim=-1, keepdim=True)
    return int(torch.multinomial(probs, 1, generator=generator).item())


def push_history(recent, recent_len, toks):
    """Append toks[r] to row r of the left-aligned history (drop the oldest when full)."""
    cap = recent.shape[1]
    for r in range(recent.shape[0]):
        n = int(recent_len[r])
        if n >= cap:
            recent[r, :-1] = recent[r, 1:].clone()
            n = cap - 1
        recent[r, n] = int(toks[r])
        recent_len[r] = n + 1


def sample(logits, temps, top_ps, top_ks, rep_pens, recent, recent_len, seeds, workspace=None, out=None):
    R = logits.shape[0]
    res = torch.empty(R, dtype=torch.long, device=logits.device)
    for r in range(R):
        n = int(recent_len[r])
        hist = [int(t) for t in recent[r, :n].tolist()]
        g = torch.Generator(device="cpu")
        g.manual_seed(int(seeds[r]) & 0x7FFFFFFFFFFFFFFF)
        res[r] = sample_row(logits[r].cpu(), float(temps[r]), float(top_ps[r]), int(top_ks[r]),
                            float(rep_pens[r]), hist, generator=g)
    if out is not None:
        out.copy_(res)
        return out
    return res


# ------------------------------------------------------------------ fp8 (OCP e4m3fn) W8A8
FP8_MAX = 448.0


def pack_weight_fp8(w):
    """W [N, K] -> (Wq uint8 [N/16, K/64, 64, 16], per-row scale fp32 [N]); see csrc/fp8.hip."""
    N, K = w.shape
    wf = w.float()
    s = wf.abs().amax(1).clamp_min(1e-30) / FP8_MAX
    q = (wf / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).view(torch.uint8)
    qp = q.view(N // 16, 16, K // 64, 2, 4, 8).permute(0, 2, 4, 1, 3, 5).reshape(N // 16, K // 64, 64, 16)
    return qp.contiguous(), s.contiguous()


def unpack_weight_fp8(qp, s, dtype=torch.float32):
    n16, k64 = qp.shape[0], qp.shape[1]
    q = qp.view(n16, k64, 4, 16, 2, 8).permute(0, 3, 1, 4, 2, 5).reshape(n16 * 16, k64 * 64)
    return (q.view(torch.float8_e4m3fn).float() * s.float()[:, None]).to(dtype)


def quant_rows_fp8(x):
    """x [R, K] float -> (q float8 [R, K], scale [R]) with per-row absmax / 448 (1 for zero rows)."""
    x = x.float()
    amax = x.abs().amax(1)
    s = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
    return (x / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn), s


def quant_act_fp8(xp, M, K):
    """Packed bf16 activation (M rows) -> (A8 uint8 flat [K/64][MT][64][16], scale fp32 [MT*16])."""
    MT = (M + 15) // 16
    x = torch.zeros(MT * 16, K, dtype=torch.float32, device=xp.device)
    x[:M] = unpack_act(xp, M, K).float()
    q, s = quant_rows_fp8(x)
    a8 = q.view(torch.uint8).view(MT, 16, K // 64, 2, 4, 8).permute(2, 0, 4, 1, 3, 5).reshape(-1)
    return a8.contiguous(), s


def dequant_act_fp8(a8, s, M, K):
    MT = (M + 15) // 16
    q = a8[: MT * 16 * K].view(K // 64, MT, 4, 16, 2, 8).permute(1, 3, 0, 4, 2, 5).reshape(MT * 16, K)
    return (q.view(torch.float8_e4m3fn).float() * s[: MT * 16, None].float())[:M]


def linear_fp8(a8, a_scale, wq, w_scale, M, epilogue=0, residual=None, dtype=torch.bfloat16):
    """fp32 reference of csrc/fp8.hip gemm_fp8 (same epilogue rounding as the kernel)."""
    N, K = 16 * wq.shape[0], 64 * wq.shape[1]
    y = dequant_act_fp8(a8, a_scale, M, K) @ unpack_weight_fp8(wq, w_scale).t()
    if epilogue == 1:
        F = N // 2
        v = y.view(M, F // GU_BLOCK, 2, GU_BLOCK)
        g = v[:, :, 0].reshape(M, F).to(dtype).float()
        u = v[:, :, 1].reshape(M, F).to(dtype).float()
        a = torch.nn.functional.silu(g).to(dtype).float()
        return (a * u).to(dtype)
    if epilogue == 2:
        return (y.to(dtype).float() + residual.float()).to(dtype)
    return y.to(dtype)
