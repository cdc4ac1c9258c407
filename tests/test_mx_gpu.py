"""W8A8-MX decode GEMM (ops/csrc/gemm_mx.hip): the MX activation quantizer against its fp32
reference (``ops.mx_block_quant``) bit for bit, and the block-scaled MFMA GEMM against the fp32
oracle x_mx @ dequant(W)^T at M in {1, 30, 64} on 7B and 70B projection shapes: epilogue 0 (with and
without the fused-norm row scale), the residual-stream producer (epilogue 3) and the split-K partial
slabs the qkv fold reads.  CPU part: the reference quantizer's block map and error bound."""
import pytest
import torch

from src import ops

DEV = "cuda"


def bf(t):
    return t.to(torch.bfloat16)


def test_mx_block_quant_reference():
    """Every 32-value block (k-slices 4 kb + 2 sh + {0, 1}, lane groups 2 qh + {0, 1}) shares one power
    of two scale, the block maximum lands in (224, 448], the element error is e4m3's (<= 2^-4)."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(5, 256, generator=g) * torch.logspace(-3, 3, 256)[None, :]
    x[2, 128:] = 0.0  # an all-zero step: scale 1, zeros
    d = ops.mx_block_quant(x)
    xb = x.to(torch.bfloat16).float()
    assert torch.all(d[2, 128:] == 0)
    v = xb.view(5, 2, 2, 2, 2, 2, 8)
    dv = d.view(5, 2, 2, 2, 2, 2, 8)
    amax = v.abs().amax(dim=(3, 5, 6), keepdim=True)
    err = (dv - v).abs()
    # relative to the block max: 3 mantissa bits (max rel 2^-4), subnormals near 2^-9 of the max
    assert torch.all(err <= amax * 2.0 ** -4 + 1e-30)
    rel = (dv - v).abs() / v.abs().clamp_min(1e-30)
    big = v.abs() >= amax / 8
    assert torch.all(rel[big] <= 2.0 ** -4 + 1e-6)


def _dequant_gpu(ax, as_, M, K):
    """Decode the kernel's MX layout back to fp32 [M, K] (lane 16 q + r, byte 8 s + j in two 16-byte
    halves [h][lane]; the scale of block 2 (s >> 1) + (q >> 1) in byte mt of lane 16 b + r's word)."""
    MT = (M + 15) // 16
    nkb = K // 128
    q8 = ax.view(torch.float8_e4m3fn).float().view(nkb, MT, 2, 4, 16, 2, 8)  # kb, mt, h, q, r, s_lo, j
    q8 = q8.permute(0, 1, 3, 4, 2, 5, 6).reshape(nkb, MT, 4, 16, 4, 8)  # kb, mt, q, r, s = 2 h + s_lo, j
    e = as_.float().view(nkb, 4, 16, 4)[..., :MT].permute(0, 3, 1, 2) - 127.0  # kb, mt, b, r
    sc = torch.empty(nkb, MT, 4, 16, 4, 8, device=ax.device)
    for q in range(4):
        for s in range(4):
            sc[:, :, q, :, s, :] = torch.exp2(e[:, :, 2 * (s >> 1) + (q >> 1), :])[..., None]
    v = (q8 * sc).permute(1, 3, 0, 4, 2, 5).reshape(MT * 16, K)  # rows (mt, r), k = 128 kb + 32 s + 8 q + j
    return v[:M]


@pytest.mark.gpu
@pytest.mark.parametrize("M,K", [(1, 4096), (30, 8192), (64, 28672)])
def test_quant_mx_matches_reference(M, K):
    ops.load_library()
    x = bf(torch.randn(M, K, device=DEV) * torch.logspace(-2, 2, K, device=DEV)[None, :])
    ax, as_ = ops.quant_mx(ops.pack_act(x), M, K)
    got = _dequant_gpu(ax, as_, M, K)
    want = ops.mx_block_quant(x.float())
    assert torch.equal(got, want)
    MT = (M + 15) // 16
    if M % 16:  # rows past M: zero bytes, unit scales
        assert torch.all(ax.view(K // 128, MT, 2, 4, 16, 16)[:, MT - 1, :, :, M % 16:] == 0)
        assert torch.all(as_.view(K // 128, 4, 16, 4)[:, :, M % 16:, MT - 1] == 127)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 30, 64])
@pytest.mark.parametrize("N,K", [(12288, 4096), (4096, 11008), (10240, 8192), (8192, 8192), (8192, 28672)])
def test_mx_gemm_matches_oracle(M, N, K):
    ops.load_library()
    torch.manual_seed(M * 7 + N + K)
    x = bf(torch.randn(M, K, device=DEV))
    w = torch.randn(N, K, device=DEV) * 0.02
    wq, ws = ops.pack_weight_fp8(w)
    w8 = ops.w8_from_fp8(wq)
    wdq = ops.unpack_weight_w8(w8, ws, torch.float32)
    xp = ops.pack_act(x)
    ax, as_ = ops.quant_mx(xp, M, K)
    exact = ops.mx_block_quant(x.float()) @ wdq.t()
    y = ops.linear_mx(ax, as_, w8, ws, M)
    assert float((y.float() - exact).norm() / exact.norm()) < 6e-3  # bf16 outputs, fp32 accumulation
    torch.testing.assert_close(y.float(), exact, atol=3e-2, rtol=2e-2)
    # against the unquantized product: MX e4m3 activations cost a few percent, no more
    full = x.float() @ wdq.t()
    assert float((y.float() - full).norm() / full.norm()) < 0.05
    # fused-norm consumer row scale
    ss = ops.norm_stats_buffer(DEV)[0]
    ss.zero_()
    sq = (x.float() ** 2).sum(1)
    ss[0, :M] = torch.round(sq * 2.0 ** 20).long()
    y2 = ops.linear_mx(ax, as_, w8, ws, M, ss_in=ss, eps=1e-5)
    want = exact * torch.rsqrt(sq / K + 1e-5)[:, None]
    assert float((y2.float() - want).norm() / want.norm()) < 6e-3
    # partial slabs (the qkv fold's input): their sum is the unscaled product
    S = ops.rwk_split(M, N, K, 2)
    assert S >= 2
    part = ops.linear_mx(ax, as_, w8, ws, M, partials=True)
    assert part.shape == (S, M, N)
    assert float((part.sum(0) - exact).norm() / exact.norm()) < 1e-4  # fp32 sums in another order
    # residual-stream producer: residual, packed copy, row sums of squares
    res = bf(torch.randn(M, N, device=DEV))
    r0 = res.clone()
    ap = torch.zeros(ops.packed_numel(M, N), dtype=torch.bfloat16, device=DEV)
    ss_out, ss_zero = ops.norm_stats_buffer(DEV, 2)
    ss_out.zero_()
    ops.linear_mx(ax, as_, w8, ws, M, out=res, epilogue=3, residual=res, ap_out=ap, ss_out=ss_out, ss_zero=ss_zero)
    torch.testing.assert_close(res.float(), exact + r0.float(), atol=6e-2, rtol=2e-2)
    assert torch.equal(ops.unpack_act(ap, M, N), res)
    got_ss = ss_out.view(-1, 64).sum(0)[:M].double() / 2.0 ** 20
    torch.testing.assert_close(got_ss, (res.double() ** 2).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("nh,nkv", [(32, 8), (64, 8)])
@pytest.mark.parametrize("T", [1, 6, 33])
def test_attention_writes_mx(nh, nkv, T):
    """The GQA decode attention's MX output (``mx_out``) is bit for bit ``quant_mx`` of its bf16 packed
    output: same bf16 rounding, same block maxima, same e4m3 bytes and e8m0 scales (rows < T)."""
    import math

    from tests.test_kernels_gpu import _attn_case

    D = 128
    ctxs = [((7 * i) % 190) + 1 for i in range(T)]
    ps = 64
    q, kc, vc, bt, q_seq, q_ctx = _attn_case(nh, nkv, D, ctxs, ps=ps)
    pos = (q_ctx.long() - 1).clamp(min=0)
    slots = torch.stack([bt[i, int(p) // ps].long() * ps + int(p) % ps for i, p in enumerate(pos.tolist())])
    qb = torch.from_numpy(ops.query_blocks([1] * T, nh // nkv)).to(DEV)
    cos, sin = ops.rope_cos_sin(D, 2048, 10000.0, DEV)
    scale = 1 / math.sqrt(D)
    kc2, vc2 = kc.clone(), vc.clone()
    o = ops.attention_mfma_rope(q, kc, vc, bt, q_seq, q_ctx, qb, pos, cos, sin, slots, nh, nkv, scale, packed=True,
                                part_size=256, num_parts=1)
    K = nh * D
    ax, as_ = ops.mx_buffers(T, K, DEV)
    ops.attention_mfma_rope(q, kc2, vc2, bt, q_seq, q_ctx, qb, pos, cos, sin, slots, nh, nkv, scale, packed=True,
                            part_size=256, num_parts=1, mx_out=(ax, as_))
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)
    ax2, as2 = ops.quant_mx(o, T, K)
    assert torch.equal(_dequant_gpu(ax, as_, T, K), _dequant_gpu(ax2, as2, T, K))


@pytest.mark.gpu
def test_executor_mx_mode_tracks_w8a16(monkeypatch):
    """MPAMD_FP8_MODE=mx (the o projection on the MX GEMM, its input written by the GQA attention)
    against the default W8A16 executor on the same fp8 weights: a 2-layer Llama-3-8B-shaped stage,
    30-session prefill + graph-replayed decode steps."""
    import dataclasses

    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor

    cfg = dataclasses.replace(resolve_model("llama3-8b"), num_hidden_layers=2)
    calls = []
    real = ops.linear_mx
    monkeypatch.setattr(ops, "linear_mx", lambda *a, **k: calls.append(1) or real(*a, **k))
    B, P = 30, 16
    g = torch.Generator().manual_seed(5)
    prompts = torch.randint(0, cfg.vocab_size, (B * P,), generator=g).to(DEV)
    toks = torch.randint(0, cfg.vocab_size, (3, B), generator=g).to(DEV)
    outs = {}
    for mode in ("w8a16", "mx"):
        monkeypatch.setenv("MPAMD_FP8_MODE", mode)
        w = random_stage_weights(cfg, 0, 2, has_embed=True, has_head=True, device=DEV, seed=3, fp8=True)
        ex = StageExecutor(cfg, w, DEV, max_sessions=B + 2, max_seq_len=64, kv_cache_bytes=1 << 30,
                           graph_max_batch=B, max_tokens_per_step=B * P, warmup=False)
        assert ex._mx == (mode == "mx")
        sids = [f"s{i}" for i in range(B)]
        ex.forward([(s, P) for s in sids], prompts, reset=[True] * B)
        got = [ex.forward([(s, 1) for s in sids], toks[t]).float().clone() for t in range(3)]
        outs[mode] = torch.stack(got)
        del ex, w
        torch.cuda.empty_cache()
    assert calls, "the MX o projection never ran"
    a, b = outs["mx"], outs["w8a16"]
    assert torch.isfinite(a).all()
    rel = float((a - b).norm() / b.norm())
    assert rel < 0.06, rel  # MX e4m3 activations on two of the four projections
    agree = float((a.argmax(-1) == b.argmax(-1)).float().mean())
    assert agree >= 0.6, agree
