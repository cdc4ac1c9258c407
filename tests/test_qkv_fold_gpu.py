"""The qkv projection folded into decode attention (ops.linear_partials + the attention kernels'
``qkv_part`` loads, csrc/common.h qkv_part_load8): the split-K ring leaves fp32 partial slabs, the
attention kernel sums them, applies the fused-norm row scale and rounds to bf16 on its q / k / v
loads.  Contract: bit-identical to the unfolded pair (split-K ring + reduce launch, then the same
attention kernel on the bf16 qkv) - outputs and the KV-cache slot writes - for the MHA
flash-decoding kernel and the GQA MFMA kernel, bf16 and fp8 (W8A16) weights; and an fp32 oracle
of the projection + row scale."""
import math

import pytest
import torch

from src import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(nh, nkv, D, M, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    K = 1024
    N = (nh + 2 * nkv) * D
    ps, maxc = 64, 96
    ctxs = torch.randint(1, maxc, (M,), generator=g, device=DEV).to(torch.int32)
    P = M * 2 + 3
    kc = (torch.randn(P, nkv, ps, D, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.randperm(P, device=DEV)[: M * 2].view(M, 2).to(torch.int32)
    pos = (ctxs.long() - 1).clamp(min=0)
    slots = torch.stack([bt[i, int(p) // ps].long() * ps + int(p) % ps for i, p in enumerate(pos.tolist())])
    x = (torch.randn(M, K, device=DEV, generator=g) * 0.7).to(torch.bfloat16)
    ss = ops.norm_stats_buffer(DEV)[0]
    ss.zero_()
    ss[0, :M] = torch.round((x.float() ** 2).sum(1) * 2.0 ** 20).long()
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.03).to(torch.bfloat16)
    return dict(N=N, K=K, x=x, xp=ops.pack_act(x), ss=ss, w=w, kc=kc, vc=vc, bt=bt,
                q_seq=torch.arange(M, dtype=torch.int32, device=DEV), q_ctx=ctxs, pos=pos, slots=slots)


def _attend(c, nh, nkv, D, qkv, qkv_part, gqa):
    cos, sin = ops.rope_cos_sin(D, 2048, 10000.0, DEV)
    kc, vc = c["kc"].clone(), c["vc"].clone()
    M = qkv.shape[0]
    scale = 1 / math.sqrt(D)
    if gqa:
        qb = torch.stack([torch.arange(M), torch.ones(M, dtype=torch.long)]).to(torch.int32).to(DEV)
        o = ops.attention_mfma_rope(qkv, kc, vc, c["bt"], c["q_seq"], c["q_ctx"], qb, c["pos"], cos, sin, c["slots"],
                                    nh, nkv, scale, max_ctx=96, packed=True, qkv_part=qkv_part)
    else:
        o = ops.paged_attention_rope(qkv, kc, vc, c["bt"], c["q_seq"], c["q_ctx"], c["pos"], cos, sin, c["slots"],
                                     nh, nkv, scale, max_ctx=96, packed=True, qkv_part=qkv_part)
    torch.cuda.synchronize()
    return ops.unpack_act(o, M, nh * D).clone(), kc, vc  # the real rows (packed padding is never written)


@pytest.mark.parametrize("nh,nkv,D,gqa", [(32, 32, 128, False), (32, 8, 128, True), (64, 8, 128, True),
                                          (16, 16, 64, False)])
@pytest.mark.parametrize("M", [1, 16, 48, 64])
@pytest.mark.parametrize("fp8", [False, True])
def test_fold_bit_identical_to_reduce_launch(nh, nkv, D, gqa, M, fp8, monkeypatch):
    c = _case(nh, nkv, D, M, seed=M)
    N, K = c["N"], c["K"]
    if ops.rwk_split(M, N, K, fp8) <= 0:
        pytest.skip("no split-K ring form for this width")
    eps = 1e-5
    if fp8:
        wq, wsc = ops.pack_weight_fp8(c["w"])
        w8 = ops.w8_from_fp8(wq)
        monkeypatch.setattr(ops, "_W8_MODE", "rwk")
        qkv = ops.linear_w8(c["xp"], w8, wsc, M, ss_in=c["ss"], eps=eps)
        wdq = ops.unpack_weight_w8(w8, wsc, torch.float32).to(torch.bfloat16).float()
    else:
        wp = ops.pack_weight(c["w"])
        ops.set_gemm_sk("rwk")
        try:
            qkv = ops.linear(c["xp"], None, wp=wp, a_rows=M, ss_in=c["ss"], eps=eps)
        finally:
            ops.set_gemm_sk("auto")
        wdq = c["w"].float()
    # the unfolded pair: reduce launch -> bf16 qkv -> attention
    o1, k1, v1 = _attend(c, nh, nkv, D, qkv, None, gqa)
    # the fold: partial slabs -> attention sums them
    dummy = torch.full_like(qkv, float("nan"))  # never read on the fold path
    part = (ops.linear_partials(c["xp"], M, w8=w8, w_scale=wsc, out=dummy) if fp8
            else ops.linear_partials(c["xp"], M, wp=wp, out=dummy))
    assert part.shape == (ops.rwk_split(M, N, K, fp8), M, N)
    o2, k2, v2 = _attend(c, nh, nkv, D, dummy, (part, c["ss"], 1.0 / K, eps), gqa)
    assert torch.equal(o1, o2)
    assert torch.equal(k1, k2) and torch.equal(v1, v2)
    # oracle: the partials are the fp32 projection, the row scale the RMS of x
    rs = torch.rsqrt((c["x"].float() ** 2).mean(1) + eps)
    want = (c["x"].float() @ wdq.t()) * rs[:, None]
    got = ops.reduce_qkv_part((part, c["ss"], 1.0 / K, eps), torch.float32)
    torch.testing.assert_close(got, want, atol=3e-2, rtol=2e-2)
    assert bool(torch.isfinite(o2.float()).all())


def test_executor_fold_on_off_same_logits(monkeypatch):
    """A Llama decode step through the fused executor with the fold forced on == forced off."""
    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor

    import dataclasses

    monkeypatch.setenv("MPAMD_GEMM_AUTOTUNE", "0")
    # (8 + 2 x 4) heads x 128: a qkv width the split-K ring covers (N % 2048 == 0)
    cfg = dataclasses.replace(resolve_model("small-llama"), hidden_size=1024, num_attention_heads=8,
                              num_key_value_heads=4, intermediate_size=2048, num_hidden_layers=2)
    outs = []
    for fold in (False, True):
        w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device=DEV, seed=3)
        ex = StageExecutor(cfg, w, DEV, kv_cache_bytes=64 << 20, max_sessions=16, max_seq_len=256, use_graphs=False)
        N, K = cfg.q_dim + 2 * cfg.kv_dim, cfg.hidden_size
        ex.qkv_fold_by_bucket = {ex._bucket(8): fold}
        monkeypatch.setattr(ops, "_SK_CHOICE", {(ops._m_bucket(8), N, K, 0): "rwk"})
        ids = torch.arange(8 * 12, device=DEV) % cfg.vocab_size
        ex.forward([(f"s{i}", 12) for i in range(8)], ids)
        used = ex._qkv_fold(8)
        lg = ex.forward([(f"s{i}", 1) for i in range(8)], ids[:8])
        torch.cuda.synchronize()
        outs.append((used, lg.float().cpu()))
    assert outs[0][0] is False and outs[1][0] is True
    assert torch.equal(outs[0][1], outs[1][1])
