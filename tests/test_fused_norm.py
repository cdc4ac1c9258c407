"""Fused-norm decode path (ops/csrc/gemm.hip EpiArgs, norm.hip mode 3, executor fused branch).

RMSNorm(x) W^T == rsqrt(mean x^2 + eps) * (x (g W)^T): the consumer GEMMs take the raw
residual stream with the norm weight folded into the packed weight and scale rows in the
epilogue; the producer GEMMs (o, down) add into the residual in place, write the packed copy
and accumulate per-row sums of squares with atomics.  Every kernel family (pk, stream-K,
shared-A) is checked against an fp32 PyTorch reference of the unfused math, and a whole
decode step of the fused executor against the unfused packed path and the fp32 oracle.
"""
import pytest
import torch

from src import ops
from src.ops import reference as ref

EPS = 1e-5


def _rms_ref(x, g):
    xf = x.float()
    n = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + EPS)).to(x.dtype)
    return (n.float() * g.float()).to(x.dtype)


def test_reference_fold_identity_cpu():
    """The CPU reference ops implement the same identity the kernels use."""
    g = torch.Generator().manual_seed(0)
    M, K, N = 5, 64, 48
    x = torch.randn(M, K, generator=g)
    gw = torch.rand(K, generator=g) + 0.5
    w = torch.randn(N, K, generator=g) * 0.05
    ss = ops.norm_stats_buffer("cpu")[0]
    res = torch.zeros(M, K)
    xr = ops.rmsnorm(x, gw, EPS, residual=res, mode=3, ss=ss)
    torch.testing.assert_close(ss.sum(0)[:M].double() / 2 ** 20, x.double().pow(2).sum(-1), atol=1e-3, rtol=1e-6)
    torch.testing.assert_close(res, x)
    y = ops.linear(xr, w * gw[None, :], ss_in=ss, eps=EPS)
    torch.testing.assert_close(y, _rms_ref(x, gw) @ w.t(), atol=1e-4, rtol=1e-4)
    # producer: residual in place + packed copy + sum of squares
    a = torch.randn(M, N, generator=g)
    wo = torch.randn(K, N, generator=g) * 0.05
    res0 = res.clone()
    ap = torch.zeros(ops.packed_numel(M, K))
    sso, ssz = ops.norm_stats_buffer("cpu")[0], ops.norm_stats_buffer("cpu")[0] + 5
    ops.linear(a, wo, out=res, epilogue=3, residual=res, ap_out=ap, ss_out=sso, ss_zero=ssz)
    o = res0 + a @ wo.t()
    torch.testing.assert_close(res, o, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(ref.unpack_act(ap, M, K), o, atol=1e-5, rtol=1e-5)
    assert torch.equal(sso.sum(0)[:M], ref.fx_sumsq(res))
    assert int(ssz.abs().sum()) == 0


def test_t2d_row_range_policy_cpu(monkeypatch):
    """Which decode row counts the two-dimensionally tiled kernel owns (ops.T2D_MIN .. 256), and
    how far the packed (hand-written GEMM) path reaches with and without it."""
    monkeypatch.setattr(ops, "T2D_MIN", 129)
    assert [ops.t2d_rows(m) for m in (64, 128, 129, 200, 256, 257)] == [False, False, True, True, True, False]
    assert ops.wide_rows() == 256
    monkeypatch.setattr(ops, "T2D_MIN", 257)  # off: the ring kernels up to WIDE_ROWS, hipBLASLt above
    assert not any(ops.t2d_rows(m) for m in (129, 256))
    assert ops.wide_rows() == ops.WIDE_ROWS
    monkeypatch.setattr(ops, "T2D_MIN", 10)  # never below 65 rows (the M <= 64 kernels own that range)
    assert not ops.t2d_rows(64) and ops.t2d_rows(65)
    assert "t2d" in ops._KERNEL_FLAGS and not ops._covered("t2d", 64, 4096, 4096, 0)


KERNELS = ["pk", "sk", "lds22", "lds24", "lds42", "rw", "rwk", "rwki", "rwr"]


@pytest.mark.gpu
@pytest.mark.parametrize("kern", KERNELS)
@pytest.mark.parametrize("M", [1, 17, 64])
def test_consumer_row_scale_matches_rmsnorm_then_gemm(kern, M):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(M)
    K, N = 1024, 2048  # N % 2048 == 0: the split-K ring form applies too (plain-epilogue consumer)
    x = (torch.randn(M, K, device=dev, generator=g) * 0.7).to(torch.bfloat16)
    gw = (torch.rand(K, device=dev, generator=g) + 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    ss = ops.norm_stats_buffer(dev)[0] + 3  # stale shards: mode 3 must overwrite all of a row's
    res = torch.empty_like(x)
    xp = torch.zeros(ops.packed_numel(M, K), dtype=torch.bfloat16, device=dev)
    ops.rmsnorm(x, gw, EPS, out=xp, residual=res, mode=3, packed=True, ss=ss)
    assert torch.equal(ss.sum(0)[:M].cpu(), ref.fx_sumsq(x.cpu()))  # exact fixed-point sums
    assert torch.equal(res, x)
    wp = ops.pack_weight((w.float() * gw.float()[None, :]).to(torch.bfloat16).contiguous())
    ops.set_gemm_sk(kern)
    try:
        y = ops.linear(xp, None, wp=wp, a_rows=M, ss_in=ss, eps=EPS)
        # SwiGLU consumer (gate/up interleaved weight), packed output
        wgu = (torch.randn(2 * N, K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
        wgup = ops.pack_weight((wgu.float() * gw.float()[None, :]).to(torch.bfloat16).contiguous())
        act = torch.zeros(ops.packed_numel(M, N), dtype=torch.bfloat16, device=dev)
        ops.linear(xp, None, out=act, epilogue=1, wp=wgup, a_rows=M, out_packed=True, ss_in=ss, eps=EPS)
    finally:
        ops.set_gemm_sk("auto")
    xn = _rms_ref(x, gw).float()
    torch.testing.assert_close(y.float(), xn @ w.float().t(), atol=3e-2, rtol=3e-2)
    gu = xn @ wgu.float().t()
    exp = ref.swiglu(gu.to(torch.bfloat16)).float()
    torch.testing.assert_close(ref.unpack_act(act, M, N).float(), exp, atol=3e-2, rtol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("kern", KERNELS)
@pytest.mark.parametrize("M", [1, 16, 33, 48, 64])
def test_producer_epilogue_residual_pack_and_sumsq(kern, M):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(100 + M)
    K, N = 2048, 2048
    a = (torch.randn(M, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    res = (torch.randn(M, N, device=dev, generator=g)).to(torch.bfloat16)
    res0 = res.clone()
    ap = torch.zeros(ops.packed_numel(M, N), dtype=torch.bfloat16, device=dev)
    sso = ops.norm_stats_buffer(dev)[0]
    ssz = ops.norm_stats_buffer(dev)[0] + 7
    ops.set_gemm_sk(kern)
    try:
        ops.linear(ops.pack_act(a), None, out=res, epilogue=3, residual=res, wp=ops.pack_weight(w), a_rows=M,
                   ap_out=ap, ss_out=sso, ss_zero=ssz)
    finally:
        ops.set_gemm_sk("auto")
    exp = (res0.float() + (a.float() @ w.float().t()).to(torch.bfloat16).float()).to(torch.bfloat16)
    torch.testing.assert_close(res.float(), exp.float(), atol=2e-2, rtol=2e-2)
    assert torch.equal(ref.unpack_act(ap, M, N), res)
    assert torch.equal(sso.sum(0)[:M].cpu(), ref.fx_sumsq(res.cpu()))  # exact, order-independent
    assert int(ssz.abs().sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("M", [65, 96, 128, 129, 192, 200, 256])
def test_wide_rows_consumer_and_producer(M, monkeypatch):
    """65..256 rows (decode steps of 65..256 sessions): the consumers (qkv: split-K ring +
    reduce with the row scale; gate/up: balanced ring with the row scale and packed SwiGLU) and
    the producer (split-K ring + the reduce launch's residual / packed copy / statistics), against
    fp32 oracles.  Above 128 rows: the 12 / 16-row-tile ring instantiations."""
    monkeypatch.setattr(ops, "WIDE_ROWS", 256)  # above 128 rows the ring forms are opt-in
    monkeypatch.setattr(ops, "T2D_MIN", 257)  # (the tiled kernel's own test is below)
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(500 + M)
    K, N = 2048, 2048
    assert ops.wide_gemm_ok(M, N, K, 3)
    x = (torch.randn(M, K, device=dev, generator=g) * 0.7).to(torch.bfloat16)
    gw = (torch.rand(K, device=dev, generator=g) + 0.5).to(torch.bfloat16)
    ss = ops.norm_stats_buffer(dev)[0] + 3
    res = torch.empty_like(x)
    xp = torch.zeros(ops.packed_numel(M, K), dtype=torch.bfloat16, device=dev)
    ops.rmsnorm(x, gw, EPS, out=xp, residual=res, mode=3, packed=True, ss=ss)
    assert torch.equal(ss.sum(0)[:M].cpu(), ref.fx_sumsq(x.cpu()))
    w = (torch.randn(N, K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    wp = ops.pack_weight((w.float() * gw.float()[None, :]).to(torch.bfloat16).contiguous())
    y = ops.linear(xp, None, wp=wp, a_rows=M, ss_in=ss, eps=EPS)
    wgu = (torch.randn(2 * N, K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    wgup = ops.pack_weight((wgu.float() * gw.float()[None, :]).to(torch.bfloat16).contiguous())
    act = torch.zeros(ops.packed_numel(M, N), dtype=torch.bfloat16, device=dev)
    ops.linear(xp, None, out=act, epilogue=1, wp=wgup, a_rows=M, out_packed=True, ss_in=ss, eps=EPS)
    xn = _rms_ref(x, gw).float()
    torch.testing.assert_close(y.float(), xn @ w.float().t(), atol=3e-2, rtol=3e-2)
    exp = ref.swiglu((xn @ wgu.float().t()).to(torch.bfloat16)).float()
    # K = 2048: bf16 rounding of gate and up before the product (one element in 1e5 lands at 0.031)
    torch.testing.assert_close(ref.unpack_act(act, M, N).float(), exp, atol=5e-2, rtol=3e-2)
    # producer
    a = (torch.randn(M, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    wo = (torch.randn(N, K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    r0 = r.clone()
    ap = torch.zeros(ops.packed_numel(M, N), dtype=torch.bfloat16, device=dev)
    sso, ssz = ops.norm_stats_buffer(dev)[0], ops.norm_stats_buffer(dev)[0] + 7
    ops.linear(ops.pack_act(a), None, out=r, epilogue=3, residual=r, wp=ops.pack_weight(wo), a_rows=M,
               ap_out=ap, ss_out=sso, ss_zero=ssz)
    exp = (r0.float() + (a.float() @ wo.float().t()).to(torch.bfloat16).float()).to(torch.bfloat16)
    torch.testing.assert_close(r.float(), exp.float(), atol=2e-2, rtol=2e-2)
    assert torch.equal(ref.unpack_act(ap, M, N), r)
    assert torch.equal(sso.sum(0)[:M].cpu(), ref.fx_sumsq(r.cpu()))
    assert int(ssz.abs().sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("M", [200, 256])
def test_wide_ring_in_kernel_epilogues(M, monkeypatch):
    """The ring kernel's 12 / 16-row-tile forms with the decode epilogue in the kernel, at the
    Llama-2-7B qkv (N = 12288) and gate/up (N = 22016) widths and 129..256 rows: row-scaled
    consumer and packed SwiGLU vs fp32."""
    monkeypatch.setattr(ops, "WIDE_ROWS", 256)
    monkeypatch.setattr(ops, "T2D_MIN", 257)
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(900 + M)
    K = 1024
    x = (torch.randn(M, K, device=dev, generator=g) * 0.7).to(torch.bfloat16)
    gw = (torch.rand(K, device=dev, generator=g) + 0.5).to(torch.bfloat16)
    ss = ops.norm_stats_buffer(dev)[0]
    res = torch.empty_like(x)
    xp = torch.zeros(ops.packed_numel(M, K), dtype=torch.bfloat16, device=dev)
    ops.rmsnorm(x, gw, EPS, out=xp, residual=res, mode=3, packed=True, ss=ss)
    xn = _rms_ref(x, gw).float()
    N = 12288
    w = (torch.randn(N, K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    wp = ops.pack_weight((w.float() * gw.float()[None, :]).to(torch.bfloat16).contiguous())
    y = ops.linear(xp, None, wp=wp, a_rows=M, ss_in=ss, eps=EPS)
    torch.testing.assert_close(y.float(), xn @ w.float().t(), atol=3e-2, rtol=3e-2)
    F = 11008
    wgu = (torch.randn(2 * F, K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    wgup = ops.pack_weight((wgu.float() * gw.float()[None, :]).to(torch.bfloat16).contiguous())
    act = torch.zeros(ops.packed_numel(M, F), dtype=torch.bfloat16, device=dev)
    ops.linear(xp, None, out=act, epilogue=1, wp=wgup, a_rows=M, out_packed=True, ss_in=ss, eps=EPS)
    exp = ref.swiglu((xn @ wgu.float().t()).to(torch.bfloat16)).float()
    torch.testing.assert_close(ref.unpack_act(act, M, F).float(), exp, atol=5e-2, rtol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("dims", [(2048, 2048, 2048), (4096, 12288, 11008), (4096, 6144, 14336)])
@pytest.mark.parametrize("gl", [False, True])
def test_t2d_consumers_and_producers(M, dims, gl, monkeypatch):
    """The two-dimensionally tiled kernel (csrc/gemm_t2d.h) at 129..256 rows, every decode
    epilogue against fp32 oracles: the row-scaled consumer (qkv), the row-scaled packed SwiGLU
    (gate/up: 12- and 10-tile column groups at F = 11008), the residual-stream producer straight
    from the accumulators (o) and as split-K slabs + the reduce launch (down, K = 11008); the
    Llama-3-8B widths (8-tile waves for gate/up); ``gl``: the LDS-DMA staging ring."""
    monkeypatch.setattr(ops, "T2D_MIN", 129)
    monkeypatch.setattr(ops, "T2D_GL", gl)
    dev = "cuda"
    H, Nq, F = dims
    g = torch.Generator(device=dev).manual_seed(1300 + M + H)
    for N, K, epi, pk in ((Nq, H, 0, False), (2 * F, H, 1, True), (H, H, 3, False), (H, F, 3, False)):
        assert ops.t2d_ok(M, N, K, epi, pk), (N, K, epi)
    x = (torch.randn(M, H, device=dev, generator=g) * 0.7).to(torch.bfloat16)
    gw = (torch.rand(H, device=dev, generator=g) + 0.5).to(torch.bfloat16)
    ss = ops.norm_stats_buffer(dev)[0] + 3
    res = torch.empty_like(x)
    xp = torch.zeros(ops.packed_numel(M, H), dtype=torch.bfloat16, device=dev)
    ops.rmsnorm(x, gw, EPS, out=xp, residual=res, mode=3, packed=True, ss=ss)
    xn = _rms_ref(x, gw).float()
    sd = 0.03 * (1024 / H) ** 0.5  # outputs of the size the K = 1024 tests above see
    w = (torch.randn(Nq, H, device=dev, generator=g) * sd).to(torch.bfloat16)
    wp = ops.pack_weight((w.float() * gw.float()[None, :]).to(torch.bfloat16).contiguous())
    y = ops.linear(xp, None, wp=wp, a_rows=M, ss_in=ss, eps=EPS)
    torch.testing.assert_close(y.float(), xn @ w.float().t(), atol=3e-2, rtol=3e-2)
    wgu = (torch.randn(2 * F, H, device=dev, generator=g) * sd).to(torch.bfloat16)
    wgup = ops.pack_weight((wgu.float() * gw.float()[None, :]).to(torch.bfloat16).contiguous())
    act = torch.zeros(ops.packed_numel(M, F), dtype=torch.bfloat16, device=dev)
    ops.linear(xp, None, out=act, epilogue=1, wp=wgup, a_rows=M, out_packed=True, ss_in=ss, eps=EPS)
    exp = ref.swiglu((xn @ wgu.float().t()).to(torch.bfloat16)).float()
    torch.testing.assert_close(ref.unpack_act(act, M, F).float(), exp, atol=5e-2, rtol=3e-2)
    for K in (H, F):  # o (direct producer epilogue), down (split-K slabs + reduce)
        a = (torch.randn(M, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        wo = (torch.randn(H, K, device=dev, generator=g) * 0.03 * (2048 / K) ** 0.5).to(torch.bfloat16)
        r = torch.randn(M, H, device=dev, generator=g).to(torch.bfloat16)
        r0 = r.clone()
        ap = torch.zeros(ops.packed_numel(M, H), dtype=torch.bfloat16, device=dev)
        sso, ssz = ops.norm_stats_buffer(dev)[0], ops.norm_stats_buffer(dev)[0] + 7
        ops.linear(ops.pack_act(a), None, out=r, epilogue=3, residual=r, wp=ops.pack_weight(wo), a_rows=M,
                   ap_out=ap, ss_out=sso, ss_zero=ssz)
        exp = (r0.float() + (a.float() @ wo.float().t()).to(torch.bfloat16).float()).to(torch.bfloat16)
        torch.testing.assert_close(r.float(), exp.float(), atol=2e-2, rtol=2e-2)
        assert torch.equal(ref.unpack_act(ap, M, H), r)
        assert torch.equal(sso.sum(0)[:M].cpu(), ref.fx_sumsq(r.cpu()))
        assert int(ssz.abs().sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("n", [100, 200])
@pytest.mark.parametrize("t2d", [False, True])
def test_fused_executor_wide_batch_matches_unfused(graphs, n, t2d, monkeypatch):
    """A 100- / 200-session decode step takes the fused-norm path (wide kernels; with ``t2d`` the
    two-dimensionally tiled kernel from 129 rows) and matches the unfused packed path step by step."""
    import dataclasses

    monkeypatch.setattr(ops, "WIDE_ROWS", 256)
    monkeypatch.setattr(ops, "T2D_MIN", 129 if t2d else 257)

    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor

    cfg = dataclasses.replace(resolve_model("small-llama"), hidden_size=2048, intermediate_size=4096,
                              num_attention_heads=16, num_key_value_heads=16, num_hidden_layers=2,
                              name="wide-test")

    def build(fused):
        monkeypatch.setenv("MPAMD_FUSED_NORM", "1" if fused else "0")
        w = random_stage_weights(cfg, 0, 2, has_embed=True, has_head=True, device="cuda", seed=5)
        for i, lay in enumerate(w.layers):
            gen = torch.Generator(device="cuda").manual_seed(70 + i)
            lay.input_norm = (torch.rand(cfg.hidden_size, device="cuda", generator=gen) + 0.5).to(torch.bfloat16)
            lay.post_norm = (torch.rand(cfg.hidden_size, device="cuda", generator=gen) + 0.5).to(torch.bfloat16)
        return StageExecutor(cfg, w, "cuda", kv_cache_bytes=512 << 20, max_sessions=256, max_seq_len=64,
                             use_graphs=graphs, graph_max_batch=256)

    fx, ux = build(True), build(False)
    assert fx._fused and fx._fused_wide_ok(n)
    gen = torch.Generator().manual_seed(9)
    lens = [int(x) for x in torch.randint(3, 12, (n,), generator=gen)]
    seqs = [(f"s{i}", L) for i, L in enumerate(lens)]
    ids = torch.randint(0, cfg.vocab_size, (sum(lens),), generator=gen).cuda()
    lf = fx.forward(seqs, ids, reset=[True] * n)
    lu = ux.forward(seqs, ids, reset=[True] * n)
    for _ in range(3):
        tok = torch.argmax(lu.float(), -1)
        lf = fx.forward([(s, 1) for s, _ in seqs], tok)
        lu = ux.forward([(s, 1) for s, _ in seqs], tok)
        torch.testing.assert_close(lf.float(), lu.float(), atol=0.08, rtol=0.05)


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True])
def test_fused_executor_matches_unfused_and_oracle(graphs, monkeypatch):
    from src.models.config import resolve_model
    from src.models.reference_model import reference_forward
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor

    cfg = resolve_model("small-llama")
    L = cfg.num_hidden_layers

    def build(fused):
        monkeypatch.setenv("MPAMD_FUSED_NORM", "1" if fused else "0")
        w = random_stage_weights(cfg, 0, L, has_embed=True, has_head=True, device="cuda", seed=21)
        for i, lay in enumerate(w.layers):  # non-trivial norm weights: folding must matter
            gen = torch.Generator(device="cuda").manual_seed(1000 + i)
            lay.input_norm = (torch.rand(cfg.hidden_size, device="cuda", generator=gen) + 0.5).to(torch.bfloat16)
            lay.post_norm = (torch.rand(cfg.hidden_size, device="cuda", generator=gen) + 0.5).to(torch.bfloat16)
        ex = StageExecutor(cfg, w, "cuda", kv_cache_bytes=128 << 20, max_sessions=8, max_seq_len=256,
                           use_graphs=graphs)
        assert ex._fused == fused
        return w, ex

    w, fx = build(True)
    _, ux = build(False)
    gen = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, cfg.vocab_size, (n,), generator=gen) for n in (23, 70, 5)]
    seqs = [("a", 23), ("b", 70), ("c", 5)]
    ids = torch.cat(prompts).cuda()
    lf = fx.forward(seqs, ids, reset=[True] * 3)
    lu = ux.forward(seqs, ids, reset=[True] * 3)
    cur = [p.clone() for p in prompts]
    for step in range(4):
        tok = torch.argmax(lu.float(), -1)
        cur = [torch.cat([c, tok[i:i + 1].cpu()]) for i, c in enumerate(cur)]
        lf = fx.forward([(s, 1) for s, _ in seqs], tok)
        lu = ux.forward([(s, 1) for s, _ in seqs], tok)
        torch.testing.assert_close(lf.float(), lu.float(), atol=0.08, rtol=0.05)
        for i in range(3):
            r = reference_forward([w], cur[i].cuda())[-1]
            torch.testing.assert_close(lf[i].float(), r, atol=0.08, rtol=0.05)


@pytest.mark.gpu
@pytest.mark.parametrize("T,H", [(1, 4096), (37, 4096), (64, 8192)])
def test_embed_stage_entry_matches_embedding_then_mode3(T, H):
    """The first stage's fused entry (embedding rows gathered by the mode-3 kernel) == embedding, then
    rmsnorm mode 3: same residual rows, same packed rows, same fixed-point row statistics (bit for
    bit); an out-of-range id reads row 0 in both."""
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(T)
    V = 1000
    table = torch.randn(V, H, device=dev, generator=g).to(torch.bfloat16)
    ids = torch.randint(0, V, (T,), device=dev, generator=g)
    if T > 1:
        ids[-1] = V + 5
    h = ops.embedding(ids, table)
    res1, res2 = torch.empty(T, H, dtype=torch.bfloat16, device=dev), torch.empty(T, H, dtype=torch.bfloat16, device=dev)
    xp1 = torch.zeros(ops.packed_numel(T, H), dtype=torch.bfloat16, device=dev)
    xp2 = torch.zeros_like(xp1)
    ss1, ss2 = ops.norm_stats_buffer(dev, 2)
    ss1.fill_(7)
    ss2.fill_(9)
    ops.rmsnorm(h, table[0], EPS, out=xp1, residual=res1, mode=3, packed=True, ss=ss1)
    ops.embed_stage_entry(ids, table, xp2, res2, ss2)
    assert torch.equal(res1, res2) and torch.equal(xp1, xp2)
    assert torch.equal(ss1.view(-1, 256)[:, :T], ss2.view(-1, 256)[:, :T])
