"""fp8 (OCP e4m3fn) W8A8 path: packing/quantization references on CPU, executor on CPU."""
import pytest
import torch

from src import ops
from src.models.config import resolve_model
from src.models.reference_model import greedy_generate, reference_forward
from src.models.weights import random_stage_weights
from src.ops import reference as ref
from src.runtime.executor import StageExecutor


def test_fp8_weight_pack_roundtrip():
    torch.manual_seed(0)
    w = torch.randn(96, 512) * 0.02
    w[3] = 0  # zero row keeps a finite scale
    q, s = ops.pack_weight_fp8(w)
    assert q.shape == (6, 8, 64, 16) and q.dtype == torch.uint8 and s.shape == (96,)
    wd = ops.unpack_weight_fp8(q, s, torch.float32)
    assert torch.isfinite(wd).all() and float(wd[3].abs().max()) == 0.0
    rel = (wd - w).norm() / w.norm()
    assert rel < 0.04
    # per-row absmax maps exactly onto the fp8 max
    assert torch.allclose(wd.abs().amax(1)[s > 1e-20], w.abs().amax(1)[s > 1e-20], rtol=1e-6)
    q2, s2 = ops.pack_weight_fp8(wd)  # quantizing the dequantized weight is a fixed point
    assert torch.equal(q2, q)


def test_fp8_activation_quant_and_gemm_reference():
    torch.manual_seed(1)
    M, K, N = 21, 512, 64
    x = torch.randn(M, K).bfloat16()
    a8, s = ops.quant_act_fp8(ref.pack_act(x), M, K)
    assert s.numel() == 32 and a8.numel() == 32 * K
    xd = ref.dequant_act_fp8(a8, s, M, K)
    assert ((xd - x.float()).norm() / x.float().norm()) < 0.04
    w = torch.randn(N, K) * 0.02
    wq, ws = ops.pack_weight_fp8(w)
    y = ops.linear_fp8(a8, s, wq, ws, M)
    exact = xd @ ops.unpack_weight_fp8(wq, ws, torch.float32).t()
    torch.testing.assert_close(y.float(), exact, atol=2e-3, rtol=1e-2)


def test_fp8_stage_executor_matches_dequantized_reference():
    cfg = resolve_model("small-llama")
    w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cpu",
                             dtype=torch.float32)
    w.quantize_fp8(drop_dense=True)
    assert w.fp8 and w.layers[0].qkv is None
    # the oracle runs on the dequantized weights
    wd = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cpu",
                              dtype=torch.float32)
    for L, Ld in zip(w.layers, wd.layers):
        for name in L.PROJ:
            setattr(Ld, name, L.dense(name, torch.float32))
    ids = torch.randint(0, cfg.vocab_size, (12,), generator=torch.Generator().manual_seed(3))
    want = greedy_generate([wd], ids, 6)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=16 << 20, max_sessions=2, max_seq_len=64)
    logits = ex.forward([("s", len(ids))], ids, reset=[True])
    got = [int(torch.argmax(logits[-1]))]
    for _ in range(5):
        logits = ex.forward([("s", 1)], torch.tensor([got[-1]]))
        got.append(int(torch.argmax(logits[-1])))
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 17, 64])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_rmsnorm_fp8_output_equals_norm_then_quant(M, mode):
    """norm.hip a8 output (the fp8 path's norm sites) == bf16 packed norm + quant_act_fp8, bit for
    bit: same per-row absmax / 448 scale, same e4m3 bytes in the fp8 GEMM's A layout."""
    from src import ops

    H = 1024
    g = torch.Generator(device="cuda").manual_seed(M + 10 * mode)
    x = (torch.randn(M, H, device="cuda", generator=g) * 2).to(torch.bfloat16)
    w = (torch.rand(H, device="cuda", generator=g) + 0.5).to(torch.bfloat16)
    res0 = (torch.randn(M, H, device="cuda", generator=g)).to(torch.bfloat16)
    r1, r2 = res0.clone(), res0.clone()
    xp = torch.zeros(ops.packed_numel(M, H), dtype=torch.bfloat16, device="cuda")
    ops.rmsnorm(x, w, 1e-5, out=xp, residual=r1, mode=mode, packed=True)
    a8_ref, s_ref = ops.quant_act_fp8(xp, M, H)
    a8 = torch.zeros(ops.packed_numel(M, H), dtype=torch.uint8, device="cuda")
    sc = torch.zeros(((M + 15) // 16) * 16, dtype=torch.float32, device="cuda")
    ops.rmsnorm(x, w, 1e-5, out=xp, residual=r2, mode=mode, packed=True, a8=a8, a8_scale=sc)
    assert torch.equal(r1, r2)
    assert torch.equal(sc[:M], s_ref[:M])
    # compare the valid rows' bytes (padding rows of the last 16-row tile are don't-care)
    ar = ops.reference.dequant_act_fp8(a8_ref, s_ref, M, H)
    an = ops.reference.dequant_act_fp8(a8, sc, M, H)
    assert torch.equal(ar, an)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["w8a8", "w8a16"])
@pytest.mark.parametrize("graphs", [False, True])
def test_fp8_executor_gpu_decode_tracks_dequantized_oracle(graphs, mode, monkeypatch):
    """The GPU fp8 decode paths stay within the fp8 error budget of the fp32 oracle on the
    dequantized weights, with and without hipGraphs (which must agree bit for bit):
    w8a8 - norm-emitted fp8, row-major attention / SwiGLU outputs through the row quantization
    kernel, fp8 MFMA GEMMs; w8a16 - the fused-norm path with fp8 weights dequantized into the
    bf16 MFMA (norm weights folded into qkv / gate_up and re-quantized: non-unit norms here)."""
    monkeypatch.setenv("MPAMD_FP8_MODE", mode)
    cfg = resolve_model("small-llama")
    L = cfg.num_hidden_layers
    w = random_stage_weights(cfg, 0, L, has_embed=True, has_head=True, device="cuda", seed=5)
    wd = random_stage_weights(cfg, 0, L, has_embed=True, has_head=True, device="cuda", seed=5, dtype=torch.float32)
    w.quantize_fp8(drop_dense=True)
    gn = torch.Generator(device="cuda").manual_seed(11)
    for Lq, Ld in zip(w.layers, wd.layers):
        for name in Lq.PROJ:
            setattr(Ld, name, Lq.dense(name, torch.float32))
        for nm in ("input_norm", "post_norm"):
            g = (0.5 + torch.rand(cfg.hidden_size, device="cuda", generator=gn)).to(torch.bfloat16)
            setattr(Lq, nm, g)
            setattr(Ld, nm, g.float())
    gen = torch.Generator().manual_seed(7)
    outs = {}
    for g in sorted({False, graphs}):
        ex = StageExecutor(cfg, w, "cuda", kv_cache_bytes=64 << 20, max_sessions=32, max_seq_len=128, use_graphs=g)
        if mode == "w8a8":
            assert ex._fp8_ok(17) and not ex._w8
        else:
            assert ex._w8 and ex._fused and not ex._fp8_ok(17)
        n = 17
        prompts = [torch.randint(0, cfg.vocab_size, (5 + i % 7,), generator=torch.Generator().manual_seed(i))
                   for i in range(n)]
        seqs = [(f"s{i}", len(p)) for i, p in enumerate(prompts)]
        ex.forward(seqs, torch.cat(prompts).cuda(), reset=[True] * n)
        cur = [p.clone() for p in prompts]
        steps = []
        for _ in range(3):
            tok = torch.tensor([int(c[-1]) * 7 % cfg.vocab_size for c in cur])
            cur = [torch.cat([c, tok[i:i + 1]]) for i, c in enumerate(cur)]
            steps.append(ex.forward([(s, 1) for s, _ in seqs], tok.cuda()).float())
        outs[g] = (steps, cur)
    steps, cur = outs[graphs]
    if graphs:
        for a, b in zip(outs[False][0], steps):
            assert torch.equal(a, b)
    for i in (0, 5, 16):
        ref_logits = reference_forward([wd], cur[i].cuda())[-1].float()
        got = steps[-1][i]
        cos = torch.nn.functional.cosine_similarity(got, ref_logits, dim=0)
        assert float(cos) > 0.99, (i, float(cos))
