"""fp8 (OCP e4m3fn) W8A8 path: packing/quantization references on CPU, executor on CPU."""
import torch

from src import ops
from src.models.config import resolve_model
from src.models.reference_model import greedy_generate
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
