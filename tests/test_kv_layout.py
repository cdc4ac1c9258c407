"""KV export/import between the paged cache and dense LLaMA/BLOOM layouts (petals/llama/block.py:306-326)."""
import pytest
import torch

from src.models.config import resolve_model
from src.models.weights import random_stage_weights
from src.runtime.executor import StageExecutor
from src.runtime.kv_layout import bloom_to_llama, export_session_kv, import_session_kv, llama_to_bloom


def test_bloom_llama_roundtrip():
    k, v = torch.randn(3, 2, 7, 16), torch.randn(3, 2, 7, 16)
    bk, bv = llama_to_bloom(k, v)
    assert bk.shape == (6, 16, 7) and bv.shape == (6, 7, 16)
    assert torch.equal(bk[1 * 2 + 1, :, 4], k[1, 1, 4]) and torch.equal(bv[5, 3], v[2, 1, 3])
    k2, v2 = bloom_to_llama(bk, bv, 3)
    assert torch.equal(k2, k) and torch.equal(v2, v)


def test_export_import_migrates_a_session():
    cfg = resolve_model("tiny-llama")
    w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cpu",
                             dtype=torch.float32, seed=1)
    kw = dict(kv_cache_bytes=8 << 20, max_sessions=4, max_seq_len=256)
    src = StageExecutor(cfg, w, "cpu", dtype=torch.float32, **kw)
    dst = StageExecutor(cfg, w, "cpu", dtype=torch.float32, **kw)
    ids = torch.randint(0, cfg.vocab_size, (70,), generator=torch.Generator().manual_seed(0))  # 2 pages
    src.forward([("a", 70)], ids, reset=[True])
    kv = export_session_kv(src.cache, src.sessions.get("a"))
    assert len(kv) == cfg.num_hidden_layers
    assert kv[0][0].shape == (1, cfg.num_key_value_heads, 70, cfg.head_dim)
    # a later position must not leak into the export of a shorter prefix
    part = export_session_kv(src.cache, src.sessions.get("a"), layers=[1], length=65)
    torch.testing.assert_close(part[0][1], kv[1][1][:, :, :65])
    import_session_kv(dst.sessions, "b", kv)
    assert dst.sessions.get("b").length == 70
    tok = torch.tensor([5])
    torch.testing.assert_close(dst.forward([("b", 1)], tok), src.forward([("a", 1)], tok))
    with pytest.raises(ValueError):
        export_session_kv(src.cache, src.sessions.get("a"), length=500)
