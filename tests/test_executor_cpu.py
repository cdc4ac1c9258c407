"""Stage executor on the CPU data path vs the dense fp32 oracle; sessions, paging, ragged batches."""
import pytest
import torch

from src import native, ops
from src.models.config import resolve_model
from src.models.reference_model import reference_forward
from src.models.weights import interleave_gate_up, random_stage_weights, split_gate_up
from src.runtime.executor import StageExecutor
from src.runtime.kv_cache import AllocationFailed, PageAllocator


def _ex(model="tiny-llama", start=0, end=None, embed=True, head=True, dtype=torch.float32, **kw):
    cfg = resolve_model(model)
    end = cfg.num_hidden_layers if end is None else end
    w = random_stage_weights(cfg, start, end, has_embed=embed, has_head=head, device="cpu", dtype=dtype, seed=7)
    kw.setdefault("kv_cache_bytes", 32 << 20)
    kw.setdefault("max_sessions", 8)
    kw.setdefault("max_seq_len", 256)
    return cfg, w, StageExecutor(cfg, w, "cpu", dtype=dtype, **kw)


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-gpt2"])
def test_prefill_decode_matches_reference(model):
    cfg, w, ex = _ex(model)
    g = torch.Generator().manual_seed(0)
    a = torch.randint(0, cfg.vocab_size, (13,), generator=g)
    b = torch.randint(0, cfg.vocab_size, (70,), generator=g)  # crosses a 64-token page
    lg = ex.forward([("a", 13), ("b", 70)], torch.cat([a, b]))
    torch.testing.assert_close(lg[0], reference_forward([w], a)[-1], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(lg[1], reference_forward([w], b)[-1], atol=1e-4, rtol=1e-4)
    seqs = [a, b]
    for _ in range(3):
        nxt = torch.argmax(lg, -1)
        seqs = [torch.cat([s, nxt[i:i + 1]]) for i, s in enumerate(seqs)]
        lg = ex.forward([("a", 1), ("b", 1)], nxt)
        for i in range(2):
            torch.testing.assert_close(lg[i], reference_forward([w], seqs[i])[-1], atol=1e-4, rtol=1e-4)


def test_chunked_prefill_equals_one_shot():
    cfg, w, ex = _ex()
    ids = torch.arange(50) % cfg.vocab_size
    one = ex.forward([("x", 50)], ids)
    ex.forward([("y", 20)], ids[:20])
    two = ex.forward([("y", 30)], ids[20:])
    torch.testing.assert_close(one, two, atol=1e-5, rtol=1e-5)


def test_stage_split_equals_full():
    cfg, w, full = _ex()
    _, _, s0 = _ex(start=0, end=2, head=False)
    _, _, s1 = _ex(start=2, embed=False)
    ids = torch.arange(30) % cfg.vocab_size
    torch.testing.assert_close(full.forward([("s", 30)], ids), s1.forward([("s", 30)], s0.forward([("s", 30)], ids)))


def test_rewind_is_idempotent_and_reset():
    cfg, w, ex = _ex()
    ids = torch.arange(10)
    ex.forward([("s", 10)], ids)
    a = ex.forward([("s", 1)], torch.tensor([5]))
    b = ex.forward([("s", 1)], torch.tensor([5]), starts=[10])  # retried step overwrites its slot
    torch.testing.assert_close(a, b)
    assert ex.sessions.get("s").length == 11
    c = ex.forward([("s", 10)], ids, reset=[True])
    d = ex.forward([("t", 10)], ids)
    torch.testing.assert_close(c, d)


def test_session_limits_and_eviction():
    cfg, w, ex = _ex(max_sessions=2, max_seq_len=128)
    ex.forward([("a", 4)], torch.arange(4))
    ex.forward([("b", 4)], torch.arange(4))
    with pytest.raises(AllocationFailed):
        ex.forward([("c", 4)], torch.arange(4))
    ex.sessions.close("a")
    ex.forward([("c", 4)], torch.arange(4))
    with pytest.raises(ValueError):
        ex.forward([("b", 200)], torch.arange(200) % cfg.vocab_size)  # > max_seq_len
    ex.sessions.ttl = 0.0
    assert ex.sessions.evict_expired() == 2
    assert ex.sessions.free_pages == ex.cache.num_pages


def test_page_allocator_native_and_double_free():
    a = PageAllocator(8)
    p = a.alloc(5)
    assert len(set(p)) == 5 and a.free_pages == 3
    with pytest.raises(AllocationFailed):
        a.alloc(4)
    a.free(p[:2])
    with pytest.raises(Exception):
        a.free(p[:1])
    assert native.BACKEND in ("native", "python")


def test_packed_layouts_cpu_roundtrip():
    x = torch.randn(37, 256)
    assert torch.equal(ops.unpack_act(ops.pack_act(x), 37, 256), x)
    w = torch.randn(64, 128)
    assert torch.equal(ops.unpack_weight(ops.pack_weight(w)), w)
    g, u = torch.randn(32, 8), torch.randn(32, 8)
    g2, u2 = split_gate_up(interleave_gate_up(g, u))
    assert torch.equal(g, g2) and torch.equal(u, u2)
    y = ops.linear(ops.pack_act(x[:, :128]), None, wp=ops.pack_weight(w), a_rows=37)
    torch.testing.assert_close(y, x[:, :128] @ w.t())


def test_chunked_prefill_matches_single_step():
    """A prompt longer than max_tokens_per_step runs as chunks with identical results."""
    import torch

    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor

    cfg = resolve_model("tiny-llama")
    for head in (True, False):
        w = random_stage_weights(cfg, 0, 2, has_embed=True, has_head=head, device="cpu", dtype=torch.float32)
        big = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=4,
                            max_seq_len=128, max_tokens_per_step=64)
        small = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=4,
                              max_seq_len=128, max_tokens_per_step=7)
        g = torch.Generator().manual_seed(4)
        ids = torch.randint(0, cfg.vocab_size, (20 + 9,), generator=g)
        seqs = [("a", 20), ("b", 9)]
        ref = big.forward(seqs, ids, reset=[True, True])
        got = small.forward(seqs, ids, reset=[True, True])
        torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)
        assert small.sessions.get("a").length == 20 and small.sessions.get("b").length == 9
        # decode continues on the chunk-written KV
        nxt = torch.tensor([3, 5])
        torch.testing.assert_close(small.forward([("a", 1), ("b", 1)], nxt), big.forward([("a", 1), ("b", 1)], nxt),
                                   atol=1e-4, rtol=1e-4)


def test_session_fork_and_beam_reorder():
    import torch

    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor

    cfg = resolve_model("tiny-llama")
    w = random_stage_weights(cfg, 0, 4, has_embed=True, has_head=True, device="cpu", dtype=torch.float32)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=8, max_seq_len=128)
    ids = torch.randint(0, cfg.vocab_size, (11,), generator=torch.Generator().manual_seed(2))
    ex.forward([("a", 11)], ids, reset=[True])
    ex.forward([("b", 5)], ids[:5], reset=[True])
    ex.sessions.fork("a", "c")
    assert ex.sessions.get("c").length == 11
    la = ex.forward([("a", 1)], torch.tensor([7]))
    lc = ex.forward([("c", 1)], torch.tensor([7]))
    torch.testing.assert_close(la, lc)
    # beam reorder: hypothesis "a" continues from old "b" and "b" from old "a"
    ex.forward([("a", 1), ("b", 1)], torch.tensor([3, 4]))
    ex.sessions.fork("a", "a_old")
    ex.sessions.fork("b", "b_old")
    ex.sessions.reorder(["a", "b"], [1, 0])
    assert ex.sessions.get("a").length == 6 and ex.sessions.get("b").length == 13
    torch.testing.assert_close(ex.forward([("b", 1)], torch.tensor([9])), ex.forward([("a_old", 1)], torch.tensor([9])))
    torch.testing.assert_close(ex.forward([("a", 1)], torch.tensor([8])), ex.forward([("b_old", 1)], torch.tensor([8])))
    assert not any(k.startswith("__reorder") for k in ex.sessions.sessions)
