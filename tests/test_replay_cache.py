"""Stage-local recovery building blocks (CPU): the per-stage replay cache of output rows
(``parallel.engine.ReplayCache``) and session adoption by rename (``SessionManager.rename``)."""
import numpy as np
import pytest
import torch

from src.parallel.engine import ReplayCache
from src.runtime.kv_cache import PagedKVCache
from src.runtime.session import SessionManager


def test_replay_cache_stores_rows_by_handle_and_position():
    rc = ReplayCache(max_handles=4, max_len=8, hidden=3, dtype=torch.float32, device="cpu")
    # a step: handle 2 prefills 3 tokens from position 0, handle 0 decodes 1 token at position 5
    out = torch.arange(12, dtype=torch.float32).view(4, 3)
    rc.store([(2, 3, 0, 0, 0), (0, 1, 5, 0, 0)], out)
    assert torch.equal(rc.rows(2, 3), out[:3])
    assert torch.equal(rc.buf[0 * 8 + 5], out[3])
    # a later step appends at positions 3, 4 of handle 2; rows past max_len are dropped, not wrapped
    rc.store([(2, 2, 3, 0, 0), (1, 3, 6, 0, 0)], torch.ones(5, 3))
    assert torch.equal(rc.rows(2, 5)[3:], torch.ones(2, 3))
    assert torch.equal(rc.buf[1 * 8 + 6:1 * 8 + 8], torch.ones(2, 3))
    assert torch.equal(rc.buf[2 * 8], out[0])  # handle 1's overflow did not reach handle 2


def test_session_rename_moves_kv_and_closes_target():
    cache = PagedKVCache(num_layers=1, num_pages=16, page_size=4, num_kv_heads=1, head_dim=8,
                         dtype=torch.float32, device="cpu")
    sm = SessionManager(cache, max_sessions=4, max_seq_len=32)
    s = sm.open("chan-a:3")
    sm.reserve(s, 10)
    s.length = 10
    pages = list(s.pages)
    other = sm.open("chan-b:0")
    sm.reserve(other, 4)
    free0 = sm.free_pages
    moved = sm.rename("chan-a:3", "chan-b:0")
    assert moved is s and moved.sid == "chan-b:0" and moved.pages == pages and moved.length == 10
    assert "chan-a:3" not in sm.sessions and sm.get("chan-b:0") is s
    assert sm.free_pages == free0 + 1  # the replaced target's page went back
    assert sm.rename("missing", "x") is None
    assert int(np.sum(sm.table[s.row] >= 0)) == len(pages)


@pytest.mark.gpu
def test_replay_cache_on_gpu_pinned_staging():
    """The device path: row indices staged through the double-buffered pinned area (no host block),
    many steps in a row so both staging buffers are reused."""
    rc = ReplayCache(max_handles=8, max_len=64, hidden=16, dtype=torch.bfloat16, device="cuda")
    ref = torch.zeros(8 * 64, 16, dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(0)
    for step in range(40):
        recs = [(h, 1, step, 0, 0) for h in range(8)]
        out = torch.randn(8, 16, generator=g).to(torch.bfloat16)
        rc.store(recs, out.cuda())
        for h in range(8):
            ref[h * 64 + step] = out[h]
    torch.cuda.synchronize()
    assert torch.equal(rc.buf.cpu(), ref)
    assert torch.equal(rc.rows(3, 40).cpu(), ref[3 * 64: 3 * 64 + 40])


def test_failed_channel_replay_caches_bounded_by_age_and_bytes():
    """two client pipelines failing close together both keep their replay rows (the
    handler used to keep only the newest); caches past the age or byte budget are dropped, oldest
    first."""
    import types

    from src.rpc_handler import StageConnectionHandler

    def eng(failed_at, nbytes):
        rc = types.SimpleNamespace(buf=torch.zeros(nbytes // 4, dtype=torch.float32))
        return types.SimpleNamespace(failed="peer died", failed_at=failed_at, replay=rc)

    h = types.SimpleNamespace(replay_keep_s=300.0, replay_keep_bytes=1000,
                              _chan_engines={"a": eng(100.0, 400), "b": eng(110.0, 400), "c": eng(120.0, 400),
                                             "old": eng(-500.0, 4), "live": types.SimpleNamespace(failed=None)})
    StageConnectionHandler._prune_failed_channels(h, now=130.0)
    assert set(h._chan_engines) == {"b", "c", "live"}  # newest two fit 1000 bytes; "a" over budget, "old" aged
