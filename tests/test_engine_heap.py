"""Heap freeze and graph-hook hygiene of ``PipelineServingEngine``.

* ``settle_heap``: the setup heap is collected and frozen at most once per PROCESS, and only by
  driver engines (``freeze_heap``: bench.py, the CLI client); server engines built per client
  channel never freeze, so opening and closing many channels does not grow the permanent
  generation.
* graph hook: one owner at a time on an executor; ``release`` (stop / failure / end of serve)
  removes the owner's hook."""
import gc

import pytest

from src.parallel import engine as engmod


class _Probe(engmod.PipelineServingEngine):
    def __init__(self, ex=None, freeze=False):  # no channel: only the driving hooks are exercised
        self.ex = ex
        self.freeze_heap = freeze


@pytest.fixture
def fresh(monkeypatch):
    calls = []
    monkeypatch.setattr(engmod, "_HEAP_FROZEN", False)
    monkeypatch.setattr(gc, "freeze", lambda: calls.append("freeze"))
    monkeypatch.setattr(gc, "collect", lambda *a: calls.append("collect") or 0)
    return calls


def test_driver_freezes_once_per_process(fresh):
    e = _Probe(freeze=True)
    e._settle_heap()
    e._settle_heap()
    _Probe(freeze=True)._settle_heap()  # a second driver engine in the same process: no new freeze
    assert fresh == ["collect", "freeze"]


def test_server_engines_never_freeze(fresh):
    for _ in range(5):  # one engine per client channel
        _Probe(freeze=False)._settle_heap()
    assert fresh == []


def test_real_freeze_count_does_not_grow_with_channels():
    before = gc.get_freeze_count()
    for _ in range(3):
        _Probe(freeze=False)._settle_heap()
    assert gc.get_freeze_count() == before


def test_graph_hook_single_owner_and_release():
    import torch

    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor

    cfg = resolve_model("tiny-llama")
    w = random_stage_weights(cfg, 0, 2, has_embed=True, has_head=False, device="cpu", dtype=torch.float32)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=4, max_seq_len=64)
    a, b = _Probe(ex), _Probe(ex)
    assert ex.graph_hook_free(a) and ex.graph_hook_free(b)
    ex.set_graph_hook(lambda out: None, owner=a)
    assert ex.graph_hook_free(a) and not ex.graph_hook_free(b)
    with pytest.raises(RuntimeError):
        ex.set_graph_hook(lambda out: None, owner=b)
    b.release()  # not the owner: no-op
    assert ex.graph_hook is not None
    a.release()
    assert ex.graph_hook is None and ex.graph_hook_free(b)
    # a step with a stale owner runs normally and records nothing
    out = ex.forward([("s", 3)], torch.arange(3), hook_owner=a)
    assert out.shape[0] == 3 and not ex.last_hooked
