"""``PipelineServingEngine._settle_heap``: the setup heap is collected and frozen exactly once per
engine before its first step (``MPAMD_GC_FREEZE=0`` keeps the default collector)."""
import gc

from src.parallel import engine as engmod


class _Probe(engmod.PipelineServingEngine):
    def __init__(self):  # no channel / executor: only the heap hook is exercised
        pass


def test_freeze_once(monkeypatch):
    calls = []
    monkeypatch.setattr(gc, "freeze", lambda: calls.append("freeze"))
    monkeypatch.setattr(gc, "collect", lambda *a: calls.append("collect") or 0)
    monkeypatch.delenv("MPAMD_GC_FREEZE", raising=False)
    e = _Probe()
    e._settle_heap()
    e._settle_heap()
    assert calls == ["collect", "freeze"]
    _Probe()._settle_heap()  # a second engine settles its own (larger) heap
    assert calls == ["collect", "freeze"] * 2


def test_freeze_disabled(monkeypatch):
    calls = []
    monkeypatch.setattr(gc, "freeze", lambda: calls.append("freeze"))
    monkeypatch.setenv("MPAMD_GC_FREEZE", "0")
    _Probe()._settle_heap()
    assert calls == []
