"""roctx ranges + phase timer (SURVEY §5 tracing)."""
from src.utils import tracing


def test_phase_timer_and_ranges():
    t = tracing.PhaseTimer()
    tracing.enable(True)
    try:
        for _ in range(3):
            with t("decode"):
                tracing.mark("tick")
        with t("prefill", trace=False):
            pass
    finally:
        tracing.enable(False)
    s = t.summary()
    assert s["decode"]["count"] == 3 and s["prefill"]["count"] == 1
    assert s["decode"]["max_s"] >= 0 and "mean_ms" in s["decode"]
    assert list(t.summary("pre")) == ["prefill"]
    t.reset()
    assert t.summary() == {}
    assert isinstance(tracing.available(), bool)
