"""Cost-balanced pipeline splits (``partition.balanced_splits`` / ``resolve_splits``, ``--splits
auto:N``): the dynamic programme is optimal (brute force over every contiguous layout), the
tail's lm_head + sampler and the head's embedding land where the model says, and the CLI
resolves ``auto:N`` identically in every process."""
import itertools

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from src.models.config import resolve_model
from src.partition import (balanced_splits, even_splits, resolve_splits, stage_cost_model, stage_ranges,
                           stage_times)


def _brute(L, S, blk, head, tail):
    """(max, sum of squares) of the best layout over every choice of S-1 cuts."""
    best = None
    for cuts in itertools.combinations(range(1, L), S - 1):
        rng = stage_ranges(cuts, L)
        c = [(e - s) * blk + (head if k == 0 else 0) + (tail if k == S - 1 else 0) for k, (s, e) in enumerate(rng)]
        key = (max(c), sum(x * x for x in c))
        if best is None or key[0] < best[0] - 1e-12 or (abs(key[0] - best[0]) <= 1e-12 and key[1] < best[1]):
            best = key
    return best


@settings(max_examples=60, deadline=None)
@given(L=st.integers(2, 12), S=st.integers(1, 4), tail_blocks=st.floats(0.0, 4.0), head_blocks=st.floats(0.0, 1.0))
def test_dp_matches_brute_force(L, S, tail_blocks, head_blocks):
    if S > L:
        return
    cfg = resolve_model("llama2-7b")
    blk = 1.0
    import src.partition as part

    orig = part.stage_cost_model
    part.stage_cost_model = lambda *a, **k: (blk, head_blocks, tail_blocks)
    try:
        cuts = balanced_splits(cfg, S, num_layers=L)
    finally:
        part.stage_cost_model = orig
    assert len(cuts) == S - 1
    rng = stage_ranges(cuts, L)
    c = [(e - s) * blk + (head_blocks if k == 0 else 0) + (tail_blocks if k == S - 1 else 0)
         for k, (s, e) in enumerate(rng)]
    if S == 1:
        return
    bm, bs = _brute(L, S, blk, head_blocks, tail_blocks)
    assert max(c) == pytest.approx(bm, abs=1e-9)
    assert sum(x * x for x in c) == pytest.approx(bs, abs=1e-6)


def test_tail_gets_fewer_blocks():
    """The tail carries lm_head + sampler: it never holds more blocks than any other stage."""
    for name, fp8 in (("llama2-7b", False), ("llama3-8b", False), ("llama3-70b", True)):
        cfg = resolve_model(name)
        for S in (2, 4, 8):
            rng = stage_ranges(balanced_splits(cfg, S, fp8=fp8), cfg.num_hidden_layers)
            sizes = [e - s for s, e in rng]
            assert sizes[-1] == min(sizes), (name, S, sizes)
            assert sum(sizes) == cfg.num_hidden_layers


def test_70b_fp8_pp8_is_near_even_in_time():
    """Llama-3-70B fp8 on 8 stages: the modelled slowest stage is within 8 % of the mean (the even
    10-block split puts the bf16 lm_head on top of the tail's blocks: ~20 % over)."""
    cfg = resolve_model("llama3-70b")
    cuts = balanced_splits(cfg, 8, fp8=True)
    t = stage_times(cfg, cuts, fp8=True)
    assert max(t) / (sum(t) / len(t)) <= 1.08
    te = stage_times(cfg, even_splits(80, 8), fp8=True)
    assert max(te) / (sum(te) / len(te)) > max(t) / (sum(t) / len(t))


def test_fp8_block_cost_is_lower():
    cfg = resolve_model("llama3-70b")
    b16 = stage_cost_model(cfg)[0]
    b8 = stage_cost_model(cfg, fp8=True)[0]
    assert b8 < 0.7 * b16


def test_resolve_splits_forms():
    cfg = resolve_model("llama2-7b")
    assert resolve_splits("8,16,24", cfg) == [8, 16, 24]
    assert resolve_splits("8,16,32", cfg) == [8, 16]  # trailing cut == L dropped
    assert resolve_splits("auto:4", cfg) == balanced_splits(cfg, 4)
    assert resolve_splits("auto:1", cfg) == []
    with pytest.raises(ValueError):
        resolve_splits("auto", cfg)
    with pytest.raises(ValueError):
        resolve_splits("auto:64", cfg)


def test_cli_accepts_auto_splits(monkeypatch):
    """``python -m src.main --splits auto:N``: the CLI resolves the cuts before dispatching."""
    from src import main as cli

    seen = {}
    monkeypatch.setattr(cli, "run_stage_server", lambda args, device, cuts: seen.setdefault("cuts", cuts))
    cli.main(["--model", "llama2-7b", "--splits", "auto:4", "--stage", "1", "--device", "cpu"])
    assert seen["cuts"] == balanced_splits(resolve_model("llama2-7b"), 4)
    with pytest.raises(SystemExit):
        cli.main(["--model", "llama2-7b", "--splits", "auto", "--stage", "1", "--device", "cpu"])
