"""Split semantics and load-balancing algorithms (reference src/load_balancing.py semantics)."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from src.load_balancing import (RemoteModuleInfo, ServerInfo, ServerState, _choose_best_start, choose_best_blocks,
                                compute_spans, compute_throughputs, should_choose_other_blocks)
from src.partition import even_splits, parse_splits, stage_ranges


def test_parse_splits_and_ranges():
    assert parse_splits("10,20,30", 32) == [10, 20, 30]
    assert stage_ranges([10, 20, 30], 32) == [(0, 10), (10, 20), (20, 30), (30, 32)]
    assert parse_splits("6,12", 12) == [6]  # trailing cut == L is allowed and dropped
    assert stage_ranges([6], 12) == [(0, 6), (6, 12)]
    for bad in ("0,5", "5,5", "7,3", "40"):
        with pytest.raises(ValueError):
            parse_splits(bad, 32)


@given(st.integers(1, 96), st.integers(1, 16))
def test_even_splits_cover(L, n):
    if n > L:
        with pytest.raises(ValueError):
            even_splits(L, n)
        return
    rng = stage_ranges(even_splits(L, n), L)
    assert len(rng) == n and rng[0][0] == 0 and rng[-1][1] == L
    sizes = [e - s for s, e in rng]
    assert max(sizes) - min(sizes) <= 1


def _infos(spans):
    """spans: list of (peer, start, end, thr)"""
    out = []
    for pid, s, e, thr in spans:
        si = ServerInfo(pid, ServerState.ONLINE, thr, s, e)
        out += [RemoteModuleInfo(f"block_{b}", si) for b in range(s, e)]
    return out


def test_compute_spans_and_throughputs():
    infos = _infos([("a", 0, 4, 2.0), ("b", 2, 6, 3.0)])
    sp = compute_spans(infos)
    assert (sp["a"].start, sp["a"].end, sp["b"].start, sp["b"].end) == (0, 4, 2, 6)
    thr = compute_throughputs(sp, 8)
    assert thr.tolist() == [2, 2, 5, 5, 3, 3, 0, 0]
    # a gap: the peer's last contiguous run is its span
    si = ServerInfo("c", ServerState.ONLINE, 1.0, 0, 8)
    sp2 = compute_spans([RemoteModuleInfo(f"block_{b}", si) for b in (0, 1, 5, 6)])
    assert (sp2["c"].start, sp2["c"].end) == (5, 7)
    # OFFLINE servers are not counted with the default JOINING floor? (OFFLINE ranks above JOINING: counted)
    assert compute_spans(infos, ServerState.OFFLINE) == {}


def test_choose_best_blocks_fills_weakest_region():
    infos = _infos([("a", 8, 16, 5.0), ("b", 16, 24, 5.0)])
    assert choose_best_blocks(4, infos, total_blocks=32, min_block=8) == [24, 25, 26, 27]
    assert choose_best_blocks(8, [], total_blocks=32, min_block=8) == list(range(8, 16))
    # min_block protects the client's local span
    assert choose_best_blocks(4, infos, total_blocks=32, min_block=30)[0] == 28


@given(st.lists(st.floats(0, 100, allow_nan=False), min_size=1, max_size=40), st.integers(1, 8), st.integers(0, 40))
def test_choose_best_start_matches_bruteforce(thr, nb, mb):
    thr = np.array(thr)
    got = _choose_best_start(thr, nb, mb)
    if len(thr) < nb:
        assert got == max(0, mb)
        return
    last = len(thr) - nb
    lo = max(0, min(mb, last))
    want = min(((thr[i:i + nb].min(), thr[i:i + nb].mean(), i) for i in range(lo, last + 1)))[2]
    assert got == want


def test_should_choose_other_blocks():
    # two servers stacked on the same span, the rest uncovered... a moves to improve the min
    infos = _infos([("a", 0, 4, 10.0), ("b", 0, 4, 10.0), ("c", 4, 8, 10.0)])
    assert should_choose_other_blocks("a", infos, 0.75, total_blocks=8, rng=np.random.default_rng(0)) is False
    # balanced swarm: no move
    infos = _infos([("a", 0, 4, 10.0), ("b", 4, 8, 10.0), ("c", 0, 4, 10.0), ("d", 4, 8, 10.0)])
    assert should_choose_other_blocks("a", infos, 0.75, total_blocks=8, rng=np.random.default_rng(0)) is False
    # a weak block range and a redundant strong server -> move
    infos = _infos([("a", 0, 4, 10.0), ("b", 0, 4, 10.0), ("c", 0, 4, 10.0), ("d", 4, 8, 1.0)])
    assert should_choose_other_blocks("a", infos, 0.75, total_blocks=8, rng=np.random.default_rng(0)) is True
    # forced (debug switch), unknown peer
    assert should_choose_other_blocks("zz", infos, 1.5, total_blocks=8) is True
    assert should_choose_other_blocks("zz", infos, 0.75, total_blocks=8) is False


@settings(max_examples=40, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 11), st.integers(1, 6), st.floats(0.5, 20)), min_size=1, max_size=6))
def test_rebalance_never_uncovers(spec):
    total = 12
    spans = [(f"p{i}", s, min(s + n, total), t) for i, (s, n, t) in enumerate(spec) if s < total]
    if not spans:
        return
    infos = _infos(spans)
    for pid, *_ in spans:
        should_choose_other_blocks(pid, infos, 0.75, total_blocks=total, rng=np.random.default_rng(1))
    # the call must not mutate the caller's records
    assert compute_throughputs(compute_spans(infos), total).sum() > 0


def test_block_utils_sizes_and_auto_num_blocks():
    import torch

    from src.block_utils import (auto_num_blocks, default_attn_cache_tokens, get_block_size, kv_cache_bytes_per_block,
                                 resolve_block_dtype)
    from src.models.config import resolve_model

    cfg = resolve_model("llama2-7b")
    # 4096*12288 + 4096*4096 + 3*4096*11008 + 2*4096 parameters
    n = 4096 * 12288 + 4096 * 4096 + 3 * 4096 * 11008 + 2 * 4096
    assert get_block_size(cfg, "memory", torch.bfloat16) == 2 * n
    assert get_block_size(cfg, "disk", torch.float32) == 4 * n
    fp8 = get_block_size(cfg, "memory", torch.bfloat16, quant_type="fp8")
    assert n - 2 * 4096 < fp8 < 1.01 * n
    assert resolve_block_dtype(cfg, "auto") == torch.bfloat16
    assert default_attn_cache_tokens(cfg) == 4096
    assert default_attn_cache_tokens(resolve_model("llama3-8b")) == 16384
    per = get_block_size(cfg) + kv_cache_bytes_per_block(cfg)
    assert auto_num_blocks(cfg, free_bytes=10 * per + (2 << 30)) == 10
    assert auto_num_blocks(cfg, free_bytes=288 << 30) == 32  # a whole Llama-2-7B fits one MI355X
    assert auto_num_blocks(cfg, free_bytes=1) == 1


def test_throughput_cache_roundtrip(tmp_path):
    import torch

    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor
    from src.throughput_measurement import ThroughputCache, get_server_throughput, measure_forward_throughput

    cfg = resolve_model("tiny-llama")
    w = random_stage_weights(cfg, 0, 2, has_embed=False, has_head=False, device="cpu", dtype=torch.float32)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=4, max_seq_len=256,
                       max_tokens_per_step=128)
    cache = ThroughputCache(str(tmp_path / "tp.json"))
    t1 = get_server_throughput(ex, 1e6, cache=cache, n_steps=2)
    key = ThroughputCache.key(ex)
    assert cache.get(key)["compute_rps"] > 0
    cache.put(key, {"compute_rps": 12.5})
    assert get_server_throughput(ex, 1e6, cache=cache) == 12.5  # served from the cache
    assert t1 > 0
    assert measure_forward_throughput(ex, n_tokens=64, n_steps=1) > 0
