"""Every decode-GEMM kernel the autotuner can pick, through graph-captured executor steps, against
the fp32 oracle.

The kernel mix a box runs used to be the winner of a start-up timing race (``ops.autotune_gemm``),
so a box could run a combination no test had run (4 of 35 Llama-2-7B shapes differed
between two boxes).  The committed table pins the mix now; this test still drives EACH candidate -
forced everywhere it applies (``ops.set_gemm_sk``), plain and with the rotated k walk, with the qkv
fold on and off - through decode hipGraphs whose batch buckets carry padding rows (3 / 13 / 29 /
50 sessions in buckets 4 / 16 / 32 / 64), on the small-llama test model and on two-layer stages
with Llama-2-7B and Llama-3-8B (GQA) dimensions.  Tokens are teacher-forced, so one oracle pass
serves every kernel.  Reference: the decode step of petals/llama/block.py:183-248."""
import dataclasses

import pytest
import torch

from src import ops
from src.models.config import resolve_model
from src.models.reference_model import reference_forward
from src.models.weights import random_stage_weights
from src.runtime.executor import StageExecutor

pytestmark = pytest.mark.gpu

PROMPT, STEPS = 8, 2
BATCHES = (3, 13, 29, 50)


def _cfg(name):
    cfg = resolve_model(name)
    if cfg.num_hidden_layers > 8:
        cfg = dataclasses.replace(cfg, num_hidden_layers=2)
    return cfg


def _candidates(cfg):
    H, F = cfg.hidden_size, cfg.intermediate_size
    shapes = [(cfg.q_dim + 2 * cfg.kv_dim, H, 0), (H, cfg.q_dim, 3), (2 * F, H, 1), (H, F, 3)]
    names = set()
    for M in BATCHES:
        for N, K, e in shapes:
            names.update(k for k in ops._KERNEL_FLAGS if k != "t2d" and ops._covered(k, M, N, K, e))
    return sorted(names)


@pytest.fixture(scope="module", params=["small-llama", "llama2-7b", "llama3-8b"])
def setup(request):
    cfg = _cfg(request.param)
    w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cuda", seed=11)
    ex = StageExecutor(cfg, w, "cuda", kv_cache_bytes=512 << 20, max_sessions=64, max_seq_len=256,
                       graph_max_batch=64, max_tokens_per_step=1024, warmup=False)
    g = torch.Generator().manual_seed(3)
    n = max(BATCHES)
    seqs = torch.randint(0, cfg.vocab_size, (n, PROMPT + STEPS), generator=g)
    oracle = torch.stack([reference_forward([w], seqs[i].cuda())[PROMPT - 1:].float() for i in range(n)])
    yield cfg, ex, seqs.cuda(), oracle
    del ex, w
    torch.cuda.empty_cache()


def _run(ex, seqs, oracle, B, tag):
    """(relative error, argmax agreement) of a prefill + STEPS graph-replayed decode steps."""
    sids = [f"{tag}:{i}" for i in range(B)]
    out = [ex.forward([(s, PROMPT) for s in sids], seqs[:B, :PROMPT].reshape(-1), reset=[True] * B).float()]
    for t in range(STEPS):
        # (.float() copies now: a graph replay returns its static output, which the next replay overwrites)
        out.append(ex.forward([(s, 1) for s in sids], seqs[:B, PROMPT + t].contiguous()).float())
        assert ex.last_graphed, (tag, B, t)
    torch.cuda.synchronize()
    for s in sids:
        ex.sessions.close(s)
    got = torch.stack(out, 1)                            # [B, STEPS + 1, V]
    ref = oracle[:B]
    assert torch.isfinite(got).all(), (tag, B)
    return float((got - ref).norm() / ref.norm()), float((got.argmax(-1) == ref.argmax(-1)).float().mean())


def _check(res):
    """Every candidate within bf16 distance of the fp32 oracle, and no worse than the reference
    one-group kernel ("pk", no fold) on the same rows by more than rounding noise."""
    lines = [f"{k}: err {e:.4f} agree {a:.3f}" for k, (e, a) in sorted(res.items())]
    for (name, B), (e, a) in res.items():
        base = res.get(("pk/f0", B), (e, a))[0]
        # (argmax agreement is only a gross check: random-init logits have near-ties, and 3 sessions x
        # 3 steps = 9 rows; the bf16-vs-fp32 distance is the measure)
        assert e < max(0.03, 1.3 * base) and a >= 0.6, "\n".join(lines)


def test_every_gemm_candidate_through_decode_graphs(setup, monkeypatch):
    cfg, ex, seqs, oracle = setup
    monkeypatch.setattr(ops, "_GEMM_SK", "auto")
    names = _candidates(cfg)
    assert "pk" in names and len(names) >= 3, names
    folds = (False, True) if ex._fused and ex._fuse_rope else (False,)
    res = {}
    try:
        for name in ["pk"] + [n for n in names if n != "pk"]:
            for rot in ("", "+r"):
                ops.set_gemm_sk(name + rot)
                for fold in folds:
                    ex.clear_graphs()
                    ex.qkv_fold_by_bucket = {ex._bucket(B): fold for B in BATCHES}
                    for B in BATCHES:
                        res[(f"{name}{rot}/f{int(fold)}", B)] = _run(ex, seqs, oracle, B, f"{name}{rot}/f{int(fold)}")
    finally:
        ops.set_gemm_sk("auto")
        ex.clear_graphs()
        ex.qkv_fold_by_bucket = {}
    print("\n".join(f"{k}: err {e:.4f} agree {a:.3f}" for k, (e, a) in sorted(res.items())))
    _check(res)


def test_committed_table_through_decode_graphs(setup):
    """The mix the benches and the serving path run: the committed table, unforced."""
    cfg, ex, seqs, oracle = setup
    assert ops._GEMM_SK == "auto"
    assert ops.kernel_table_report()["gemm_table_sha"] is not None, "no committed kernel table loaded"
    ex.clear_graphs()
    res = {}
    for B in BATCHES:
        ex.qkv_fold_by_bucket[ex._bucket(B)] = bool(ops.qkv_fold_pinned(ex._bucket(B), cfg.q_dim + 2 * cfg.kv_dim,
                                                                        cfg.hidden_size, False))
        res[("table", B)] = _run(ex, seqs, oracle, B, "table")
    ops.set_gemm_sk("pk")
    ex.clear_graphs()
    ex.qkv_fold_by_bucket = {}
    try:
        for B in BATCHES:
            res[("pk/f0", B)] = _run(ex, seqs, oracle, B, "pk")
    finally:
        ops.set_gemm_sk("auto")
        ex.clear_graphs()
    print("\n".join(f"{k}: err {e:.4f} agree {a:.3f}" for k, (e, a) in sorted(res.items())))
    _check(res)
