"""Replica failover by token replay (parallel/failover.py) with CPU executors as replicas."""
import torch

from src.models.config import resolve_model
from src.models.weights import random_stage_weights
from src.parallel.failover import ReplicaRouter
from src.runtime.executor import StageExecutor


def _replica():
    cfg = resolve_model("tiny-llama")
    w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cpu",
                             dtype=torch.float32, seed=9)
    return StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=8, max_seq_len=128)


def _step(ex, sid, toks, reset=False):
    logits = ex.forward([(sid, len(toks))], torch.tensor(toks), reset=[reset])
    return int(torch.argmax(logits[-1]))


def test_failed_replica_sessions_resume_identically():
    reps = [_replica(), _replica()]
    router = ReplicaRouter(2, throughputs=[1.0, 1.0])
    prompts = {"a": [1, 2, 3, 4], "b": [9, 8, 7], "c": [5, 5, 6, 7, 8], "d": [11]}
    where = router.place(list(prompts), list(prompts.values()))
    assert sorted(where.values()) == [0, 0, 1, 1]

    # reference: every session decoded without interruption on a fresh replica
    ref = {}
    solo = _replica()
    for sid, p in prompts.items():
        toks = [_step(solo, sid, p, reset=True)]
        for _ in range(7):
            toks.append(_step(solo, sid, [toks[-1]]))
        ref[sid] = toks

    out = {sid: [] for sid in prompts}
    for sid, p in prompts.items():
        t = _step(reps[where[sid]], sid, p, reset=True)
        out[sid].append(t)
        router.record(sid, t)
    for step in range(7):
        if step == 3:  # replica 0 dies: its sessions move to replica 1 and rebuild KV from tokens
            plans = router.fail(0)
            assert {pl.session_id for pl in plans} == {s for s, r in where.items() if r == 0}
            for pl in plans:
                assert pl.replica == 1
                # re-prefill everything but the last generated id (that one is the next input)
                reps[1].forward([(pl.session_id, len(pl.tokens) - 1)], torch.tensor(pl.tokens[:-1]), reset=[True])
        for sid in prompts:
            r = router.placement[sid]
            t = _step(reps[r], sid, [out[sid][-1]])
            out[sid].append(t)
            router.record(sid, t)
    assert out == ref
    assert router.live() == [1] and router.sessions_on(0) == []


def test_heartbeat_expiry_and_weighted_replacement():
    router = ReplicaRouter(3, throughputs=[1.0, 3.0, 1.0], timeout_s=5.0)
    router.place([f"s{i}" for i in range(10)], [[1]] * 10)
    for r in range(3):
        router.heartbeat(r, now=100.0)
    router.heartbeat(1, now=104.0)
    assert router.expired(now=106.0) == [0, 2]
    plans = router.fail(0)
    moved = [p.replica for p in plans]
    assert moved and all(m in (1, 2) for m in moved)
    assert moved.count(1) >= moved.count(2)  # the 3x faster replica takes the larger share
    assert router.fail(0) == []
