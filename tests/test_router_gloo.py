"""Replica routing + failover over device channels (parallel/router.py), 2 replicas x 2 stages
on CPU/gloo: a throughput all-gather places sessions, one replica's tail is SIGKILLed
mid-decode, its sessions are re-prefilled from token history on the survivor, and every
session's tokens equal an uninterrupted single-engine run; every surviving process exits 0."""
import os
import signal
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

from src.models.config import resolve_model
from src.models.weights import random_stage_weights
from src.parallel.engine import PipelineServingEngine, Request
from src.runtime.executor import StageExecutor
from src.runtime.sampler import SamplingParams

MODEL = "tiny-llama"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ex(start, end, embed, head):
    cfg = resolve_model(MODEL)
    w = random_stage_weights(cfg, start, end, has_embed=embed, has_head=head, device="cpu", dtype=torch.float32,
                             seed=9)
    return StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=16 << 20, max_sessions=24,
                         max_seq_len=256, max_tokens_per_step=512)


def _reqs(n=10):
    cfg = resolve_model(MODEL)
    g = torch.Generator().manual_seed(4)
    out = []
    for i in range(n):
        L = int(torch.randint(4, 30, (1,), generator=g))
        out.append(dict(prompt=torch.randint(0, cfg.vocab_size, (L,), generator=g).tolist(), max_new_tokens=12,
                        params=SamplingParams(1.0, 0.92, 50, 1.5), seed=500 + i, stop_on_repeat=0))
    return out


def _reference():
    cfg = resolve_model(MODEL)
    out = []
    for r in _reqs():
        eng = PipelineServingEngine(_ex(0, cfg.num_hidden_layers, True, True), None, batch=1)
        q = eng.submit(Request(**r))
        eng.run_until_idle(max_rounds=200)
        out.append(list(q.generated))
    return out


def _worker(rank, world, S, port, q, kill_rank, kill_after):
    torch.set_num_threads(1)
    from src.parallel.channel import Channel, HostLink, make_store
    from src.parallel.router import ReplicaFrontend, gather_replica_throughput, serve_replica_head
    from src.partition import even_splits, stage_ranges

    R = world // S
    r, s = divmod(rank, S)
    cfg = resolve_model(MODEL)
    a, b = stage_ranges(even_splits(cfg.num_hidden_layers, S), cfg.num_hidden_layers)[s]
    ex = _ex(a, b, s == 0, s == S - 1)
    store = make_store("127.0.0.1", port, world, rank == 0, timeout_s=60)
    all_link = HostLink(store, "all", rank, world, timeout_s=60)
    ch = Channel(store, f"rep{r}", s, S, "cpu", timeout_s=20)
    eng = PipelineServingEngine(ex, ch, n_slots=S + 1, batch=3, name=f"rep{r}")
    thr = gather_replica_throughput(all_link, ex, r, s, R, batch=2)
    if rank == 0:
        links = {k: HostLink(store, f"link{k}", 0, 2, timeout_s=20) for k in range(1, R)}
        fe = ReplicaFrontend(R, eng, links, throughputs=thr, timeout_s=20)
        reqs = [fe.submit(Request(**d)) for d in _reqs()]
        placed = [fe.router.placement[str(i)] for i in range(len(reqs))]
        fe.run()
        q.put({"tokens": [list(x.generated) for x in reqs], "failures": [f[0] for f in fe.failures],
               "placed": placed, "thr": thr})
        q.close()
        q.join_thread()
    elif s == 0:
        link = HostLink(store, f"link{r}", 1, 2, timeout_s=20)
        serve_replica_head(eng, link, timeout_s=20)
    elif rank == kill_rank:
        for _ in range(kill_after):
            eng._stage_step()
        os.kill(os.getpid(), signal.SIGKILL)
    else:
        eng.serve()
    os._exit(0)


def _run(kill_rank=None, kill_after=None, world=4, S=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(k, world, S, port, q, kill_rank, kill_after)) for k in range(world)]
    for p in ps:
        p.start()
    try:
        res = q.get(timeout=240)
        for p in ps:
            p.join(60)
        return res, [p.exitcode for p in ps]
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()


@pytest.mark.timeout(600)
def test_replicas_route_and_fail_over_exactly():
    ref = _reference()
    ok, codes = _run()
    assert ok["tokens"] == ref and ok["failures"] == [] and codes == [0, 0, 0, 0]
    assert sorted(set(ok["placed"])) == [0, 1]  # throughput-proportional placement used both replicas
    t0 = time.time()
    res, codes = _run(kill_rank=3, kill_after=9)
    assert res["failures"] == [1]
    assert res["tokens"] == ref
    assert codes[3] == -signal.SIGKILL and codes[0] == codes[1] == codes[2] == 0, codes
    assert time.time() - t0 < 120
