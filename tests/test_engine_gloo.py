"""Continuous-batching pipeline serving engine (parallel/engine.py) on CPU.

* 1 stage, in process: batched continuous serving == every request run alone (seeds depend
  only on (request seed, position)); greedy == the fp32 oracle model's argmax loop;
  EOS / max_new_tokens / repetition stops; chunked prefill; admission beyond one batch.
* N stages over gloo channels (one process per stage, TCPStore rendezvous like the device
  channel's RCCL groups): identical tokens for stages in {2, 3} and slots in {S, S+1, 2S}.
* A stage that stops answering makes its peers fail within the channel timeout (non-zero
  exit, no hang).
"""
import os
import signal
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

from src.models.config import resolve_model
from src.models.reference_model import reference_forward
from src.models.weights import random_stage_weights
from src.parallel.engine import PipelineServingEngine, Request
from src.runtime.executor import StageExecutor
from src.runtime.sampler import SamplingParams

MODEL = "tiny-llama"
SEED = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _executor(start, end, embed, head, max_sessions=16):
    cfg = resolve_model(MODEL)
    w = random_stage_weights(cfg, start, end, has_embed=embed, has_head=head, device="cpu", dtype=torch.float32,
                             seed=SEED)
    return cfg, w, StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=16 << 20,
                                 max_sessions=max_sessions, max_seq_len=256, max_tokens_per_step=512)


def _requests(n=7, greedy=False, eos=None):
    cfg = resolve_model(MODEL)
    g = torch.Generator().manual_seed(11)
    out = []
    for i in range(n):
        L = int(torch.randint(3, 40, (1,), generator=g))
        prompt = torch.randint(0, cfg.vocab_size, (L,), generator=g).tolist()
        sp = SamplingParams(0.0, 1.0, 0, 1.0) if greedy else SamplingParams(1.0, 0.92, 50, 1.5)
        out.append(dict(prompt=prompt, max_new_tokens=6 + (i % 4), params=sp, eos_token_id=eos, seed=1000 + i,
                        rid=f"r{i}", stop_on_repeat=0 if greedy else 5))
    return out


def _serve_local(reqs, batch=4, n_slots=1, prefill_chunk=None, max_step_tokens=None):
    cfg, w, ex = _executor(0, resolve_model(MODEL).num_hidden_layers, True, True)
    eng = PipelineServingEngine(ex, None, n_slots=n_slots, batch=batch, prefill_chunk=prefill_chunk,
                                max_step_tokens=max_step_tokens)
    rs = [eng.submit(Request(**r)) for r in reqs]
    eng.run_until_idle(max_rounds=500)
    assert all(r.done for r in rs)
    return {r.rid: (list(r.generated), r.finish_reason) for r in rs}, w


def test_batched_equals_alone_and_chunked():
    reqs = _requests()
    batched, _ = _serve_local(reqs, batch=3, n_slots=2)
    alone = {}
    for r in reqs:
        alone.update(_serve_local([r], batch=1)[0])
    assert batched == alone
    chunked, _ = _serve_local(reqs, batch=8, prefill_chunk=7, max_step_tokens=16)
    assert chunked == alone
    assert all(len(g) == r["max_new_tokens"] or fr == "repeat" for r, (g, fr) in
               zip(reqs, (alone[r["rid"]] for r in reqs)))


def test_greedy_matches_oracle_and_eos():
    reqs = _requests(4, greedy=True)
    got, w = _serve_local(reqs, batch=4)
    for r in reqs:
        seq = list(r["prompt"])
        for _ in range(r["max_new_tokens"]):
            seq.append(int(torch.argmax(reference_forward([w], torch.tensor(seq))[-1])))
        assert got[r["rid"]][0] == seq[len(r["prompt"]):], r["rid"]
    # EOS: the first greedy token not seen before position k >= 1 becomes EOS -> generation
    # stops right before it (EOS itself is not emitted)
    cands = [(r["rid"], k) for r in reqs for k, t in enumerate(got[r["rid"]][0]) if k >= 1
             and t not in got[r["rid"]][0][:k]]
    assert cands
    rid, k = cands[0]
    r0 = dict(next(r for r in reqs if r["rid"] == rid), eos_token_id=got[rid][0][k], max_new_tokens=20)
    g2, _ = _serve_local([r0], batch=1)
    assert g2[rid] == (got[rid][0][:k], "eos")


# ---------------------------------------------------------------------------- multi-process
def _stage_worker(rank, world, port, n_slots, out_q, kill_rank=None, kill_after=None):
    torch.set_num_threads(1)
    from src.parallel.channel import Channel, make_store
    from src.parallel.engine import PipelineFailure
    from src.partition import even_splits, stage_ranges

    cfg = resolve_model(MODEL)
    s, e = stage_ranges(even_splits(cfg.num_hidden_layers, world), cfg.num_hidden_layers)[rank]
    _, _, ex = _executor(s, e, rank == 0, rank == world - 1)
    store = make_store("127.0.0.1", port, world, rank == 0)
    ch = Channel(store, "pipe0", rank, world, "cpu", timeout_s=20.0)
    eng = PipelineServingEngine(ex, ch, n_slots=n_slots, batch=3)
    try:
        if rank == 0:
            rs = [eng.submit(Request(**r)) for r in _requests()]
            eng.run_until_idle(max_rounds=500)
            eng.stop()
            out_q.put({r.rid: (list(r.generated), r.finish_reason) for r in rs})
        else:
            if rank == kill_rank:
                for _ in range(kill_after * n_slots):
                    eng._stage_step()
                os.kill(os.getpid(), signal.SIGSTOP if os.environ.get("ENGINE_TEST_STOP") else signal.SIGKILL)
            eng.serve()
    except PipelineFailure as e:
        if rank == 0:
            out_q.put(("failed", rank, str(e)[:200]))
            out_q.close()
            out_q.join_thread()  # flush the queue's feeder thread before the hard exit
        os._exit(3)
    ch.close()


def _run_stages(world, n_slots, kill_rank=None, kill_after=None, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stage_worker, args=(r, world, port, n_slots, q, kill_rank, kill_after))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=timeout)
        for p in procs:
            p.join(90)
        return res, [p.exitcode for p in procs]
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()


@pytest.mark.timeout(900)
def test_stages_and_slots_agree():
    ref = {}
    for r in _requests():
        ref.update(_serve_local([r], batch=1)[0])
    for world, slots in ((2, 2), (2, 3), (3, 4), (3, 6)):
        got, codes = _run_stages(world, slots)
        assert got == ref, (world, slots)
        assert codes == [0] * world, (world, slots, codes)


@pytest.mark.timeout(300)
def test_dead_stage_fails_peers_fast():
    """SIGKILL the middle stage mid-decode: the head's next send / token wait fails, it
    reports a PipelineFailure and exits non-zero; nobody hangs."""
    t0 = time.time()
    got, codes = _run_stages(3, 4, kill_rank=1, kill_after=3, timeout=120)
    assert got[0] == "failed" and got[1] == 0, got
    assert codes[1] == -signal.SIGKILL
    assert codes[0] == 3 and codes[2] in (3, 0), codes
    assert time.time() - t0 < 60
