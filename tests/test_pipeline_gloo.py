"""Multi-process pipeline (the RCCL engine's protocol) on CPU with gloo: N stages == 1 stage."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, steps, out_q, stages=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.parallel import dist as pdist
    from src.parallel.pipeline import PipelineEngine, make_replica_groups, make_token_groups
    from src.partition import even_splits, stage_ranges
    from src.runtime.executor import StageExecutor
    from src.runtime.sampler import SamplingParams

    rank, world, _, dev = pdist.init_distributed("cpu")
    S = stages or world
    groups = make_replica_groups(world, S)
    tok_groups = make_token_groups(world, S)
    cfg = resolve_model("tiny-llama")
    st = rank % S
    s, e = stage_ranges(even_splits(cfg.num_hidden_layers, S), cfg.num_hidden_layers)[st]
    w = random_stage_weights(cfg, s, e, has_embed=st == 0, has_head=st == S - 1, device="cpu",
                             dtype=torch.float32, seed=3)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=16 << 20, max_sessions=8, max_seq_len=128)
    M, B = 2, 3
    eng = PipelineEngine(ex, rank, world, SamplingParams(0.0, 1.0, 0, 1.0), n_micro=M, batch=B, stages=S,
                         groups=groups, tok_groups=tok_groups)
    eng.record = True
    g = torch.Generator().manual_seed(5)
    prompts = [torch.randint(0, cfg.vocab_size, (B, 9), generator=g) for _ in range(M)]
    eng.prefill(prompts)
    eng.decode(steps)
    eng.finish()
    if st == 0:
        out_q.put((rank, eng.generated()))
    pdist.barrier()
    pdist.shutdown()


def _run(world, steps=4, stages=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, steps, q, stages)) for r in range(world)]
    for p in procs:
        p.start()
    n_rep = world // (stages or world)
    res = dict(q.get(timeout=240) for _ in range(n_rep))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res[0] if n_rep == 1 else res


@pytest.mark.timeout(600)
def test_pipeline_stages_agree():
    one = _run(1)
    two = _run(2)
    four = _run(4)
    assert one == two == four
    assert len(one) == 2 and len(one[0]) == 3 and len(one[0][0]) == 5  # prefill token + 4 decode tokens


@pytest.mark.timeout(600)
def test_pipeline_replicas_two_by_two():
    """4 ranks = 2 replicas x 2 stages (sub-communicator per replica): both replicas generate
    exactly what one stage generates (greedy, same prompts)."""
    one = _run(1)
    reps = _run(4, stages=2)
    assert sorted(reps) == [0, 2]
    assert reps[0] == one and reps[2] == one


def test_assign_sessions_proportional():
    from src.parallel.pipeline import assign_sessions

    a = assign_sessions(10, [1.0, 1.0])
    assert a.count(0) == 5 and a.count(1) == 5
    a = assign_sessions(9, [2.0, 1.0])
    assert a.count(0) == 6 and a.count(1) == 3
    assert assign_sessions(3, [0.0, 0.0]).count(0) == 2
