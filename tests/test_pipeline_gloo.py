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


def _worker(rank, world, port, steps, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.parallel import dist as pdist
    from src.parallel.pipeline import PipelineEngine
    from src.partition import even_splits, stage_ranges
    from src.runtime.executor import StageExecutor
    from src.runtime.sampler import SamplingParams

    rank, world, _, dev = pdist.init_distributed("cpu")
    cfg = resolve_model("tiny-llama")
    s, e = stage_ranges(even_splits(cfg.num_hidden_layers, world), cfg.num_hidden_layers)[rank]
    w = random_stage_weights(cfg, s, e, has_embed=rank == 0, has_head=rank == world - 1, device="cpu",
                             dtype=torch.float32, seed=3)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=16 << 20, max_sessions=8, max_seq_len=128)
    M, B = 2, 3
    eng = PipelineEngine(ex, rank, world, SamplingParams(0.0, 1.0, 0, 1.0), n_micro=M, batch=B)
    eng.record = True
    g = torch.Generator().manual_seed(5)
    prompts = [torch.randint(0, cfg.vocab_size, (B, 9), generator=g) for _ in range(M)]
    eng.prefill(prompts)
    eng.decode(steps)
    eng.finish()
    if rank == 0:
        out_q.put(eng.generated())
    pdist.barrier()
    pdist.shutdown()


def _run(world, steps=4):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(600)
def test_pipeline_stages_agree():
    one = _run(1)
    two = _run(2)
    four = _run(4)
    assert one == two == four
    assert len(one) == 2 and len(one[0]) == 3 and len(one[0][0]) == 5  # prefill token + 4 decode tokens
