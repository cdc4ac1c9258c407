"""Tensor parallelism inside a stage (parallel/tensor_parallel.py): sharding math on one process,
and a 2-rank gloo run whose sharded executors reproduce the unsharded stage."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from src.models.config import resolve_model
from src.models.reference_model import reference_forward
from src.models.weights import random_stage_weights
from src.parallel.tensor_parallel import check_tp, shard_config, shard_stage_weights
from src.runtime.executor import StageExecutor


def _w(model, dtype=torch.float32):
    cfg = resolve_model(model)
    return cfg, random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cpu",
                                     dtype=dtype, seed=13)


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_shards_reassemble_the_block(model):
    """Sum over ranks of the row-parallel outputs == the unsharded projections (one layer, fp64)."""
    cfg, w = _w(model, torch.float64)
    tp = 2
    shards = [shard_stage_weights(w, r, tp) for r in range(tp)]
    assert shards[0].cfg.num_attention_heads == cfg.num_attention_heads // tp
    L = w.layers[0]
    x = torch.randn(5, cfg.hidden_size, dtype=torch.float64)
    full_qkv = x @ L.qkv.t()
    D, nh, nkv = cfg.head_dim, cfg.num_attention_heads, cfg.num_key_value_heads
    q = torch.cat([x @ s.layers[0].qkv[: nh // tp * D].t() for s in shards], 1)
    torch.testing.assert_close(q, full_qkv[:, : nh * D])
    a = torch.randn(5, nh * D, dtype=torch.float64)
    o = sum(a[:, r * nh // tp * D:(r + 1) * nh // tp * D] @ shards[r].layers[0].o.t() for r in range(tp))
    torch.testing.assert_close(o, a @ L.o.t())


def test_check_tp_rejects_bad_degrees():
    cfg = resolve_model("tiny-llama")  # 4 heads, 2 kv heads
    check_tp(cfg, 2)
    with pytest.raises(ValueError):
        check_tp(cfg, 4)  # kv heads not divisible
    assert shard_config(cfg, 1) is cfg


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, model, q, device="cpu"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.parallel.tensor_parallel import TPGroup

        torch.set_num_threads(1)
        dt = torch.float32 if device == "cpu" else torch.bfloat16
        cfg = resolve_model(model)
        w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device=device,
                                 dtype=dt, seed=13)
        sw = shard_stage_weights(w, rank, world)
        ex = StageExecutor(sw.cfg, sw, device, dtype=dt, kv_cache_bytes=8 << 20, max_sessions=2,
                           max_seq_len=256, tp=TPGroup(None), use_graphs=False)
        g = torch.Generator().manual_seed(2)
        a = torch.randint(0, cfg.vocab_size, (70,), generator=g).to(device)
        outs = [ex.forward([("a", 70)], a)]
        for _ in range(2):
            nxt = torch.argmax(outs[-1], -1)
            outs.append(ex.forward([("a", 1)], nxt))
        if rank == 0:
            q.put(torch.cat(outs).float().cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_tp2_gloo_matches_unsharded(model):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, model, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = torch.from_numpy(q.get(timeout=240))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg, w = _w(model)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=2, max_seq_len=256)
    g = torch.Generator().manual_seed(2)
    a = torch.randint(0, cfg.vocab_size, (70,), generator=g)
    ref = [ex.forward([("a", 70)], a)]
    for _ in range(2):
        ref.append(ex.forward([("a", 1)], torch.argmax(ref[-1], -1)))
    torch.testing.assert_close(got, torch.cat(ref), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ref[0][-1], reference_forward([w], a)[-1], atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_tp2_sharded_hip_path_matches_oracle(model):
    """Two ranks share the one GPU (gloo all-reduce of device tensors): the sharded weights run
    through the packed HIP GEMMs / attention with half the heads and half the MLP width."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, model, q, "cuda")) for r in range(2)]
    for p in procs:
        p.start()
    got = torch.from_numpy(q.get(timeout=100))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg = resolve_model(model)
    w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cuda",
                             dtype=torch.bfloat16, seed=13)
    a = torch.randint(0, cfg.vocab_size, (70,), generator=torch.Generator().manual_seed(2))
    torch.testing.assert_close(got[0], reference_forward([w], a.cuda())[-1].cpu(), atol=0.06, rtol=0.05)
