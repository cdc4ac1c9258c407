"""Direct RCCL communicators (parallel/rccl.py, native/rccl.cpp) on the 1-GPU box: a world-1
communicator's all-reduce, a self send/recv, both captured into a hipGraph and replayed, and a
tensor-parallel executor whose all-reduces go through the communicator with its decode steps
graph-captured (the multi-GPU TP path's graph mechanics, at one rank).  Everything runs in one
spawned process (RCCL state and any hang stay out of the pytest process)."""
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _say(*a):
    import sys

    print("[rccl-test]", *a, file=sys.stderr, flush=True)


def _body(port, q):
    try:
        import torch.distributed as dist

        from src.parallel import rccl
        from src.parallel.tensor_parallel import TPGroup

        out = {"version": None}
        store = dist.TCPStore("127.0.0.1", port, 1, True)
        comm = rccl.RcclComm(store, "t", 0, 1, "cuda:0")
        out["version"] = rccl.VERSION
        _say("comm up", rccl.VERSION)
        # all-reduce (world 1: identity), eager then captured
        x = torch.arange(4096, device="cuda", dtype=torch.float32)
        comm.all_reduce(x)
        torch.cuda.synchronize()
        out["ar_eager"] = bool(torch.equal(x, torch.arange(4096, device="cuda", dtype=torch.float32)))
        _say("eager all-reduce", out["ar_eager"])
        dst0 = torch.zeros(1024, device="cuda")
        comm.send_recv(x[:1024], 0, dst0, 0)
        torch.cuda.synchronize()
        _say("eager self send/recv", bool(torch.equal(dst0, x[:1024])))
        # self send -> recv in one group, captured: replays move the CURRENT contents of src
        src = torch.zeros(64, 4096, dtype=torch.bfloat16, device="cuda")
        dst = torch.zeros_like(src)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            comm.send_recv(src, 0, dst, 0)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        _say("side-stream send/recv done; capturing")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y = src * 2
            comm.send_recv(y, 0, dst, 0)
            comm.all_reduce(dst)
        ok = []
        for v in (1.5, -3.0, 7.25):
            src.fill_(v)
            g.replay()
            torch.cuda.synchronize()
            ok.append(bool((dst == 2 * v).all()))
        out["sendrecv_graph"] = ok
        _say("graph replays", ok)
        # TP executor at one forced rank: graphs captured with the RCCL all-reduces inside
        from src.models.config import resolve_model
        from src.models.weights import random_stage_weights
        from src.runtime.executor import StageExecutor

        cfg = resolve_model("small-llama")
        tp = TPGroup(None, comm=comm, force=True)
        outs = {}
        for graphs in (False, True):
            w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cuda",
                                     seed=3)
            ex = StageExecutor(cfg, w, "cuda", kv_cache_bytes=64 << 20, max_sessions=8, max_seq_len=256, tp=tp,
                               use_graphs=graphs)
            ids = torch.arange(3 * 9, device="cuda") % cfg.vocab_size
            lg = ex.forward([(f"s{i}", 9) for i in range(3)], ids)
            toks = [lg.float().argmax(-1)]
            for _ in range(4):
                lg = ex.forward([(f"s{i}", 1) for i in range(3)], toks[-1])
                toks.append(lg.float().argmax(-1))
            torch.cuda.synchronize()
            outs[graphs] = (torch.stack(toks).tolist(), lg.float().cpu(), ex.use_graphs, len(ex._graphs))
            _say("tp executor graphs =", graphs, "done")
        out["tp_graphs_on"] = outs[True][2] and outs[True][3] > 0
        out["tp_tokens_equal"] = outs[True][0] == outs[False][0]
        out["tp_logits_maxdiff"] = float((outs[True][1] - outs[False][1]).abs().max())
        # a decode graph that ends with an RCCL send recorded by the executor's graph hook (the
        # engine's graph hop): every replay moves the step's static output
        w2 = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=False, device="cuda",
                                  seed=4)
        ex2 = StageExecutor(cfg, w2, "cuda", kv_cache_bytes=64 << 20, max_sessions=8, max_seq_len=256)
        sink = torch.zeros(16, cfg.hidden_size, dtype=torch.bfloat16, device="cuda")
        owner = object()
        ex2.set_graph_hook(lambda o: comm.send_recv(o, 0, sink[: o.shape[0]], 0), owner=owner)
        ids = torch.arange(3 * 9, device="cuda") % cfg.vocab_size
        ex2.forward([(f"g{i}", 9) for i in range(3)], ids)
        hook_ok = []
        for st in range(3):
            hh = ex2.forward([(f"g{i}", 1) for i in range(3)], ids[st * 3:st * 3 + 3], hook_owner=owner)
            torch.cuda.synchronize()
            hook_ok.append(bool(ex2.last_hooked) and bool(torch.equal(sink[:3], hh[:3])))
        # a caller that is not the hook's owner replays a hook-free graph: the sink keeps its bytes
        sink.zero_()
        hh = ex2.forward([(f"g{i}", 1) for i in range(3)], ids[:3])
        torch.cuda.synchronize()
        hook_ok.append(bool(ex2.last_graphed) and not ex2.last_hooked and float(sink.abs().sum()) == 0.0)
        ex2.clear_graph_hook(owner)
        hook_ok.append(ex2.graph_hook is None and not any(k[-1] for k in ex2._graphs))
        out["graph_hook"] = hook_ok
        out["graph_rows"] = ex2.graph_rows(3, True)
        _say("graph hook", hook_ok)
        del ex, g, ex2
        import gc

        gc.collect()
        torch.cuda.synchronize()
        out["alive"] = comm.alive and comm.async_error() == 0
        _say("async error polled", out["alive"])
        comm.close()
        _say("destroyed")
        # abort: the failure path (a stream blocked on a dead peer is released)
        c2 = rccl.RcclComm(store, "t2", 0, 1, "cuda:0")
        y2 = torch.ones(16, device="cuda")
        c2.all_reduce(y2)
        torch.cuda.synchronize()
        c2.abort()
        out["aborted"] = not c2.alive
        _say("aborted")
        q.put(("ok", out))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put(("error", traceback.format_exc()[-3000:]))


def test_rccl_world1_capture_and_tp_graphs():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_body, args=(_port(), q))
    p.start()
    try:
        status, out = q.get(timeout=110)
    finally:
        p.join(30)
        if p.is_alive():
            p.kill()
    print("rccl direct:", status, out)
    assert status == "ok", out
    assert out["version"] and out["version"] >= 22000
    assert out["ar_eager"]
    assert out["sendrecv_graph"] == [True, True, True]
    assert out["tp_graphs_on"]
    assert out["tp_tokens_equal"]
    # graph steps pad the batch to its bucket (the decode GEMMs may pick another row-tile form)
    assert out["tp_logits_maxdiff"] < 5e-2
    assert out["alive"] and out["aborted"]
    assert out["graph_hook"] == [True] * 5 and out["graph_rows"] == 4
