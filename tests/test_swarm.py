"""End-to-end swarm on localhost (registry + TCP RPC + stage servers in threads), CPU path.

Covers the reference's manual integration procedures (scripts/run_all.py, test_fault_tolerance.py,
elice_test_load_balancing.sh) as automated tests.
"""
import uuid

import pytest
import torch

from src import main as M
from src.dht_utils import get_remote_module_infos, get_stage_key
from src.models.config import resolve_model
from src.models.reference_model import greedy_generate
from src.models.tokenizer import load_tokenizer
from src.models.weights import random_stage_weights
from src.rpc_transport import RpcTransport
from src.runtime.executor import StageExecutor

from .swarm_utils import ServerThread, client_args, server_argv, wait_for

MODEL = "tiny-gpt2"


def _reference(n_new, prompt="Hello, how are you?"):
    cfg = resolve_model(MODEL)
    w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cpu",
                             dtype=torch.float32)
    ids = torch.tensor(load_tokenizer(MODEL, cfg).encode(prompt))
    return greedy_generate([w], ids, n_new)


@pytest.mark.timeout(120)
def test_fixed_three_stage_generation_matches_reference():
    s1 = ServerThread(server_argv(MODEL, "1,2", 1)).wait()
    s2 = ServerThread(server_argv(MODEL, "1,2", 2, peers=s1.addr)).wait()
    try:
        assert wait_for(lambda: s1.dht.get(get_stage_key(2)) is not None)
        args = client_args(MODEL, "1,2", s1.addr, "--max_new_tokens 6 --temperature 0")
        gen = M.run_rank0(args, torch.device("cpu"), [1, 2])
        ref = _reference(len(gen))
        assert gen == ref
    finally:
        s1.close()
        s2.close()


def _client(peers, cuts, routing="stage", total=None, push=False):
    cfg = resolve_model(MODEL)
    w = random_stage_weights(cfg, 0, cuts[0], has_embed=True, has_head=False, device="cpu", dtype=torch.float32)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=4, max_seq_len=128)
    tx = RpcTransport("cpu", 0, [peers], timeout=5.0, temperature=0.0,
                      stage_keys=[get_stage_key(i) for i in range(1, len(cuts) + 1)], routing=routing,
                      model_name=MODEL, total_blocks=total or cfg.num_hidden_layers, start_block=cuts[0], push=push)
    return cfg, ex, tx


def _generate(ex, tx, n, on_step=None):
    cfg = resolve_model(MODEL)
    ids = torch.tensor(load_tokenizer(MODEL, cfg).encode("Hello, how are you?"))
    sid = str(uuid.uuid4())
    h = ex.forward([(sid, len(ids))], ids, reset=[True])
    tx.send_prefill(len(ids), h, sid, len(ids) + n + 1)
    out = [tx.recv_token()]
    cur = len(ids) + 1
    for i in range(n - 1):
        if on_step:
            on_step(i)
        h = ex.forward([(sid, 1)], torch.tensor([out[-1]]), starts=[cur - 1])
        tx.send_decode_step(cur, h, sid, len(ids) + n + 1, out)
        out.append(tx.recv_token())
        cur += 1
    return out


@pytest.mark.timeout(180)
def test_failover_to_replica_replays_kv():
    s1 = ServerThread(server_argv(MODEL, "2", 1)).wait()
    s1b = ServerThread(server_argv(MODEL, "2", 1, peers=s1.addr)).wait()
    try:
        assert wait_for(lambda: len(s1.dht.get(get_stage_key(1)).value) == 2)
        cfg, ex, tx = _client(s1.addr, [2])
        killed = []

        def kill_current(i):
            if i == 3:
                pid = tx.session_routes[next(iter(tx.session_routes))][0].peer_id
                victim = s1 if s1.srv.peer_id == pid else s1b
                victim.kill()
                killed.append(victim)

        gen = _generate(ex, tx, 10, kill_current)
        assert killed, "no server was killed"
        assert gen == _reference(10)
        assert tx.failed_peers  # a failover actually happened
        tx.shutdown()
    finally:
        s1.close()
        s1b.close()


@pytest.mark.timeout(180)
def test_load_balanced_servers_and_module_routing():
    extra = "--use_load_balancing --num_blocks 1 --mean_balance_check_period 1000"
    a = ServerThread(server_argv(MODEL, "2", 1, extra=extra)).wait()
    b = ServerThread(server_argv(MODEL, "2", 1, peers=a.addr, extra=extra)).wait()
    try:
        spans = sorted([(a.srv.ex.start, a.srv.ex.end), (b.srv.ex.start, b.srv.ex.end)])
        assert spans == [(2, 3), (3, 4)], spans  # the second server filled the uncovered block
        assert wait_for(lambda: len(get_remote_module_infos(a.dht, MODEL, 4)) >= 2)
        cfg, ex, tx = _client(a.addr, [2], routing="module", total=4)
        gen = _generate(ex, tx, 5)
        assert gen == _reference(5)
        assert [h.start for h in next(iter(tx.session_routes.values()))] == [2, 3]
        tx.shutdown()
    finally:
        a.close()
        b.close()


@pytest.mark.timeout(180)
def test_push_chain_matches_reference_and_records_history():
    """Server-to-server forwarding (upstream rpc_push): one client call per token."""
    s1 = ServerThread(server_argv(MODEL, "1,2", 1)).wait()
    s2 = ServerThread(server_argv(MODEL, "1,2", 2, peers=s1.addr)).wait()
    try:
        assert wait_for(lambda: s1.dht.get(get_stage_key(2)) is not None)
        cfg, ex, tx = _client(s1.addr, [1, 2], push=True)
        gen = _generate(ex, tx, 6)
        assert gen == _reference(6)
        assert s1.srv.handler.stats["pushed"] >= 6
        assert all(name.startswith("push:") for name, _ in tx.last_decode_stage_times)
        hist = next(iter(tx.client_cache.values()))
        assert sorted(hist) == [1, 2] and len(hist[1]) == len(hist[2]) == 6
        tx.shutdown()
    finally:
        s1.close()
        s2.close()


@pytest.mark.timeout(180)
def test_push_chain_downstream_failure_recovers_on_replica():
    s1 = ServerThread(server_argv(MODEL, "1,2", 1)).wait()
    s2 = ServerThread(server_argv(MODEL, "1,2", 2, peers=s1.addr)).wait()
    s2b = ServerThread(server_argv(MODEL, "1,2", 2, peers=s1.addr)).wait()
    try:
        assert wait_for(lambda: len(s1.dht.get(get_stage_key(2)).value) == 2)
        cfg, ex, tx = _client(s1.addr, [1, 2], push=True)
        killed = []

        def kill_last(i):
            if i == 2:
                pid = tx.session_routes[next(iter(tx.session_routes))][1].peer_id
                victim = s2 if s2.srv.peer_id == pid else s2b
                victim.kill()
                killed.append(victim)

        gen = _generate(ex, tx, 8, kill_last)
        assert killed and tx.failed_peers
        assert gen == _reference(8)
        tx.shutdown()
    finally:
        for s in (s1, s2, s2b):
            s.close()


@pytest.mark.timeout(120)
def test_rpc_inference_step_dedup_and_reachability():
    from src.comm.rpc import RpcClient, get_loop
    from src.comm.wire import Message

    s1 = ServerThread(server_argv(MODEL, "2", 1)).wait()
    try:
        cfg = resolve_model(MODEL)
        addr = s1.srv.maddrs[0]
        cl = RpcClient()
        loop = get_loop()
        h = torch.randn(1, 3, cfg.hidden_size)

        def call(name, md, tensors=()):
            return loop.run(cl.call(addr, "StageConnectionHandler." + name, Message(md, list(tensors)), 10.0))

        md = {"session_id": "s-1", "step_id": "a", "temperature": 0.0}
        r1 = call("rpc_inference", md, [h])
        r2 = call("rpc_inference", md, [h])  # same step id: served from the dedup cache
        assert r1.metadata["token_id"] == r2.metadata["token_id"]
        assert s1.srv.ex.sessions.get("s-1").length == 3
        r3 = call("rpc_inference", {"session_id": "s-1", "step_id": "b", "temperature": 0.0}, [h[:, :1]])
        assert s1.srv.ex.sessions.get("s-1").length == 4
        # rewind: re-run step b's position
        call("rpc_inference", {"session_id": "s-1", "step_id": "c", "start_from_position": 3, "temperature": 0.0},
             [h[:, :1]])
        assert s1.srv.ex.sessions.get("s-1").length == 4
        assert "token_id" in r3.metadata
        ok = call("rpc_check_reachability", {"target": addr})
        assert ok.metadata["ok"] is True
        bad = call("rpc_check_reachability", {"target": "/ip4/127.0.0.1/tcp/1/p2p/x", "timeout": 1.0})
        assert bad.metadata["ok"] is False
        loop.run(cl.close())
    finally:
        s1.close()


def test_task_prioritizer_orders_decode_first():
    from src.rpc_handler import TaskPrioritizer

    p = TaskPrioritizer()
    assert p.prioritize(1, False) < p.prioritize(128, True)
    assert p.prioritize(1, True) == p.prioritize(5, False)


@pytest.mark.timeout(120)
def test_strict_block_indices_and_models_record():
    """--block_indices pins the span (upstream Server strict_block_indices); _petals.models is announced."""
    from src.dht_utils import get_models_on_dht
    from src.main import parse_block_indices

    extra = "--use_load_balancing --block_indices 3:4 --public_name box-a --inference_max_length 64"
    a = ServerThread(server_argv(MODEL, "2", 1, extra=extra)).wait()
    try:
        assert (a.srv.ex.start, a.srv.ex.end) == (3, 4) and a.srv.final
        assert a.srv.ex.sessions.max_seq_len == 64
        models = get_models_on_dht(a.dht)
        assert models[MODEL]["num_blocks"] == 4 and models[MODEL]["public_name"] == "box-a"
        e = next(iter(a.dht.get(get_stage_key(1)).value.values()))
        e = e.value if hasattr(e, "value") else e
        assert e["public_name"] == "box-a"
    finally:
        a.close()
    assert parse_block_indices("0:2", 4) == [0, 1] and parse_block_indices(None, 4) is None
    with pytest.raises(SystemExit):
        parse_block_indices("3:9", 4)


@pytest.mark.timeout(120)
def test_next_pings_announced():
    """Servers measure RTTs to the next span's servers (upstream ModuleAnnouncer next_pings)."""
    s1 = ServerThread(server_argv(MODEL, "1,2", 1)).wait()
    s2 = ServerThread(server_argv(MODEL, "1,2", 2, peers=s1.addr)).wait()
    try:
        assert wait_for(lambda: s1.dht.get(get_stage_key(2)) is not None)
        pings = s1.srv.measure_next_pings()
        assert list(pings) == [s2.srv.peer_id] and 0 < pings[s2.srv.peer_id] < 2.0
        s1.srv.store_once()
        rec = s1.dht.get(get_stage_key(1)).value
        e = next(iter(rec.values()))
        e = e.value if hasattr(e, "value") else e
        assert e["next_pings"] == pings and e["cache_tokens_left"] > 0
        assert s2.srv.measure_next_pings() == {}  # final stage: nothing after it
    finally:
        s1.close()
        s2.close()


@pytest.mark.timeout(240)
def test_cli_client_over_device_channel_matches_reference(capsys):
    """``python -m src.main`` servers + the stage-0 client with ``--device_channel on``: the
    client rendezvouses a channel through both servers (rpc_channel_open over TCP), then the
    hidden states and token ids move on the channel (gloo here, RCCL on GPUs).  Greedy output
    equals the single-process reference; the servers keep serving TCP afterwards."""
    from src import main as M

    s1 = ServerThread(server_argv(MODEL, "1,2", 1)).wait()
    s2 = ServerThread(server_argv(MODEL, "1,2", 2, peers=s1.addr)).wait()
    try:
        assert wait_for(lambda: s1.dht.get(get_stage_key(2)) is not None)
        rec = s1.dht.get(get_stage_key(1)).value
        assert all("channel_host" in (v.value if hasattr(v, "value") else v) for v in rec.values())
        args = client_args(MODEL, "1,2", s1.addr, "--device_channel on --temperature 0 --max_new_tokens 6 "
                                                  "--num_sessions 3")
        gen = M.run_rank0(args, M.pick_device(args), [1, 2])
        assert gen == _reference(6)
        assert s1.srv.handler.stats.get("channels") == 1 and s2.srv.handler.stats.get("channels") == 1
        assert wait_for(lambda: not s1.srv.ex.sessions.sessions and not s2.srv.ex.sessions.sessions)
        # the TCP path still works on the same servers
        cfg, ex, tx = _client(s1.addr, [1, 2])
        assert _generate(ex, tx, 4) == _reference(4)
        tx.shutdown()
    finally:
        s1.close()
        s2.close()


@pytest.mark.timeout(180)
def test_cli_client_concurrent_tcp_sessions_batch_on_servers():
    """``--num_sessions 4 --device_channel off``: four sessions go over TCP concurrently; each
    server's batching window runs them as ragged multi-session steps, every session's greedy
    output equals the reference, and all sessions are closed afterwards."""
    from src import main as M

    s1 = ServerThread(server_argv(MODEL, "1,2", 1, extra="--batch_window_ms 20")).wait()
    s2 = ServerThread(server_argv(MODEL, "1,2", 2, peers=s1.addr, extra="--batch_window_ms 20")).wait()
    try:
        assert wait_for(lambda: s1.dht.get(get_stage_key(2)) is not None)
        seen = []
        orig = s1.srv.handler._run_batch
        s1.srv.handler._run_batch = lambda batch: (seen.append(len(batch)), orig(batch))[1]
        args = client_args(MODEL, "1,2", s1.addr, "--device_channel off --temperature 0 --max_new_tokens 6 "
                                                  "--num_sessions 4")
        gen = M.run_rank0(args, M.pick_device(args), [1, 2])
        assert gen == _reference(6)
        assert max(seen) > 1  # concurrent sessions shared a server step
        assert wait_for(lambda: not s1.srv.ex.sessions.sessions and not s2.srv.ex.sessions.sessions)
    finally:
        s1.close()
        s2.close()


@pytest.mark.timeout(240)
def test_lb_placement_follows_measured_throughput():
    """Load-balanced servers announce MEASURED throughput (batched compute probe, network term
    from a measured link): a 2-block span measures slower than a 1-block span, so the next
    server fills the slow span's blocks, not the lowest uncovered-by-one index."""
    extra = "--use_load_balancing --mean_balance_check_period 1000 --throughput_batch 16"
    a = ServerThread(server_argv(MODEL, "1", 1, extra=extra + " --num_blocks 1")).wait()
    b = ServerThread(server_argv(MODEL, "1", 1, peers=a.addr, extra=extra + " --num_blocks 2")).wait()
    c = None
    try:
        assert (a.srv.ex.start, a.srv.ex.end) == (1, 2) and (b.srv.ex.start, b.srv.ex.end) == (2, 4)
        assert a.srv.throughput > b.srv.throughput > 0, (a.srv.throughput, b.srv.throughput)
        # the network term came from a measured link, not the 100 Mbit/s constant
        assert a.srv.link_mbps is not None and b.srv.link_mbps is not None and b.srv.link_mbps > 100
        assert wait_for(lambda: len(get_remote_module_infos(a.dht, MODEL, 4)) >= 3)
        c = ServerThread(server_argv(MODEL, "1", 1, peers=a.addr, extra=extra + " --num_blocks 1")).wait()
        assert c.srv.ex.start in (2, 3), (c.srv.ex.start, a.srv.throughput, b.srv.throughput)
    finally:
        for s in (a, b, c):
            if s is not None:
                s.close()
