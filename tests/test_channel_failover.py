"""Same-node fast path: replica routing and failover behind the CLI client.

Reference: the client routes each session over whatever replicas the registry holds and, when
a hop fails, excludes the peer, rediscovers and replays (src/rpc_transport.py:393-501,
587-712; scripts/test_fault_tolerance.py + kill_stage.py are its manual procedure).  Here the
client heads one device channel per disjoint same-node route (``--device_channel on`` forces
the channel over gloo on CPU), the replica front end places sessions, and a SIGKILLed server
makes its pipeline fail over: dead servers are found over TCP, the unfinished sessions are
re-prefilled from their token history on the surviving replica, and - sampling being seeded by
(session seed, position) - every session's tokens equal an uninterrupted run's.
"""
import json
import os
import re
import signal
import subprocess
import sys
import time

import pytest
import torch

from src import main as M

from .swarm_utils import client_args

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODEL = "tiny-llama"
SPLITS = "1,2"


def _start(i, tmp_path, stage, peers=None):
    log = tmp_path / f"s{i}.log"
    cmd = [sys.executable, "-m", "src.main", "--model", MODEL, "--splits", SPLITS, "--stage", str(stage),
           "--dht_port", "0", "--rpc_port", "0", "--host", "127.0.0.1", "--device", "cpu", "--kv_cache_gb", "0.05",
           "--max_sessions", "32", "--request_timeout", "10"]
    if peers:
        cmd += ["--dht_initial_peers", peers]
    p = subprocess.Popen(cmd, cwd=ROOT, stdout=open(log, "w"), stderr=subprocess.STDOUT)
    t0 = time.time()
    while time.time() - t0 < 120:
        txt = log.read_text()
        m = re.search(r"handlers registered .*peer (\S+),", txt)
        d = re.search(r"DHT visible multiaddrs: \['([^']+)'", txt)
        if m and d:
            return p, m.group(1), d.group(1)
        assert p.poll() is None, txt[-2000:]
        time.sleep(0.2)
    raise TimeoutError(txt[-2000:])


@pytest.fixture
def swarm(tmp_path):
    """2 replicas x 2 server stages (4 server processes): stage 1 = block [1, 2), stage 2 =
    blocks [2, L) + head; the client holds block 0."""
    procs = {}
    p, pid, maddr = _start(0, tmp_path, 1)
    procs[pid] = (p, 1)
    for i, stage in ((1, 1), (2, 2), (3, 2)):
        p, pid, _ = _start(i, tmp_path, stage, maddr)
        procs[pid] = (p, stage)
    yield procs, maddr
    for p, _ in procs.values():
        if p.poll() is None:
            p.terminate()
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()


def _wait_routes(maddr, n=2, timeout=30):
    from src.rpc_transport import RpcTransport
    from src.dht_utils import get_stage_key

    tx = RpcTransport("cpu", 0, [maddr], stage_keys=[get_stage_key(1), get_stage_key(2)])
    t0 = time.time()
    try:
        while time.time() - t0 < timeout:
            if len(tx.channel_routes("cpu", same_node=False, wait_s=0.0)) >= n:
                return True
            time.sleep(0.3)
        return False
    finally:
        tx.shutdown()


ARGS = ("--device_channel on --num_sessions 8 --max_new_tokens 20 --temperature 1.0 --request_timeout 10 "
        "--max_sessions 16")


@pytest.mark.timeout(300)
def test_two_replica_routes_sigkill_one_server_tokens_exact(swarm, caplog):
    procs, maddr = swarm
    assert _wait_routes(maddr)
    cuts = [1, 2]
    ref = []
    with caplog.at_level("INFO", logger="src.main"):
        M.run_rank0(client_args(MODEL, SPLITS, maddr, ARGS), torch.device("cpu"), cuts, results=ref)
    assert "x 2 replica(s)" in caplog.text  # both disjoint routes carried sessions
    assert len(ref) == 8 and all(len(g) == 20 for g in ref)
    caplog.clear()

    killed = []
    count = [0]

    def on_token(req, tok):
        count[0] += 1
        if count[0] == 40 and not killed:  # mid-decode: every session has ~5 of its 20 tokens
            victim = next(pid for pid, (p, st) in procs.items() if st == 2)
            procs[victim][0].send_signal(signal.SIGKILL)
            procs[victim][0].wait(10)
            killed.append(victim)

    out = []
    with caplog.at_level("INFO", logger="src.main"):
        M.run_rank0(client_args(MODEL, SPLITS, maddr, ARGS), torch.device("cpu"), cuts, on_token=on_token,
                    results=out)
    assert killed, "the fault was never injected"
    assert "replica failure(s) recovered" in caplog.text, caplog.text[-3000:]
    assert out == ref


@pytest.mark.timeout(300)
def test_cli_process_client_survives_sigkill(swarm, tmp_path):
    """``python -m src.main --stage 0`` as its own process: a stage-1 server is SIGKILLed while
    the client decodes (first progress line); the client exits 0 with every session complete
    and the same tokens as an uninterrupted run."""
    procs, maddr = swarm
    assert _wait_routes(maddr)

    def client(tag, kill=None):
        dump = tmp_path / f"{tag}.json"
        log = tmp_path / f"{tag}.log"
        cmd = [sys.executable, "-m", "src.main", "--model", MODEL, "--splits", SPLITS, "--stage", "0", "--device",
               "cpu", "--dht_initial_peers", maddr, "--kv_cache_gb", "0.05", "--max_sessions", "16",
               "--dump_tokens", str(dump)] + ARGS.replace("--max_new_tokens 20", "--max_new_tokens 120").split()
        p = subprocess.Popen(cmd, cwd=ROOT, stdout=open(log, "w"), stderr=subprocess.STDOUT)
        if kill is not None:
            t0 = time.time()
            while time.time() - t0 < 120 and p.poll() is None:
                if "progress:" in log.read_text():
                    kill()
                    break
                time.sleep(0.02)
        p.wait(240)
        txt = log.read_text()
        assert p.returncode == 0, txt[-3000:]
        return json.loads(dump.read_text()), txt

    ref, _ = client("ref")
    victim = next(pid for pid, (p, st) in procs.items() if st == 1)
    got, txt = client("kill", lambda: procs[victim][0].send_signal(signal.SIGKILL))
    assert procs[victim][0].wait(10) is not None
    assert len(got) == 8 and all(v["finish"] in ("length", "eos", "repeat") for v in got.values()), got
    assert "recovered" in txt, txt[-3000:]
    assert got == ref


@pytest.mark.timeout(300)
def test_single_route_rebuilt_through_spare_server(tmp_path, caplog):
    """One replica only (``--max_replicas 1``) and a spare tail server: the tail in use is SIGKILLed
    mid-decode, so no surviving replica can take the sessions - ``recover()`` (main.py
    ``_run_rank0_channel``) finds the dead server over TCP, opens a new channel through the
    surviving stage-1 server and the spare, and the sessions are re-prefilled there; every
    session completes with the uninterrupted run's tokens."""
    procs = {}
    p, pid, maddr = _start(0, tmp_path, 1)
    procs[pid] = (p, 1, tmp_path / "s0.log")
    for i in (1, 2):
        p, pid, _ = _start(i, tmp_path, 2, maddr)
        procs[pid] = (p, 2, tmp_path / f"s{i}.log")
    try:
        assert _wait_routes(maddr, n=1)
        args = ARGS + " --max_replicas 1"
        ref = []
        M.run_rank0(client_args(MODEL, SPLITS, maddr, args), torch.device("cpu"), [1, 2], results=ref)
        assert len(ref) == 8 and all(len(g) == 20 for g in ref)
        caplog.clear()
        killed = []
        count = [0]
        tails = [(pid, p, log) for pid, (p, st, log) in procs.items() if st == 2]
        opens0 = {pid: log.read_text().count("open as rank") for pid, p, log in tails}

        def on_token(req, tok):
            count[0] += 1
            if count[0] == 40 and not killed:
                # the tail the CURRENT channel uses: the one that opened a channel since the reference run
                now = {pid: log.read_text().count("open as rank") for pid, p, log in tails}
                victim = next(t for t in tails if now[t[0]] > opens0[t[0]])
                victim[1].send_signal(signal.SIGKILL)
                victim[1].wait(10)
                killed.append(victim[0])

        out = []
        with caplog.at_level("INFO", logger="src.main"):
            M.run_rank0(client_args(MODEL, SPLITS, maddr, args), torch.device("cpu"), [1, 2], on_token=on_token,
                        results=out)
        assert killed, "the fault was never injected"
        assert "rebuilt a pipeline" in caplog.text, caplog.text[-3000:]
        assert "replica failure(s) recovered" in caplog.text
        assert out == ref
    finally:
        for p, _, _ in procs.values():
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(10)
                except subprocess.TimeoutExpired:
                    p.kill()
