"""Stage-local recovery of a device-channel pipeline (``--replay_cache``).

Reference: when a hop fails, the client re-routes ONLY that hop and replays the hop's cached
inputs to the replacement server (src/rpc_transport.py:587-712 ``_replay_past_inputs``); the
servers before and after it keep their per-session KV.  Here every non-tail stage keeps its output
rows in a ``ReplayCache``; when one server of a single-replica pipeline is SIGKILLed, ``recover()``
swaps in a spare for that hop only, the surviving servers adopt their sessions' KV into the new
channel, the stage before the spare replays its cached rows (one prefill on the spare) and decoding
resumes from each session's last token - no session is re-prefilled.  Sampling is seeded by
(session seed, position), so the tokens equal an uninterrupted run's.
"""
import signal

import pytest
import torch

from src import main as M

from .swarm_utils import client_args
from .test_channel_failover import ARGS, _start, _wait_routes


@pytest.mark.timeout(300)
@pytest.mark.parametrize("victim_stage", [2, 1])
def test_only_the_dead_stage_is_rebuilt(tmp_path, caplog, victim_stage):
    procs = {}
    p, pid, maddr = _start(0, tmp_path, 1)
    procs[pid] = (p, 1, tmp_path / "s0.log")
    stages = (2, 2) if victim_stage == 2 else (1, 2)  # a spare of the victim's stage
    for i, st in enumerate(stages, start=1):
        p, pid, _ = _start(i, tmp_path, st, maddr)
        procs[pid] = (p, st, tmp_path / f"s{i}.log")
    try:
        assert _wait_routes(maddr, n=1)
        args = ARGS + " --max_replicas 1 --replay_cache"
        ref = []
        M.run_rank0(client_args("tiny-llama", "1,2", maddr, args), torch.device("cpu"), [1, 2], results=ref)
        assert len(ref) == 8 and all(len(g) == 20 for g in ref)
        caplog.clear()
        cands = [(pid, p, log) for pid, (p, st, log) in procs.items() if st == victim_stage]
        opens0 = {pid: log.read_text().count("open as rank") for pid, _, log in cands}
        killed, count = [], [0]

        def on_token(req, tok):
            count[0] += 1
            if count[0] == 40 and not killed:  # mid-decode: every session has ~5 of its 20 tokens
                now = {pid: log.read_text().count("open as rank") for pid, _, log in cands}
                victim = next(c for c in cands if now[c[0]] > opens0[c[0]])  # the one in use now
                victim[1].send_signal(signal.SIGKILL)
                victim[1].wait(10)
                killed.append(victim[0])

        out = []
        with caplog.at_level("INFO", logger="src.main"):
            M.run_rank0(client_args("tiny-llama", "1,2", maddr, args), torch.device("cpu"), [1, 2],
                        on_token=on_token, results=out)
        assert killed, "the fault was never injected"
        assert f"(stage {victim_stage} replaced, the other stages keep their KV)" in caplog.text, caplog.text[-3000:]
        assert "8 session(s) resumed in place, 0 re-prefilled" in caplog.text, caplog.text[-3000:]
        assert out == ref
        logs = {pid: log.read_text() for pid, (p, st, log) in procs.items() if pid not in killed}
        spare = [t for t in logs.values() if "replay: rebuilt the KV of 8 session(s)" in t]
        assert len(spare) == 1, "exactly one server (the spare) rebuilds KV"
        if victim_stage == 2:  # the surviving stage-1 server adopted its KV and replayed its rows
            assert sum("replay: adopted 8 session(s)" in t for t in logs.values()) == 1
    finally:
        for p, _, _ in procs.values():
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(10)
                except Exception:  # noqa: BLE001
                    p.kill()


def _start_gpu(i, tmp_path, stage, peers, model, splits):
    """A stage server process on the one MI355X (payloads host-staged over gloo: RCCL refuses two
    ranks on one device)."""
    import os
    import re
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    log = tmp_path / f"g{i}.log"
    cmd = [sys.executable, "-m", "src.main", "--model", model, "--splits", splits, "--stage", str(stage),
           "--dht_port", "0", "--rpc_port", "0", "--host", "127.0.0.1", "--device", "cuda:0", "--dtype", "bf16",
           "--kv_cache_gb", "0.25", "--max_sessions", "32", "--request_timeout", "30"]
    if peers:
        cmd += ["--dht_initial_peers", peers]
    env = dict(os.environ, MPAMD_CHANNEL_DATA="gloo", MPAMD_GEMM_AUTOTUNE="0")
    p = subprocess.Popen(cmd, cwd=root, stdout=open(log, "w"), stderr=subprocess.STDOUT, env=env)
    t0 = time.time()
    while time.time() - t0 < 240:
        txt = log.read_text()
        m = re.search(r"handlers registered .*peer (\S+),", txt)
        d = re.search(r"DHT visible multiaddrs: \['([^']+)'", txt)
        if m and d:
            return p, m.group(1), d.group(1)
        assert p.poll() is None, txt[-2000:]
        time.sleep(0.3)
    raise TimeoutError(txt[-2000:])


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_stage_local_recovery_one_gpu(tmp_path, caplog, monkeypatch):
    """``--replay_cache`` on the GPU path: client + 3 stage servers on one MI355X, the tail in use is
    SIGKILLed mid-decode; its spare rebuilds the KV of every session from the replayed rows with
    ONE prefill (hipBLASLt + FA2 prefill kernels, whereas the lost KV was written by the decode
    kernels), the surviving middle stage adopts its KV.  Asserted: 0 sessions re-prefilled, exactly
    one server rebuilt KV, every session completes its 20 tokens, and every token drawn before the
    failure equals the uninterrupted run's.  (After the rebuild a bf16 prefill KV differs from the
    decode-written one in its last bits, so later tokens may diverge: that contract is the
    teacher-forced logit tolerance of test_failover_gpu.py.)"""
    import torch

    model, splits = "small-llama", "2,4"
    monkeypatch.setenv("MPAMD_CHANNEL_DATA", "gloo")
    monkeypatch.setenv("MPAMD_GEMM_AUTOTUNE", "0")
    procs = {}
    p, pid, maddr = _start_gpu(0, tmp_path, 1, None, model, splits)
    procs[pid] = (p, 1, tmp_path / "g0.log")
    for i, st in enumerate((2, 2), start=1):  # the tail and its spare
        p, pid, _ = _start_gpu(i, tmp_path, st, maddr, model, splits)
        procs[pid] = (p, st, tmp_path / f"g{i}.log")
    try:
        assert _wait_routes(maddr, n=1)
        args = ARGS + " --max_replicas 1 --replay_cache --dtype bf16"
        dev = torch.device("cuda:0")
        ref = []
        M.run_rank0(client_args(model, splits, maddr, args), dev, [2, 4], results=ref)
        assert len(ref) == 8 and all(len(g) == 20 for g in ref)
        caplog.clear()
        cands = [(pid, p, log) for pid, (p, st, log) in procs.items() if st == 2]
        opens0 = {pid: log.read_text().count("open as rank") for pid, _, log in cands}
        killed, count = [], [0]

        def on_token(req, tok):
            count[0] += 1
            if count[0] == 40 and not killed:  # every session has ~5 of its 20 tokens
                now = {pid: log.read_text().count("open as rank") for pid, _, log in cands}
                victim = next(c for c in cands if now[c[0]] > opens0[c[0]])
                victim[1].send_signal(signal.SIGKILL)
                victim[1].wait(10)
                killed.append(victim[0])

        out = []
        with caplog.at_level("INFO", logger="src.main"):
            M.run_rank0(client_args(model, splits, maddr, args), dev, [2, 4], on_token=on_token, results=out)
        assert killed, "the fault was never injected"
        assert "(stage 2 replaced, the other stages keep their KV)" in caplog.text, caplog.text[-3000:]
        assert "8 session(s) resumed in place, 0 re-prefilled" in caplog.text, caplog.text[-3000:]
        assert len(out) == 8 and all(len(g) == 20 for g in out)
        for got, want in zip(out, ref):  # tokens drawn before the failure (>= 3 per session) are untouched
            assert got[:3] == want[:3]
        logs = {pid: log.read_text() for pid, (p, st, log) in procs.items() if pid not in killed}
        assert sum("replay: rebuilt the KV of 8 session(s)" in t for t in logs.values()) == 1
        assert sum("replay: adopted 8 session(s)" in t for t in logs.values()) == 1
        same = sum(a == b for a, b in zip(out, ref))
        print(f"stage-local recovery on one GPU: 8 sessions resumed in place, identical end to end: {same}/8")
    finally:
        for p, _, _ in procs.values():
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(10)
                except Exception:  # noqa: BLE001
                    p.kill()
