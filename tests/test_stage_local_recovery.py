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
