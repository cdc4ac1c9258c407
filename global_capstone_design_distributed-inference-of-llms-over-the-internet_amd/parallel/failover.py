"""Replica failover for single-node pipelines (BASELINE config "... fault-tolerance replica
failover"; SURVEY §7.5 "Fault tolerance over RCCL").

Over the swarm transport a failed hop is replayed from the client's per-hop input history
(``rpc_transport.RpcTransport``, reference src/rpc_transport.py:587-712).  Inside one node the
replicas are whole RCCL pipelines (``parallel.pipeline``), and a dead rank poisons its
replica's communicator, so recovery works one level up:

* a ``ReplicaRouter`` owns the session -> replica map (throughput-proportional placement,
  ``pipeline.assign_sessions``) and each session's TOKEN history (prompt + generated ids):
  tokens are all a replica needs to rebuild its KV, and they are tiny compared with the
  hidden-state history the swarm client keeps;
* ``fail(replica)`` marks it dead, re-places its sessions on the survivors (again by
  throughput) and returns a ``ReplayPlan`` per session: re-prefill prompt + generated
  tokens on the new replica (recompute-from-tokens, the SURVEY's "recompute from tokens at
  stage 0"), after which decoding resumes exactly where it stopped;
* ``heartbeat`` / ``expired`` give a timeout-based failure detector over per-replica
  progress stamps (the RCCL analogue of the registry's TTL expiry).

The router is transport-agnostic; ``tests/test_failover.py`` drives it with two CPU
executors standing in for replicas and checks that a failed-over session produces exactly
the tokens an uninterrupted one does.
"""
from __future__ import annotations

import dataclasses
import time
from typing import Dict, List, Optional, Sequence

from .pipeline import assign_sessions


@dataclasses.dataclass
class ReplayPlan:
    session_id: str
    replica: int
    tokens: List[int]  # prompt + generated ids to re-prefill (the next input is tokens[-1]'s successor)


class ReplicaRouter:
    def __init__(self, n_replicas: int, throughputs: Optional[Sequence[float]] = None, timeout_s: float = 10.0):
        self.n = int(n_replicas)
        self.throughput = list(throughputs) if throughputs is not None else [1.0] * self.n
        self.alive = [True] * self.n
        self.timeout_s = float(timeout_s)
        self.last_beat = [time.monotonic()] * self.n
        self.placement: Dict[str, int] = {}
        self.history: Dict[str, List[int]] = {}

    # ------------------------------------------------------------------ placement
    def live(self) -> List[int]:
        return [r for r in range(self.n) if self.alive[r]]

    def place(self, session_ids: Sequence[str], prompts: Sequence[Sequence[int]]) -> Dict[str, int]:
        live = self.live()
        if not live:
            raise RuntimeError("no live replica")
        reps = assign_sessions(len(session_ids), [self.throughput[r] for r in live])
        out = {}
        for sid, p, k in zip(session_ids, prompts, reps):
            self.placement[sid] = live[k]
            self.history[sid] = list(int(t) for t in p)
            out[sid] = live[k]
        return out

    def place_one(self, session_id: str, prompt: Sequence[int]) -> int:
        """Online placement of ONE new session: the live replica with the lowest
        throughput-normalised load after adding it (ties to the lower index)."""
        live = self.live()
        if not live:
            raise RuntimeError("no live replica")
        load: Dict[int, int] = {}
        for r in self.placement.values():
            load[r] = load.get(r, 0) + 1
        best = min(live, key=lambda k: ((load.get(k, 0) + 1) / max(float(self.throughput[k]), 1e-9), k))
        self.placement[session_id] = best
        self.history[session_id] = [int(t) for t in prompt]
        return best

    def record(self, session_id: str, token: int) -> None:
        self.history[session_id].append(int(token))

    def sessions_on(self, replica: int) -> List[str]:
        return [s for s, r in self.placement.items() if r == replica]

    # ------------------------------------------------------------------ failure handling
    def heartbeat(self, replica: int, now: Optional[float] = None) -> None:
        self.last_beat[replica] = time.monotonic() if now is None else now

    def expired(self, now: Optional[float] = None) -> List[int]:
        now = time.monotonic() if now is None else now
        return [r for r in self.live() if now - self.last_beat[r] > self.timeout_s]

    def fail(self, replica: int) -> List[ReplayPlan]:
        """Mark ``replica`` dead and move its sessions to survivors (throughput-proportional)."""
        if not self.alive[replica]:
            return []
        self.alive[replica] = False
        orphans = sorted(self.sessions_on(replica))
        live = self.live()
        if orphans and not live:
            raise RuntimeError("all replicas failed")
        reps = assign_sessions(len(orphans), [self.throughput[r] for r in live]) if orphans else []
        plans = []
        for sid, k in zip(orphans, reps):
            self.placement[sid] = live[k]
            plans.append(ReplayPlan(sid, live[k], list(self.history[sid])))
        return plans

    def add_replica(self, throughput: float = 1.0) -> int:
        """A new (e.g. rebuilt) replica joins; returns its index."""
        self.n += 1
        self.throughput.append(float(throughput))
        self.alive.append(True)
        self.last_beat.append(time.monotonic())
        return self.n - 1

    def close(self, session_id: str) -> None:
        self.placement.pop(session_id, None)
        self.history.pop(session_id, None)
