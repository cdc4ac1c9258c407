"""Session placement helpers for replicated pipelines.

The round-1 static RCCL pipeline harness that lived here is superseded by the
continuous-batching serving engine (``parallel/engine.py``) on device channels
(``parallel/channel.py``) and the replica front end (``parallel/router.py``); what remains
is the throughput-proportional split of a batch of sessions over replicas (the
load_balancing.py rule re-expressed for whole pipelines, reference
src/load_balancing.py:212-244), used by ``bench.py --replicas`` and the router's failover.
"""
from __future__ import annotations

from typing import List, Sequence


def assign_sessions(n_sessions: int, throughputs: Sequence[float]) -> List[int]:
    """Replica index for each of ``n_sessions`` new sessions, proportional to replica
    throughput (largest-remainder rounding; ties to the lower index)."""
    tp = [max(float(t), 0.0) for t in throughputs]
    tot = sum(tp)
    if tot <= 0:
        tp, tot = [1.0] * len(tp), float(len(tp))
    quota = [n_sessions * t / tot for t in tp]
    base = [int(q) for q in quota]
    rem = n_sessions - sum(base)
    order = sorted(range(len(tp)), key=lambda i: (-(quota[i] - base[i]), i))
    for i in order[:rem]:
        base[i] += 1
    out: List[int] = []
    for r, n in enumerate(base):
        out.extend([r] * n)
    return out
