"""Session placement helpers for replicated pipelines.

The round-1 static RCCL pipeline harness that lived here is superseded by the
continuous-batching serving engine (``parallel/engine.py``) on device channels
(``parallel/channel.py``) and the replica front end (``parallel/router.py``); what remains
is the throughput-proportional split of a batch of sessions over replicas (the
load_balancing.py rule re-expressed for whole pipelines, reference
src/load_balancing.py:212-244), used by ``bench.py --replicas`` and the router's failover.
"""
from __future__ import annotations

from typing import List, Optional, Sequence


def assign_sessions(n_sessions: int, throughputs: Sequence[float], capacity: Optional[int] = None) -> List[int]:
    """Replica index for each of ``n_sessions`` new sessions, proportional to replica
    throughput (largest-remainder rounding; ties to the lower index).

    ``capacity``: most sessions one replica can hold; a replica's overflow is re-split over the
    replicas with room left (in proportion to their throughput), so no session is dropped
    while any replica has a free slot."""
    if capacity is not None:
        cap = [int(capacity)] * len(throughputs)
        counts = [0] * len(throughputs)
        left = n_sessions
        while left > 0:
            open_ = [r for r in range(len(cap)) if counts[r] < cap[r]]
            if not open_:
                raise ValueError(f"{n_sessions} sessions exceed {len(cap)} replicas x capacity {capacity}")
            share = assign_sessions(left, [throughputs[r] for r in open_])
            for j, r in enumerate(open_):
                take = min(share.count(j), cap[r] - counts[r])
                counts[r] += take
                left -= take
        return [r for r, n in enumerate(counts) for _ in range(n)]
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
