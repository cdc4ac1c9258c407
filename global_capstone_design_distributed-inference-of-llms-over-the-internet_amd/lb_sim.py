"""Swarm load-balancing simulator (the Petals paper's Section E / Appendix D experiment).

The reference ships the balancing rules (src/load_balancing.py:212-366) and a manual 4-server
recipe (scripts/elice_test_load_balancing.sh) but no way to measure how good the placement is.
This module replays a swarm's life -- servers with heterogeneous throughput join one by one,
some leave -- through the SAME functions the servers run (``choose_best_blocks``,
``should_choose_other_blocks`` on registry-shaped ``RemoteModuleInfo`` lists), under three
policies:

* ``none``      joining servers take a uniformly random window (no balancing);
* ``new``       rule 1 only: joining servers take the weakest window, nobody moves later;
* ``full``      rule 1 + rule 2: after every join / leave, each server (random order) runs the
                periodic ``should_choose_other_blocks`` check and re-joins if it says so.

Swarm throughput = min over blocks of the summed throughput of the servers holding that block
(a pipeline is as fast as its least-served block). The upper bound spreads every server's
capacity fractionally: ``sum(thr_i * blocks_i) / total_blocks``.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

import numpy as np

from .load_balancing import (RemoteModuleInfo, ServerInfo, ServerState, choose_best_blocks,
                             should_choose_other_blocks)

POLICIES = ("none", "new", "full")


@dataclasses.dataclass
class SimServer:
    peer_id: str
    throughput: float
    num_blocks: int
    start: int = 0


def module_infos(servers: Dict[str, SimServer], total: int) -> List[RemoteModuleInfo]:
    """Registry view of the swarm: one record per (block, server), as get_remote_module_infos builds."""
    out = []
    for s in servers.values():
        si = ServerInfo(s.peer_id, ServerState.ONLINE, s.throughput, s.start, s.start + s.num_blocks)
        out.extend(RemoteModuleInfo(f"block_{b}", si) for b in range(s.start, min(s.start + s.num_blocks, total)))
    return out


def swarm_throughput(servers: Dict[str, SimServer], total: int) -> float:
    thr = np.zeros(total)
    for s in servers.values():
        thr[s.start:s.start + s.num_blocks] += s.throughput
    return float(thr.min()) if total else 0.0


def upper_bound(servers: Dict[str, SimServer], total: int) -> float:
    return sum(s.throughput * min(s.num_blocks, total) for s in servers.values()) / total


def _join(servers, s: SimServer, total, policy, rng):
    if policy == "none":
        s.start = int(rng.integers(0, total - s.num_blocks + 1))
    else:
        s.start = choose_best_blocks(s.num_blocks, module_infos(servers, total), total)[0]
    servers[s.peer_id] = s


def _rebalance(servers, total, rng, balance_quality, max_rounds=8) -> int:
    moves = 0
    for _ in range(max_rounds):
        moved = False
        for pid in rng.permutation(sorted(servers)):
            if should_choose_other_blocks(pid, module_infos(servers, total), balance_quality, total, rng=rng):
                s = servers.pop(pid)  # leave, then re-join at the best window
                s.start = choose_best_blocks(s.num_blocks, module_infos(servers, total), total)[0]
                servers[pid] = s
                moves += 1
                moved = True
        if not moved:
            break
    return moves


def simulate(policy: str, n_servers: int = 40, total_blocks: int = 80, blocks_range: Tuple[int, int] = (8, 24),
             thr_range: Tuple[float, float] = (1.0, 10.0), leave_frac: float = 0.25, seed: int = 0,
             balance_quality: float = 0.75) -> dict:
    """Join ``n_servers`` one at a time, then remove ``leave_frac`` of them at random.

    Returns throughput / upper-bound after all joins and after the departures, plus the number of
    rule-2 moves."""
    if policy not in POLICIES:
        raise ValueError(f"policy must be one of {POLICIES}")
    rng = np.random.default_rng(seed)
    servers: Dict[str, SimServer] = {}
    moves = 0
    for i in range(n_servers):
        s = SimServer(f"peer{i:03d}", float(rng.uniform(*thr_range)),
                      int(rng.integers(blocks_range[0], blocks_range[1] + 1)))
        _join(servers, s, total_blocks, policy, rng)
        if policy == "full":
            moves += _rebalance(servers, total_blocks, rng, balance_quality)
    after_join = swarm_throughput(servers, total_blocks) / upper_bound(servers, total_blocks)
    for pid in rng.choice(sorted(servers), size=int(leave_frac * n_servers), replace=False):
        servers.pop(str(pid))
        if policy == "full":
            moves += _rebalance(servers, total_blocks, rng, balance_quality)
    after_leave = swarm_throughput(servers, total_blocks) / upper_bound(servers, total_blocks)
    return {"policy": policy, "after_join": after_join, "after_leave": after_leave, "moves": moves,
            "servers": len(servers)}


def compare(seeds=range(5), **kw) -> Dict[str, dict]:
    """Mean efficiency (fraction of the upper bound) per policy over several swarms."""
    out = {}
    for p in POLICIES:
        rs = [simulate(p, seed=s, **kw) for s in seeds]
        out[p] = {k: float(np.mean([r[k] for r in rs])) for k in ("after_join", "after_leave", "moves")}
    return out


def main(argv: Optional[List[str]] = None) -> None:
    import argparse
    import json

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--servers", type=int, default=40)
    ap.add_argument("--total_blocks", type=int, default=80)
    ap.add_argument("--min_blocks", type=int, default=8)
    ap.add_argument("--max_blocks", type=int, default=24)
    ap.add_argument("--leave_frac", type=float, default=0.25)
    ap.add_argument("--seeds", type=int, default=5)
    ap.add_argument("--balance_quality", type=float, default=0.75)
    a = ap.parse_args(argv)
    res = compare(range(a.seeds), n_servers=a.servers, total_blocks=a.total_blocks,
                  blocks_range=(a.min_blocks, a.max_blocks), leave_frac=a.leave_frac,
                  balance_quality=a.balance_quality)
    for p, r in res.items():
        print(f"{p:>5}: {100 * r['after_join']:5.1f}% of upper bound after joins, "
              f"{100 * r['after_leave']:5.1f}% after {int(100 * a.leave_frac)}% left  (moves {r['moves']:.1f})")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
