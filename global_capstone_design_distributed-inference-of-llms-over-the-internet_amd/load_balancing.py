"""Swarm load balancing: block selection for joining servers and periodic rebalancing.

Semantics of the reference's Petals-paper rules (reference src/load_balancing.py:17-366):

* ``compute_spans``: module records -> one contiguous span per peer (a peer's span
  throughput is the MIN over its blocks; a gap starts a new span and, as in the
  reference, the peer's LAST span is the one kept).
* ``compute_throughputs``: per-block sum of span throughputs.
* rule 1, ``choose_best_blocks``: a joining server takes the window of ``num_blocks``
  blocks, starting at or after ``min_block``, that minimises (min, mean, start) of the
  current per-block throughput - it fills the weakest region first.
* rule 2, ``should_choose_other_blocks``: remove yourself, re-place yourself, then let
  every server (shuffled, <= 10 rounds) re-place itself; if the swarm's bottleneck
  throughput would improve so that initial/new < balance_quality, move.
  ``balance_quality > 1`` forces a move (debug switch, as in the reference).

The window search is vectorised (sliding min / mean over all starts at once) instead of a
Python loop over windows.  Peer ids are plain strings.
"""
from __future__ import annotations

import dataclasses
import enum
import logging
from typing import Dict, List, Optional, Sequence

import numpy as np

logger = logging.getLogger(__name__)
_EPS = 1e-3


class ServerState(enum.Enum):
    JOINING = "joining"
    ONLINE = "online"
    OFFLINE = "offline"


_STATE_RANK = {ServerState.JOINING: 0, ServerState.ONLINE: 1, ServerState.OFFLINE: 2}


@dataclasses.dataclass
class ServerInfo:
    peer_id: str
    state: ServerState
    throughput: float
    start_block: int
    end_block: int
    server_address: Optional[str] = None

    @property
    def num_blocks(self) -> int:
        return self.end_block - self.start_block


@dataclasses.dataclass
class RemoteModuleInfo:
    uid: str  # "block_<i>"
    server_info: Optional[ServerInfo] = None

    @property
    def block_index(self) -> int:
        return int(self.uid.rsplit("_", 1)[-1])


@dataclasses.dataclass
class RemoteSpanInfo:
    peer_id: str
    start: int
    end: int
    length: int
    throughput: float

    def __post_init__(self):
        self.length = self.end - self.start

    def move_to(self, new_start: int) -> None:
        self.start = new_start
        self.end = new_start + self.length


def compute_spans(module_infos: Sequence[RemoteModuleInfo],
                  min_state: ServerState = ServerState.JOINING) -> Dict[str, RemoteSpanInfo]:
    per_peer: Dict[str, Dict[int, float]] = {}
    floor = _STATE_RANK[min_state]
    for mi in module_infos:
        si = mi.server_info
        if si is None or _STATE_RANK.get(si.state, 99) < floor:
            continue
        try:
            b = mi.block_index
        except ValueError:
            logger.warning(f"bad module uid {mi.uid!r}")
            continue
        blocks = per_peer.setdefault(str(si.peer_id), {})
        blocks[b] = min(blocks.get(b, si.throughput), si.throughput)
    spans: Dict[str, RemoteSpanInfo] = {}
    for pid, blocks in per_peer.items():
        idx = sorted(blocks)
        # split into maximal runs of consecutive block ids; the last run is the peer's span
        breaks = [i for i in range(1, len(idx)) if idx[i] != idx[i - 1] + 1]
        s = breaks[-1] if breaks else 0
        run = idx[s:]
        spans[pid] = RemoteSpanInfo(pid, run[0], run[-1] + 1, len(run), float(min(blocks[b] for b in run)))
    return spans


def compute_throughputs(spans: Dict[str, RemoteSpanInfo], total_blocks: int) -> np.ndarray:
    thr = np.zeros(total_blocks, dtype=np.float64)
    for pid in sorted(spans):
        sp = spans[pid]
        thr[max(sp.start, 0):min(sp.end, total_blocks)] += sp.throughput
    return thr


def _choose_best_start(throughputs: np.ndarray, num_blocks: int, min_block: int = 0) -> int:
    n = len(throughputs)
    if n < num_blocks:
        return max(0, int(min_block))
    last = n - num_blocks
    lo = int(max(0, min(min_block, last)))
    win = np.lib.stride_tricks.sliding_window_view(np.asarray(throughputs, dtype=np.float64), num_blocks)[lo:last + 1]
    mins, means = win.min(axis=1), win.mean(axis=1)
    starts = np.arange(lo, last + 1)
    order = np.lexsort((starts, means, mins))  # primary: min, then mean, then start
    return int(starts[order[0]])


def _infer_total(module_infos: Sequence[RemoteModuleInfo], default: int) -> int:
    best = -1
    for mi in module_infos:
        try:
            best = max(best, mi.block_index)
        except ValueError:
            pass
    return best + 1 if best > 0 else default


def choose_best_blocks(num_blocks: int, module_infos: Sequence[RemoteModuleInfo],
                       total_blocks: Optional[int] = None, min_block: int = 0) -> List[int]:
    if total_blocks is None:
        total_blocks = _infer_total(module_infos, num_blocks)
    thr = compute_throughputs(compute_spans(module_infos, ServerState.JOINING), total_blocks)
    start = _choose_best_start(thr, num_blocks, min_block)
    return list(range(start, start + num_blocks))


def should_choose_other_blocks(local_peer_id, module_infos: Sequence[RemoteModuleInfo],
                               balance_quality: float = 0.75, total_blocks: Optional[int] = None,
                               min_block: int = 0, rng: Optional[np.random.Generator] = None) -> bool:
    if balance_quality > 1.0:
        return True
    if total_blocks is None:
        total_blocks = _infer_total(module_infos, 32)
    spans = compute_spans(module_infos, ServerState.JOINING)
    thr = compute_throughputs(spans, total_blocks)
    initial = float(thr.min()) if len(thr) else 0.0
    me = spans.get(str(local_peer_id))
    if me is None:
        logger.warning(f"local peer {str(local_peer_id)[:16]} not among {len(spans)} spans")
        return False
    a, b = max(0, min(me.start, len(thr) - 1)), min(me.end, len(thr))
    if b > a:
        thr[a:b] -= me.throughput * (1 + _EPS)
    if initial > _EPS and thr.min() <= 0:
        return False  # leaving would uncover a block
    new_start = _choose_best_start(thr, me.length, min_block)
    if new_start == me.start:
        return False
    thr[me.start:me.end] += me.throughput * _EPS
    me.move_to(new_start)
    thr[me.start:me.end] += me.throughput
    rng = rng or np.random.default_rng()
    for _ in range(10):
        moved = False
        order = list(spans)
        rng.shuffle(order)
        for pid in order:
            sp = spans[pid]
            thr[sp.start:sp.end] -= sp.throughput * (1 + _EPS)
            cand = _choose_best_start(thr, sp.length, min_block)
            thr[sp.start:sp.end] += sp.throughput * _EPS
            if cand != sp.start:
                sp.move_to(cand)
                moved = True
            thr[sp.start:sp.end] += sp.throughput
        if not moved:
            break
    new = float(thr.min())
    if new < initial or new < _EPS:
        return False
    quality = initial / new
    logger.info(f"Swarm balance quality: {quality * 100:.1f}% (initial={initial:.2f}, new={new:.2f})")
    return quality < balance_quality - _EPS
