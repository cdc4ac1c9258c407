"""Per-stage session table over the paged KV cache.

Reference: the stage handler keeps ``self._kv_cache[session_id]`` forever
(reference src/rpc_handler.py:70,266; "no eviction") and ignores
``max_length``.  Here a session owns a row of a block table and a list of KV pages;
``max_length`` is enforced, pages are returned on close, and idle sessions expire after
a TTL (``evict_expired``) so a crashed client cannot leak HBM.
"""
from __future__ import annotations

import dataclasses
import threading
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from .kv_cache import AllocationFailed, PagedKVCache, pages_needed


@dataclasses.dataclass
class SessionState:
    sid: str
    row: int
    max_length: int
    length: int = 0
    pages: List[int] = dataclasses.field(default_factory=list)
    created: float = dataclasses.field(default_factory=time.monotonic)
    last_used: float = dataclasses.field(default_factory=time.monotonic)
    generated: List[int] = dataclasses.field(default_factory=list)
    step: int = 0


class SessionManager:
    def __init__(self, cache: PagedKVCache, max_sessions: int = 256, max_seq_len: int = 4096,
                 ttl_seconds: float = 600.0):
        self.cache = cache
        self.page_size = cache.page_size
        self.max_sessions = max_sessions
        self.max_seq_len = max_seq_len
        self.max_pages = pages_needed(max_seq_len, cache.page_size)
        self.ttl = ttl_seconds
        self.table = np.full((max_sessions, self.max_pages), -1, dtype=np.int32)
        self.table_dev = torch.from_numpy(self.table.copy()).to(cache.device)
        self._dirty = False
        # double-buffered pinned staging: the H2D copy of a changed table is asynchronous and
        # stream-ordered before the step's kernels (a pageable copy_ would block the host until
        # the GPU drained every queued step); buffer k is reused only after its copy's event
        self._pinned = None
        if self.table_dev.is_cuda:
            self._pinned = [torch.empty(self.table.shape, dtype=torch.int32, pin_memory=True) for _ in range(2)]
            self._pin_ev = [None, None]
            self._pin_k = 0
        self._free_rows = list(range(max_sessions - 1, -1, -1))
        self.sessions: Dict[str, SessionState] = {}
        self.lock = threading.RLock()

    # ------------------------------------------------------------------ lifecycle
    def open(self, sid: str, max_length: Optional[int] = None) -> SessionState:
        with self.lock:
            if sid in self.sessions:
                return self.sessions[sid]
            if not self._free_rows:
                self.evict_expired()
            if not self._free_rows:
                raise AllocationFailed(f"too many concurrent sessions (max {self.max_sessions})")
            ml = min(int(max_length or self.max_seq_len), self.max_seq_len)
            s = SessionState(sid=sid, row=self._free_rows.pop(), max_length=ml)
            self.sessions[sid] = s
            return s

    def free_rows(self) -> int:
        """Session rows still available (several engines may share one table: the head's)."""
        return len(self._free_rows)

    def get(self, sid: str) -> Optional[SessionState]:
        return self.sessions.get(sid)

    def reset(self, sid: str) -> None:
        """Drop the session's cached tokens (prefill / replay restart) but keep its row."""
        with self.lock:
            s = self.sessions.get(sid)
            if s is None:
                return
            self.cache.allocator.free(s.pages)
            s.pages = []
            s.length = 0
            s.generated = []
            self.table[s.row, :] = -1
            self._dirty = True

    def close(self, sid: str) -> None:
        with self.lock:
            s = self.sessions.pop(sid, None)
            if s is None:
                return
            self.cache.allocator.free(s.pages)
            self.table[s.row, :] = -1
            self._dirty = True
            self._free_rows.append(s.row)

    def rename(self, src: str, dst: str) -> Optional[SessionState]:
        """Move session ``src`` (row, pages, length) to the key ``dst`` - a stage adopting the
        KV it held for a failed device channel into the channel that replaces it.  None if
        ``src`` is unknown; an existing ``dst`` is closed first."""
        with self.lock:
            s = self.sessions.pop(src, None)
            if s is None:
                return None
            self.close(dst)
            s.sid = dst
            s.last_used = time.monotonic()
            self.sessions[dst] = s
            return s

    def fork(self, src: str, dst: str, max_length: Optional[int] = None) -> SessionState:
        """``dst`` becomes a copy of ``src`` (its KV pages are copied on the device): the
        building block of beam search (upstream Petals reorders a session's hypotheses by
        ``hypo_ids``; here every hypothesis is a session and ``reorder`` forks them)."""
        with self.lock:
            s = self.sessions[src]
            d = self.open(dst, max_length or s.max_length)
            self.reset(dst)
            if s.pages:
                new = self.cache.allocator.alloc(len(s.pages))
                self.cache.copy_pages(s.pages, new)
                self.table[d.row, : len(new)] = new
                d.pages = list(new)
                self._dirty = True
            d.length = s.length
            d.generated = list(s.generated)
            d.last_used = time.monotonic()
            return d

    def reorder(self, sids: List[str], hypo_ids: List[int]) -> None:
        """Beam-search reorder: hypothesis i continues from hypothesis ``hypo_ids[i]``
        (upstream TransformerBackend ``hypo_ids``).  Sources are snapshotted first."""
        if list(hypo_ids) == list(range(len(sids))):
            return
        with self.lock:
            tmp = [f"__reorder_{i}_{sids[h]}" for i, h in enumerate(hypo_ids)]
            for t, h in zip(tmp, hypo_ids):
                self.fork(sids[h], t)
            for sid, t in zip(sids, tmp):
                self.fork(t, sid)
                self.close(t)

    def evict_expired(self, now: Optional[float] = None) -> int:
        now = time.monotonic() if now is None else now
        with self.lock:
            dead = [sid for sid, s in self.sessions.items() if now - s.last_used > self.ttl]
            for sid in dead:
                self.close(sid)
            return len(dead)

    # ------------------------------------------------------------------ pages
    def reserve(self, s: SessionState, total_len: int) -> None:
        """Make sure pages exist for positions [0, total_len)."""
        if total_len > s.max_length:
            raise ValueError(f"session {s.sid[:8]}: length {total_len} exceeds max_length {s.max_length}")
        need = pages_needed(total_len, self.page_size) - len(s.pages)
        if need > 0:
            with self.lock:
                try:
                    new = self.cache.allocator.alloc(need)
                except AllocationFailed:
                    self.evict_expired()
                    new = self.cache.allocator.alloc(need)
                self.table[s.row, len(s.pages):len(s.pages) + need] = new
                s.pages.extend(new)
                self._dirty = True
        s.last_used = time.monotonic()

    def sync_table(self, stream=None) -> torch.Tensor:
        if self._dirty:
            with self.lock:
                if self._pinned is None:
                    self.table_dev.copy_(torch.from_numpy(self.table), non_blocking=False)
                else:
                    self._pin_k ^= 1
                    k = self._pin_k
                    if self._pin_ev[k] is not None:
                        self._pin_ev[k].synchronize()  # the copy issued two syncs ago
                    self._pinned[k].numpy()[...] = self.table
                    self.table_dev.copy_(self._pinned[k], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
                    self._pin_ev[k] = ev
                self._dirty = False
        return self.table_dev

    @property
    def free_pages(self) -> int:
        return self.cache.allocator.free_pages

    def cache_tokens_left(self) -> int:
        return self.free_pages * self.page_size
