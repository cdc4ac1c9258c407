"""Replicated TTL key/value registry (the role hivemind's Kademlia DHT plays in the reference).

The reference uses ``hivemind.DHT`` purely as a replicated record store with sub-keys and
expiration (reference src/dht_utils.py:34-281, src/main.py:442-537, src/rpc_transport.py:188-353):
``store(key, value, expiration_time, subkey=...)`` and ``get(key, latest=True)`` returning a
value whose sub-keyed form is ``{subkey: ValueWithExpiration}``.  This module implements
exactly that API over the framework's own TCP RPC:

* every node keeps a full local copy (swarms are tens of nodes, records are tiny);
* ``store`` applies locally and pushes to every known peer (fire-and-forget);
* joining = ``registry.join`` to the ``initial_peers`` (returns their peer list + a snapshot);
* anti-entropy: every ``sync_period`` s a node pulls a snapshot from a random peer, so a
  node that missed pushes converges; unreachable peers are dropped after repeated failures;
* merge rule: per (key, subkey) the record with the later expiration wins; expired
  records are invisible to ``get`` and purged.

Liveness semantics match the reference: servers refresh their records (TTL 45 s) every
TTL/3 = 15 s, and a crashed server simply ages out.
"""
from __future__ import annotations

import asyncio
import dataclasses
import logging
import random
import threading
import time
from typing import Any, Dict, List, Optional

from .rpc import RpcClient, RpcServer, get_loop
from .wire import Message, parse_peer_address

logger = logging.getLogger(__name__)


def get_dht_time() -> float:
    return time.time()


@dataclasses.dataclass
class ValueWithExpiration:
    value: Any
    expiration_time: float

    def __iter__(self):  # tuple-unpacking compatibility
        yield self.value
        yield self.expiration_time


_NOSUB = "\x00"  # internal marker for records stored without a subkey


class DHT:
    def __init__(self, start: bool = True, initial_peers: Optional[List[str]] = None,
                 host_maddrs: Optional[List[str]] = None, announce_maddrs: Optional[List[str]] = None,
                 sync_period: float = 5.0, request_timeout: float = 3.0, **_ignored):
        self.loop = get_loop()
        host, port = "127.0.0.1", 0
        if host_maddrs:
            host, port, _ = parse_peer_address(host_maddrs[0])
        ann_host = ann_port = None
        if announce_maddrs:
            ann_host, ann_port, _ = parse_peer_address(announce_maddrs[0])
        self._data: Dict[str, Dict[str, tuple]] = {}
        self._lock = threading.RLock()
        self.peers: Dict[str, int] = {}  # peer address -> consecutive failures
        self.initial_peers = list(initial_peers or [])
        self.sync_period = sync_period
        self.timeout = request_timeout
        self.server = RpcServer(host, port, announce_host=ann_host, announce_port=ann_port)
        self.client: Optional[RpcClient] = None
        self._sync_task = None
        self._alive = False
        for name, fn in (("registry.store", self._h_store), ("registry.get", self._h_get),
                         ("registry.join", self._h_join), ("registry.snapshot", self._h_snapshot)):
            self.server.add_handler(name, fn)
        if start:
            self.run_in_background()

    # ------------------------------------------------------------------ lifecycle
    def run_in_background(self, await_ready: bool = True):
        self.loop.run(self._start(), timeout=30)
        self._alive = True

    async def _start(self):
        self.client = RpcClient()
        await self.server.start()
        for p in self.initial_peers:
            await self._join(p)
        self._sync_task = asyncio.ensure_future(self._sync_forever())

    @property
    def peer_id(self) -> str:
        return self.server.peer_id

    @property
    def address(self) -> str:
        return self.server.maddrs[0]

    def get_visible_maddrs(self) -> List[str]:
        return list(self.server.maddrs)

    def shutdown(self):
        if not self._alive:
            return
        self._alive = False

        async def _stop():
            if self._sync_task is not None:
                self._sync_task.cancel()
            await self.server.shutdown()
            if self.client is not None:
                await self.client.close()

        try:
            self.loop.run(_stop(), timeout=5)
        except Exception:
            pass

    # ------------------------------------------------------------------ local store
    def _merge(self, key: str, subkey: Optional[str], value: Any, exp: float) -> bool:
        sk = _NOSUB if subkey is None else str(subkey)
        with self._lock:
            rec = self._data.setdefault(key, {})
            cur = rec.get(sk)
            if cur is not None and cur[1] >= exp:
                return False
            rec[sk] = (value, float(exp))
            return True

    def _snapshot(self) -> List[list]:
        now = get_dht_time()
        with self._lock:
            return [[k, (None if sk == _NOSUB else sk), v, e] for k, rec in self._data.items()
                    for sk, (v, e) in rec.items() if e > now]

    def _purge(self):
        now = get_dht_time()
        with self._lock:
            for k in list(self._data):
                rec = self._data[k]
                for sk in [sk for sk, (_, e) in rec.items() if e <= now]:
                    del rec[sk]
                if not rec:
                    del self._data[k]

    # ------------------------------------------------------------------ public API
    def store(self, key: str, value: Any, expiration_time: float, subkey: Optional[Any] = None, **_kw) -> bool:
        if expiration_time <= get_dht_time():
            return False
        self._merge(key, subkey, value, expiration_time)
        rec = [key, None if subkey is None else str(subkey), value, float(expiration_time)]
        if self.peers:
            self.loop.submit(self._push([rec]))
        return True

    def get(self, key: str, latest: bool = True, **_kw) -> Optional[ValueWithExpiration]:
        v = self._local_get(key)
        if v is None and self.peers and latest:
            try:
                self.loop.run(self._pull_key(key), timeout=self.timeout + 1)
            except Exception:
                pass
            v = self._local_get(key)
        return v

    def _local_get(self, key: str) -> Optional[ValueWithExpiration]:
        now = get_dht_time()
        with self._lock:
            rec = self._data.get(key)
            if not rec:
                return None
            live = {sk: (v, e) for sk, (v, e) in rec.items() if e > now}
        if not live:
            return None
        if _NOSUB in live and len(live) == 1:
            v, e = live[_NOSUB]
            return ValueWithExpiration(v, e)
        sub = {sk: ValueWithExpiration(v, e) for sk, (v, e) in live.items() if sk != _NOSUB}
        return ValueWithExpiration(sub, max(e for _, e in live.values()))

    # ------------------------------------------------------------------ replication
    async def _call(self, peer: str, name: str, md: dict) -> Optional[Message]:
        try:
            resp = await self.client.call(peer, name, Message(md), timeout=self.timeout)
            self.peers[peer] = 0
            return resp
        except Exception as e:
            if peer in self.peers:
                self.peers[peer] += 1
                if self.peers[peer] >= 3:
                    logger.info(f"registry: dropping unreachable peer {peer} ({e!r})")
                    self.peers.pop(peer, None)
                    self.client.drop(peer)
            return None

    async def _push(self, recs):
        me = self.address
        await asyncio.gather(*[self._call(p, "registry.store", {"recs": recs, "from": me}) for p in list(self.peers)])

    async def _join(self, peer: str):
        resp = None
        for attempt in range(3):
            self.peers.setdefault(peer, 0)
            resp = await self._call(peer, "registry.join", {"addr": self.address})
            if resp is not None:
                break
            await asyncio.sleep(0.2 * (attempt + 1))
        if resp is None:
            logger.warning(f"registry: could not reach initial peer {peer}")
            return
        for rec in resp.metadata.get("snapshot", []):
            self._merge(*rec)
        for p in resp.metadata.get("peers", []):
            if p != self.address and p not in self.peers:
                self.peers[p] = 0
                await self._call(p, "registry.join", {"addr": self.address})

    async def _pull_key(self, key: str):
        for p in list(self.peers):
            resp = await self._call(p, "registry.get", {"key": key})
            if resp is not None and resp.metadata.get("recs"):
                for rec in resp.metadata["recs"]:
                    self._merge(*rec)
                return

    async def _sync_forever(self):
        while True:
            await asyncio.sleep(self.sync_period * (0.5 + random.random()))
            self._purge()
            if not self.peers:
                for p in self.initial_peers:  # re-bootstrap after a partition
                    await self._join(p)
                continue
            p = random.choice(list(self.peers))
            resp = await self._call(p, "registry.snapshot", {"addr": self.address})
            if resp is not None:
                for rec in resp.metadata.get("snapshot", []):
                    self._merge(*rec)
                for q in resp.metadata.get("peers", []):
                    if q != self.address:
                        self.peers.setdefault(q, 0)

    # ------------------------------------------------------------------ handlers
    async def _h_store(self, msg: Message) -> Message:
        for rec in msg.metadata.get("recs", []):
            self._merge(*rec)
        src = msg.metadata.get("from")
        if src and src != self.address:
            self.peers.setdefault(src, 0)
        return Message({"ok": True})

    async def _h_get(self, msg: Message) -> Message:
        key = msg.metadata["key"]
        now = get_dht_time()
        with self._lock:
            rec = dict(self._data.get(key, {}))
        recs = [[key, None if sk == _NOSUB else sk, v, e] for sk, (v, e) in rec.items() if e > now]
        return Message({"recs": recs})

    async def _h_join(self, msg: Message) -> Message:
        addr = msg.metadata.get("addr")
        peers = [p for p in self.peers if p != addr] + [self.address]
        if addr and addr != self.address:
            self.peers.setdefault(addr, 0)
        return Message({"peers": peers, "snapshot": self._snapshot()})

    async def _h_snapshot(self, msg: Message) -> Message:
        addr = msg.metadata.get("addr")
        if addr and addr != self.address:
            self.peers.setdefault(addr, 0)
        return Message({"peers": list(self.peers) + [self.address], "snapshot": self._snapshot()})
