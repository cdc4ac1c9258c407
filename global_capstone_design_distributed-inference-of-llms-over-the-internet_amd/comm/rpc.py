"""Asyncio TCP RPC: the off-node / control-plane transport.

Replaces hivemind ``P2P`` (a Go ``p2pd`` daemon per process, reached over a Unix socket;
reference src/main.py:486, src/rpc_transport.py:249-264, :519-585) with an in-process
asyncio server and a multiplexing client:

* one TCP connection per peer, many concurrent requests on it (request ids);
* handlers registered by name (``StageConnectionHandler.rpc_forward`` ...), unary or
  streamed (chunked request frames reassembled before the handler runs, the role of
  ``iterate_protobuf_handler`` / ``split_for_streaming``);
* every call has a timeout; a dead peer surfaces as ``ConnectionError`` /
  ``asyncio.TimeoutError`` exactly where the reference catches them for failover.

The event loop runs in a daemon thread (``BackgroundLoop``) so synchronous callers (the
client's token loop, the registry API) can use it like hivemind's background DHT process.
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import secrets
import threading
from typing import Awaitable, Callable, Dict, List, Optional, Tuple

import torch

from .wire import Message, make_maddr, parse_peer_address, read_message, split_for_streaming, write_message

logger = logging.getLogger(__name__)

MAX_UNARY_PAYLOAD_SIZE = 4 << 20   # bytes; larger requests are streamed in chunks
DEFAULT_MAX_MSG_SIZE = 2 << 20


class RemoteError(RuntimeError):
    """The remote handler raised; message carries its error text."""


def new_peer_id() -> str:
    alphabet = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"
    raw = int.from_bytes(secrets.token_bytes(24), "big")
    out = []
    while raw:
        raw, r = divmod(raw, 58)
        out.append(alphabet[r])
    return "Mp" + "".join(out)


class BackgroundLoop:
    def __init__(self, name: str = "mpamd-io"):
        self.loop = asyncio.new_event_loop()
        self._thread = threading.Thread(target=self._run, name=name, daemon=True)
        self._thread.start()

    def _run(self):
        asyncio.set_event_loop(self.loop)
        self.loop.run_forever()

    def run(self, coro: Awaitable, timeout: Optional[float] = None):
        if threading.current_thread() is self._thread:
            raise RuntimeError("BackgroundLoop.run called from its own thread (would deadlock)")
        return asyncio.run_coroutine_threadsafe(coro, self.loop).result(timeout)

    def submit(self, coro: Awaitable):
        return asyncio.run_coroutine_threadsafe(coro, self.loop)

    def stop(self):
        if self.loop.is_running():
            self.loop.call_soon_threadsafe(self.loop.stop)


_LOOP: Optional[BackgroundLoop] = None
_LOOP_LOCK = threading.Lock()


def get_loop() -> BackgroundLoop:
    global _LOOP
    with _LOOP_LOCK:
        if _LOOP is None:
            _LOOP = BackgroundLoop()
        return _LOOP


Handler = Callable[[Message], Awaitable[Message]]


class RpcServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, peer_id: Optional[str] = None,
                 announce_host: Optional[str] = None, announce_port: Optional[int] = None):
        self.host, self.port = host, port
        self.peer_id = peer_id or new_peer_id()
        self.announce_host, self.announce_port = announce_host, announce_port
        self.handlers: Dict[str, Handler] = {}
        self._server: Optional[asyncio.AbstractServer] = None
        self._conns = set()

    def add_handler(self, name: str, fn: Handler) -> None:
        self.handlers[name] = fn

    async def start(self) -> "RpcServer":
        self._server = await asyncio.start_server(self._on_conn, self.host, self.port, limit=1 << 24)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    @property
    def maddrs(self) -> List[str]:
        host = self.announce_host or (self.host if self.host not in ("0.0.0.0", "") else "127.0.0.1")
        return [make_maddr(host, self.announce_port or self.port, self.peer_id)]

    async def _on_conn(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        self._conns.add(writer)
        wlock = asyncio.Lock()
        partial: Dict[int, List[Message]] = {}
        tasks = set()
        try:
            while True:
                msg = await read_message(reader)
                if msg.kind == "stream":
                    parts = partial.setdefault(msg.rid, [])
                    parts.append(msg)
                    if not msg.metadata.get("_last", False):
                        continue
                    del partial[msg.rid]
                    merged = Message(metadata={k: v for k, v in parts[0].metadata.items() if not k.startswith("_")},
                                     tensors=[torch.cat([p.tensors[0] for p in parts], 0)] if parts[0].tensors else [],
                                     kind="req", name=msg.name, rid=msg.rid)
                    msg = merged
                t = asyncio.ensure_future(self._dispatch(msg, writer, wlock))
                tasks.add(t)
                t.add_done_callback(tasks.discard)
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        except Exception as e:  # pragma: no cover
            logger.warning(f"rpc connection error: {e!r}")
        finally:
            self._conns.discard(writer)
            try:
                writer.close()
            except Exception:
                pass

    async def _dispatch(self, msg: Message, writer, wlock):
        fn = self.handlers.get(msg.name)
        try:
            if fn is None:
                raise KeyError(f"no handler {msg.name!r}")
            resp = await fn(msg)
            resp.kind, resp.rid = "resp", msg.rid
        except Exception as e:
            logger.debug(f"handler {msg.name} failed: {e!r}")
            resp = Message(metadata={"error": f"{type(e).__name__}: {e}"}, kind="err", rid=msg.rid)
        try:
            async with wlock:
                await write_message(writer, resp)
        except Exception:
            pass

    async def shutdown(self):
        if self._server is not None:
            self._server.close()
            for w in list(self._conns):
                try:
                    w.close()
                except Exception:
                    pass
            try:
                await asyncio.wait_for(self._server.wait_closed(), 2.0)
            except Exception:
                pass
            self._server = None


class _Conn:
    def __init__(self, reader, writer):
        self.reader, self.writer = reader, writer
        self.pending: Dict[int, asyncio.Future] = {}
        self.lock = asyncio.Lock()
        self.task = asyncio.ensure_future(self._pump())
        self.closed = False

    async def _pump(self):
        try:
            while True:
                msg = await read_message(self.reader)
                fut = self.pending.pop(msg.rid, None)
                if fut is not None and not fut.done():
                    fut.set_result(msg)
        except Exception as e:
            self.closed = True
            for fut in self.pending.values():
                if not fut.done():
                    fut.set_exception(ConnectionError(f"connection lost: {e!r}"))
            self.pending.clear()

    def close(self):
        self.closed = True
        self.task.cancel()
        try:
            self.writer.close()
        except Exception:
            pass


class RpcClient:
    def __init__(self):
        self._conns: Dict[Tuple[str, int], _Conn] = {}
        self._rid = itertools.count(1)
        self._connect_lock: Optional[asyncio.Lock] = None

    async def _conn(self, host: str, port: int, timeout: float) -> _Conn:
        if self._connect_lock is None:
            self._connect_lock = asyncio.Lock()
        key = (host, port)
        c = self._conns.get(key)
        if c is not None and not c.closed:
            return c
        async with self._connect_lock:
            c = self._conns.get(key)
            if c is not None and not c.closed:
                return c
            reader, writer = await asyncio.wait_for(asyncio.open_connection(host, port, limit=1 << 24), timeout)
            c = _Conn(reader, writer)
            self._conns[key] = c
            return c

    def drop(self, addr: str) -> None:
        host, port, _ = parse_peer_address(addr)
        c = self._conns.pop((host, port), None)
        if c is not None:
            c.close()

    async def call(self, addr: str, name: str, msg: Message, timeout: float = 30.0,
                   stream_chunk_bytes: Optional[int] = None) -> Message:
        host, port, _ = parse_peer_address(addr)
        conn = await self._conn(host, port, timeout)
        rid = next(self._rid)
        fut = asyncio.get_running_loop().create_future()
        conn.pending[rid] = fut
        try:
            async with conn.lock:
                if stream_chunk_bytes and msg.tensors:
                    chunks = split_for_streaming(msg.tensors[0], stream_chunk_bytes)
                    for i, ch in enumerate(chunks):
                        md = dict(msg.metadata) if i == 0 else {}
                        md["_last"] = i == len(chunks) - 1
                        await write_message(conn.writer, Message(md, [ch], kind="stream", name=name, rid=rid))
                else:
                    await write_message(conn.writer, Message(msg.metadata, msg.tensors, kind="req", name=name, rid=rid))
            resp = await asyncio.wait_for(fut, timeout)
        except (asyncio.TimeoutError, ConnectionError, OSError):
            conn.pending.pop(rid, None)
            raise
        if resp.kind == "err":
            raise RemoteError(resp.metadata.get("error", "remote error"))
        return resp

    async def close(self):
        for c in self._conns.values():
            c.close()
        self._conns.clear()
