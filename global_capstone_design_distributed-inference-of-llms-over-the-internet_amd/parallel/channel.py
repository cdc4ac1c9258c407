"""Device channel: the single-node data plane between the stages of one pipeline.

Reference data path: every hidden state crosses host memory, protobuf serialization and a
libp2p TCP stream per hop, client -> server -> client (star), reference
src/rpc_transport.py:738-766, :802-833 and src/rpc_handler.py:405-464.  On one MI355X node
the same hop becomes an RCCL send/recv over the direct xGMI link between neighbouring
GPUs.  A ``Channel`` joins the P participants of one pipeline (rank 0 = the head that owns
the embedding and the scheduler, rank P-1 = the tail that samples) with three process
groups built straight from a ``torch.distributed`` Store, so a process can hold any number
of channels and needs no default process group (a stage server may serve several clients
over its lifetime):

* ``ctrl`` (gloo, host tensors): step headers (which sessions, how many tokens, positions,
  closes, admissions), all-gathers of per-stage capacity / throughput, stop messages.
  Every receive carries a timeout, and a SIGKILLed peer surfaces as a connection error
  within milliseconds: this is the failure detector of the device path.
* ``data`` (RCCL on GPU, gloo on CPU): hidden states rank k -> k+1, straight from HBM.
* ``ret`` (RCCL on GPU, gloo on CPU): sampled token ids tail -> head.  A communicator of
  its own: RCCL serialises the P2P operations of one communicator on one stream, so with
  2 stages the forward hop (0 -> 1) and the token return (1 -> 0) would otherwise queue
  behind each other.

Headers go on the host group ahead of the payload: a stage forwards the header to its
successor BEFORE computing, so the next stage plans its step (session table, page
reservations, metadata H2D) while the payload is still being produced.

``MPAMD_CHANNEL_DATA=gloo`` stages GPU payloads through host memory over gloo (several
ranks sharing one GPU, where RCCL refuses duplicate devices).  ``MPAMD_CHANNEL_DATA=rccl`` carries
``data`` / ``ret`` on the direct communicators of ``parallel/rccl.py`` instead of
ProcessGroupNCCL: one two-rank communicator per neighbouring stage pair and one tail -> head,
all initialised when the channel is built (ProcessGroupNCCL creates its per-peer
communicator lazily, at the first send of a serving step), each driven from a dedicated HIP
stream of this rank ordered against the compute stream by events.
"""
from __future__ import annotations

import collections
import datetime
import logging
import os
import socket
import time
from typing import Deque, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

logger = logging.getLogger(__name__)


class ChannelError(RuntimeError):
    """A peer of the channel failed (timeout, connection closed, aborted communicator)."""


def host_id() -> str:
    """Identity of this machine: hostname + kernel boot id (two containers with the same
    hostname on different hosts differ in boot id).  Stages advertise it so a client can
    tell whether a device channel is possible (same node) or TCP must be used."""
    boot = ""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        pass
    return f"{socket.gethostname()}/{boot}"


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def _td(s: float) -> datetime.timedelta:
    return datetime.timedelta(seconds=float(s))


def make_store(host: str, port: int, world: int, is_master: bool, timeout_s: float = 60.0):
    return dist.TCPStore(host, int(port), int(world), bool(is_master), timeout=_td(timeout_s),
                         wait_for_workers=False)


def _gloo(store, prefix: str, rank: int, world: int, timeout_s: float):
    return dist.ProcessGroupGloo(dist.PrefixStore(prefix, store), rank, world, _td(timeout_s))


def _nccl(store, prefix: str, rank: int, world: int, timeout_s: float, device: torch.device):
    torch.cuda.set_device(device)
    opts = dist.ProcessGroupNCCL.Options()
    opts._timeout = _td(timeout_s)
    return dist.ProcessGroupNCCL(dist.PrefixStore(prefix, store), rank, world, opts)


class _Pending:
    """Outstanding sends: their buffers must stay alive until the work completes."""

    def __init__(self, limit: int = 64):
        self.q: Deque[Tuple[object, object]] = collections.deque()
        self.limit = limit

    def add(self, work, keep) -> None:
        self.q.append((work, keep))
        while len(self.q) > self.limit:
            self.q.popleft()[0].wait()

    def reap(self) -> None:
        while self.q and self.q[0][0].is_completed():
            self.q.popleft()

    def drain(self, timeout_s: Optional[float] = None) -> None:
        while self.q:
            w, _ = self.q.popleft()
            if timeout_s is None:
                w.wait()
            else:
                w.wait(_td(timeout_s))


class _EventWork:
    """Completion of an operation enqueued on a side stream, with the ProcessGroup ``Work``
    surface the slab ring and the pending-send queue use: ``wait()`` orders the CURRENT stream
    after it (no host block); ``wait(timeout)`` blocks the host with a deadline (flush)."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self, timeout=None):
        if timeout is None:
            torch.cuda.current_stream().wait_event(self.ev)
        else:
            wait_event(self.ev, timeout.total_seconds() if hasattr(timeout, "total_seconds") else float(timeout),
                       "RCCL send")
        return True

    def is_completed(self) -> bool:
        return self.ev.query()


class _Waiter:
    """``Channel.recv``'s completion: ``host_wait()`` blocks the host until the payload is here
    (gloo; a no-op on the device backends, whose completion is a stream dependency), ``__call__``
    finishes the hand-off on the current stream (stream wait, staging copy) and returns the tensor.
    Split so that the blocking part can run outside a lock that serialises device work: a device
    copy or allocation from this thread while another one captures a hipGraph would break that
    capture."""

    def __init__(self, host_wait, device):
        self._host = host_wait
        self._device = device

    def host_wait(self) -> None:
        if self._host is not None:
            fn, self._host = self._host, None
            fn()

    def __call__(self):
        self.host_wait()
        return self._device()


class _SlabRing:
    """Preallocated device byte slabs reused round-robin for RCCL payloads (no per-hop
    ``clone`` / ``empty``: the caching allocator and its cross-stream bookkeeping stay off the
    hop).  A slab is handed out again only after a stream dependency on the work that last
    used it (``work.wait()`` = the current stream waits for the RCCL stream, no host block),
    so a send is never overwritten in flight; a receive slab's readers were enqueued on the
    current stream before the next receive into it is posted, and RCCL's stream waits for
    them.  Slabs grow (per slot, lazily) to the largest payload seen."""

    def __init__(self, device: torch.device, slots: int):
        self.device = device
        self.bufs: List[Optional[torch.Tensor]] = [None] * int(slots)
        self.works: List[Optional[object]] = [None] * int(slots)
        self.k = -1

    def take(self, shape, dtype) -> Tuple[int, torch.Tensor]:
        self.k = (self.k + 1) % len(self.bufs)
        k = self.k
        w = self.works[k]
        if w is not None:
            w.wait()
            self.works[k] = None
        n = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
        buf = self.bufs[k]
        if buf is None or buf.numel() < n:
            buf = self.bufs[k] = torch.empty(max(n, 1 << 16), dtype=torch.uint8, device=self.device)
        return k, buf[:n].view(dtype).view(shape)

    def done(self, k: int, work) -> None:
        self.works[k] = work


class Channel:
    def __init__(self, store, prefix: str, rank: int, world: int, device, timeout_s: float = 120.0,
                 data_backend: Optional[str] = None, ring_slots: int = 32):
        self.rank, self.world = int(rank), int(world)
        self.device = torch.device(device)
        self.timeout_s = float(timeout_s)
        self.prefix = prefix
        if data_backend is None:
            data_backend = os.environ.get("MPAMD_CHANNEL_DATA") or ("nccl" if self.device.type == "cuda" else "gloo")
        self.data_backend = data_backend
        self.staged = data_backend == "gloo" and self.device.type == "cuda"
        self.ctrl = _gloo(store, prefix + "/ctrl", self.rank, self.world, timeout_s)
        self._rc = {}
        if data_backend == "rccl":
            if self.device.type != "cuda":
                raise ValueError("the rccl data backend needs a GPU device")
            self.data = self.ret = None
            self._init_rccl(store, prefix, timeout_s)
        elif data_backend == "nccl":
            self.data = _nccl(store, prefix + "/data", self.rank, self.world, timeout_s, self.device)
            self.ret = _nccl(store, prefix + "/ret", self.rank, self.world, timeout_s, self.device)
        else:
            self.data = _gloo(store, prefix + "/data", self.rank, self.world, timeout_s)
            self.ret = _gloo(store, prefix + "/ret", self.rank, self.world, timeout_s)
        self._sends = _Pending()
        self._msg_sends = _Pending()
        self.closed = False
        # hop statistics (bench JSON / serving logs): payload bytes and sends, and how long this
        # rank's compute stream waited for an incoming payload (device: HIP events around the
        # stream wait; host paths: wall time of the blocking wait)
        self.bytes_sent = 0
        self.sends = 0
        self.timing = False
        self._wait_events: List[Tuple[object, object]] = []
        self._wait_host_s: List[float] = []
        self._rings = {}
        if data_backend in ("nccl", "rccl") and self.device.type == "cuda":
            self._rings = {(w, d): _SlabRing(self.device, ring_slots) for w in ("data", "ret") for d in ("send", "recv")}

    def _init_rccl(self, store, prefix: str, timeout_s: float) -> None:
        """Two-rank communicators: (k, k+1) for the hidden-state hop, (tail, head) for token
        return.  Every rank initialises its pairs in increasing k (a blocking init pairs with the
        neighbour's FIRST init), then the head / tail the return pair."""
        from .rccl import RcclComm

        r, P = self.rank, self.world
        if P < 2:
            return
        if r > 0:    # (r-1, r): this rank receives, as rank 1 of the pair
            self._rc[("data", "recv")] = (RcclComm(store, f"{prefix}/rdata/{r - 1}", 1, 2, self.device, timeout_s), 0)
        if r < P - 1:  # (r, r+1): this rank sends, as rank 0
            self._rc[("data", "send")] = (RcclComm(store, f"{prefix}/rdata/{r}", 0, 2, self.device, timeout_s), 1)
        if r == P - 1:
            self._rc[("ret", "send")] = (RcclComm(store, f"{prefix}/rret", 0, 2, self.device, timeout_s), 1)
        elif r == 0:
            self._rc[("ret", "recv")] = (RcclComm(store, f"{prefix}/rret", 1, 2, self.device, timeout_s), 0)
        self._rstreams = {k: torch.cuda.Stream(self.device) for k in self._rc}

    # ------------------------------------------------------------------ host control messages
    def send_msg(self, dst: int, arr: np.ndarray) -> None:
        """Length-prefixed int64 message on the ctrl group (async; buffers kept until done)."""
        body = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64))
        n = torch.tensor([body.numel()], dtype=torch.int64)
        try:
            self._msg_sends.add(self.ctrl.send([n], dst, 1), n)
            if body.numel():
                self._msg_sends.add(self.ctrl.send([body], dst, 2), body)
            self._msg_sends.reap()
        except RuntimeError as e:
            raise ChannelError(f"ctrl send to {dst} failed: {e}") from e

    def recv_msg(self, src: int, timeout_s: Optional[float] = None) -> np.ndarray:
        t = self.timeout_s if timeout_s is None else timeout_s
        n = torch.empty(1, dtype=torch.int64)
        try:
            self.ctrl.recv([n], src, 1).wait(_td(t))
            body = torch.empty(int(n[0]), dtype=torch.int64)
            if body.numel():
                self.ctrl.recv([body], src, 2).wait(_td(t))
        except RuntimeError as e:
            raise ChannelError(f"ctrl recv from {src} failed: {e}") from e
        return body.numpy()

    def all_gather_floats(self, values: Sequence[float]) -> List[List[float]]:
        """Every participant's ``values`` (same length everywhere) on every participant: the
        channel-level registry of per-stage capacity / measured step time."""
        t = torch.tensor(list(values), dtype=torch.float64)
        out = [torch.empty_like(t) for _ in range(self.world)]
        try:
            self.ctrl.allgather([out], [t]).wait(_td(self.timeout_s))
        except RuntimeError as e:
            raise ChannelError(f"ctrl all_gather failed: {e}") from e
        return [o.tolist() for o in out]

    # ------------------------------------------------------------------ device payloads
    def _pg(self, which: str):
        return self.data if which == "data" else self.ret

    def send(self, dst: int, t: torch.Tensor, which: str = "data") -> None:
        """Send ``t`` (a private copy is taken, so the caller may overwrite ``t`` right away -
        e.g. a hipGraph output buffer - while the send is in flight)."""
        if self._rc:
            return self._rccl_send(dst, t, which)
        pg = self._pg(which)
        try:
            ring = self._rings.get((which, "send"))
            if ring is not None:
                k, buf = ring.take(tuple(t.shape), t.dtype)
                buf.copy_(t.detach())
            elif self.staged:
                buf = t.detach().to("cpu")
            else:
                buf = t.detach().clone()
            self.bytes_sent += buf.numel() * buf.element_size()
            self.sends += 1
            work = pg.send([buf], dst, 0)
            if ring is not None:
                ring.done(k, work)
            self._sends.add(work, buf)
            self._sends.reap()
        except RuntimeError as e:
            raise ChannelError(f"{which} send to {dst} failed: {e}") from e

    def recv(self, src: int, shape, dtype, which: str = "data", timeout_s: Optional[float] = None, into=None):
        """Post a receive; returns ``(tensor, waiter)``.  ``waiter()`` makes the tensor usable
        on the current stream: on RCCL it is a stream dependency (no host block), on gloo a
        blocking wait bounded by the timeout.  ``waiter.host_wait()`` does only the blocking host
        part (nothing on the device): a caller may run it outside a lock that guards device work and
        call ``waiter()`` under the lock.

        ``into = (buffer, free_event)``: receive straight into ``buffer`` - e.g. the static input of
        the decode graph the step will replay - once ``free_event`` (its last reader's completion,
        None = free now) has passed.  Every backend honours it when shape and dtype match: RCCL and
        ProcessGroupNCCL receive into it, host-staged gloo copies the host payload into it, CPU gloo
        receives into it.  The returned tensor is then ``buffer`` itself."""
        if into is not None and not (tuple(into[0].shape) == tuple(shape) and into[0].dtype == dtype and
                                     into[0].is_contiguous() and into[0].device == self.device):
            into = None
        if self._rc:
            return self._rccl_recv(src, shape, dtype, which, into)
        pg = self._pg(which)
        t = self.timeout_s if timeout_s is None else timeout_s
        try:
            if self.staged or self.device.type != "cuda":
                host = into[0] if (into is not None and not self.staged) else torch.empty(shape, dtype=dtype)
                work = pg.recv([host], src, 0)

                def host_wait():
                    t0 = time.perf_counter()
                    try:
                        work.wait(_td(t))
                    except RuntimeError as e:
                        raise ChannelError(f"{which} recv from {src} failed: {e}") from e
                    if self.timing:
                        self._wait_host_s.append(time.perf_counter() - t0)

                def device():
                    if not self.staged:
                        return host
                    if into is None:
                        return host.to(self.device, non_blocking=False)
                    buf, free = into
                    if free is not None:
                        torch.cuda.current_stream().wait_event(free)
                    buf.copy_(host)
                    return buf

                return (into[0] if into is not None else None), _Waiter(host_wait, device)
            ring = self._rings.get((which, "recv"))
            k = None
            if into is not None:
                buf, free = into
                if free is not None:  # ProcessGroupNCCL's stream waits for the current stream's work
                    torch.cuda.current_stream().wait_event(free)
            elif ring is not None:
                k, buf = ring.take(tuple(shape), dtype)
            else:
                buf = torch.empty(shape, dtype=dtype, device=self.device)
            work = pg.recv([buf], src, 0)
            if k is not None:
                ring.done(k, work)

            def waiter():
                e0 = None
                if self.timing:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                work.wait()
                if e0 is not None:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record()
                    self._wait_events.append((e0, e1))
                return buf

            return buf, _Waiter(None, waiter)
        except RuntimeError as e:
            raise ChannelError(f"{which} recv from {src} failed: {e}") from e

    def _rccl_pair(self, which: str, direction: str, other: int):
        key = (which, direction)
        if key not in self._rc:
            raise ChannelError(f"rank {self.rank} has no {which} {direction} pair (peer {other})")
        comm, peer = self._rc[key]
        expect = {("data", "send"): self.rank + 1, ("data", "recv"): self.rank - 1, ("ret", "send"): 0,
                  ("ret", "recv"): self.world - 1}[key]
        if other != expect:
            raise ChannelError(f"{which} {direction}: rank {self.rank} talks to {expect}, not {other}")
        return comm, peer, self._rstreams[key]

    def _rccl_send(self, dst: int, t: torch.Tensor, which: str) -> None:
        comm, peer, st = self._rccl_pair(which, "send", dst)
        ring = self._rings[(which, "send")]
        try:
            k, buf = ring.take(tuple(t.shape), t.dtype)   # stream-waits the slab's previous send
            buf.copy_(t.detach())                        # compute stream: the caller may reuse t
            ready = torch.cuda.Event()
            ready.record()
            st.wait_event(ready)
            comm.send(buf, peer, stream=st)
            done = torch.cuda.Event()
            done.record(st)
        except RuntimeError as e:
            raise ChannelError(f"{which} send to {dst} failed: {e}") from e
        work = _EventWork(done)
        self.bytes_sent += buf.numel() * buf.element_size()
        self.sends += 1
        ring.done(k, work)
        self._sends.add(work, buf)
        self._sends.reap()

    def send_on_stream(self, dst: int, t: torch.Tensor, which: str = "data") -> None:
        """Direct-RCCL send of ``t`` on the CURRENT stream, no private copy: recorded into a
        hipGraph when called during a capture (the engine's graph hop).  Stream order is what
        keeps ``t`` alive and unmodified until the send has read it; every send of this pair must
        then go this way (one stream per communicator keeps the op order the receiver sees)."""
        if not self._rc:
            raise ChannelError("send_on_stream needs the rccl data backend")
        comm, peer, _ = self._rccl_pair(which, "send", dst)
        try:
            comm.send(t, peer)
        except RuntimeError as e:
            raise ChannelError(f"{which} send to {dst} failed: {e}") from e
        if not torch.cuda.is_current_stream_capturing():
            self.count_send(t.numel() * t.element_size())

    def count_send(self, nbytes: int) -> None:
        """Hop statistics for a send that ran inside a graph replay."""
        self.bytes_sent += int(nbytes)
        self.sends += 1

    def _rccl_recv(self, src: int, shape, dtype, which: str, into=None):
        comm, peer, st = self._rccl_pair(which, "recv", src)
        ring = self._rings[(which, "recv")]
        k = None
        try:
            if into is not None:
                buf, free = into
                if free is not None:  # the buffer's last reader (an earlier replay) must be done
                    st.wait_event(free)
            else:
                k, buf = ring.take(tuple(shape), dtype)
                free = torch.cuda.Event()  # the slab's previous readers are on the compute stream
                free.record()
                st.wait_event(free)
            comm.recv(buf, peer, stream=st)
            done = torch.cuda.Event()
            done.record(st)
        except RuntimeError as e:
            raise ChannelError(f"{which} recv from {src} failed: {e}") from e
        work = _EventWork(done)
        if k is not None:
            ring.done(k, work)

        def waiter():
            e0 = None
            if self.timing:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            work.wait()
            if e0 is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                self._wait_events.append((e0, e1))
            return buf

        return buf, _Waiter(None, waiter)

    def stats(self, reset: bool = True) -> dict:
        """Hop statistics since the last reset: backend, payload bytes / sends, and the mean
        ms this rank's stream (device) or host (gloo) waited for an incoming payload.  ``reset``
        starts a new window for ALL of them (byte and send counters included), so a caller that
        resets before a timed region reads exactly that region's traffic afterwards."""
        waits = [1e3 * x for x in self._wait_host_s]
        if self._wait_events:
            self._wait_events[-1][1].synchronize()
            waits += [a.elapsed_time(b) for a, b in self._wait_events]
        out = {"backend": self.data_backend + ("(host-staged)" if self.staged else ""), "bytes_sent": self.bytes_sent,
               "sends": self.sends, "recv_wait_ms": (sum(waits) / len(waits)) if waits else 0.0,
               "recvs_timed": len(waits)}
        if reset:
            self._wait_events.clear()
            self._wait_host_s.clear()
            self.bytes_sent = 0
            self.sends = 0
        return out

    def flush(self, timeout_s: Optional[float] = None) -> None:
        self._sends.drain(timeout_s if timeout_s is not None else None)
        self._msg_sends.drain(timeout_s)

    # ------------------------------------------------------------------ teardown
    def abort(self) -> None:
        """Tear the channel down after a peer failure: RCCL communicators are aborted so a
        stream blocked in a receive from a dead peer is released (no hang at exit)."""
        if self.closed:
            return
        self.closed = True
        for comm, _ in self._rc.values():
            try:
                comm.abort()
            except Exception:  # noqa: BLE001 - best effort during failure handling
                pass
        for pg in (self.data, self.ret):
            if pg is None:
                continue
            for name in ("abort", "_abort", "shutdown"):
                fn = getattr(pg, name, None)
                if fn is not None:
                    try:
                        fn()
                        break
                    except Exception:  # noqa: BLE001 - best effort during failure handling
                        continue
        self._sends.q.clear()
        self._msg_sends.q.clear()

    def close(self) -> None:
        if self.closed:
            return
        try:
            self.flush(timeout_s=min(self.timeout_s, 30.0))
        except RuntimeError:
            pass
        self.closed = True
        for comm, _ in self._rc.values():
            try:
                comm.close()
            except Exception:  # noqa: BLE001
                pass
        for pg in (self.data, self.ret):
            fn = getattr(pg, "shutdown", None)
            if fn is not None:
                try:
                    fn()
                except Exception:  # noqa: BLE001
                    pass


class HostLink:
    """A host-only (gloo) group: the replica router's link to a remote replica head, or the
    node-wide control group that all-gathers measured stage throughput."""

    def __init__(self, store, prefix: str, rank: int, world: int, timeout_s: float = 120.0):
        self.rank, self.world, self.timeout_s = int(rank), int(world), float(timeout_s)
        self.ctrl = _gloo(store, prefix, self.rank, self.world, timeout_s)
        self._msg_sends = _Pending()
        self.closed = False

    send_msg = Channel.send_msg
    recv_msg = Channel.recv_msg
    all_gather_floats = Channel.all_gather_floats

    def close(self) -> None:
        if not self.closed:
            self.closed = True
            try:
                self._msg_sends.drain(timeout_s=min(self.timeout_s, 10.0))
            except RuntimeError:
                pass

    def abort(self) -> None:
        self.closed = True
        self._msg_sends.q.clear()


def wait_event(ev, timeout_s: float, what: str = "device event") -> None:
    """Poll a HIP event with a deadline: a stream stuck on a receive from a dead RCCL peer
    never completes, and ``Event.synchronize`` would hang the host with it."""
    if ev is None:
        return
    if ev.query():
        return
    deadline = time.monotonic() + timeout_s
    # short, capped sleeps: the host waits here for the step issued two steps ago while the GPU
    # runs the last one; every microsecond overslept comes out of the time the host has to
    # issue the next step (a 1 ms backoff cap left the GPU idle ~9 % of a batch-1 decode step)
    sleep = 5e-6
    while not ev.query():
        if time.monotonic() > deadline:
            raise ChannelError(f"timed out after {timeout_s:.1f}s waiting for {what}")
        time.sleep(sleep)
        sleep = min(sleep * 2, 5e-5)
