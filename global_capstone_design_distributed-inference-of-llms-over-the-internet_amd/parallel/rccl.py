"""Direct RCCL communicators on the caller's HIP stream (``native/rccl.cpp``).

Used where torch's ProcessGroupNCCL cannot go: inside a captured hipGraph.  The reference
moves hidden states host-side per hop (src/rpc_transport.py:738-766) and has no TP at all;
SURVEY §2.4 asks for the stage hop's RCCL send / recv and the TP all-reduces to be captured
with the stage's decode step.  An ``RcclComm`` is one communicator over ``world`` ranks,
initialised eagerly (no lazy per-peer communicator in the middle of a step) from a unique id
that rank 0 publishes in the caller's ``torch.distributed`` Store under ``prefix``.

Every operation is enqueued on ``stream`` (default: the current stream), so it lands in a
graph being captured on that stream, and stream order (not events or private copies)
protects the buffers.  ``abort`` releases a stream blocked on a dead peer.
"""
from __future__ import annotations

import atexit
import datetime
import importlib.util
import os
import threading
import weakref
from typing import Optional

import torch

_LOCK = threading.Lock()
_MOD = None
VERSION: Optional[int] = None

# live communicators, destroyed at interpreter exit while the HIP runtime is still up (a destructor
# running during teardown would call into RCCL after it)
_LIVE: "weakref.WeakSet[RcclComm]" = weakref.WeakSet()


@atexit.register
def _close_all() -> None:
    for c in list(_LIVE):
        try:
            c.close()
        except Exception:  # noqa: BLE001 - best effort at exit
            pass


_DTYPES = {torch.uint8: "UINT8", torch.int32: "INT32", torch.int64: "INT64", torch.float16: "FLOAT16",
           torch.float32: "FLOAT32", torch.bfloat16: "BFLOAT16"}


def module():
    """The native module with torch's librccl mapped (builds it in-tree if needed)."""
    global _MOD, VERSION
    with _LOCK:
        if _MOD is None:
            from .. import native

            try:  # a no-op when the source-hash stamp matches; rebuilds a stale library
                native._build_one(native.RCCL_SRC, native.RCCL_LIB, False, libs=("-ldl",))
            except Exception:  # noqa: BLE001 - no compiler here: a prebuilt library is used as is
                if not os.path.exists(native.RCCL_LIB):
                    raise
            spec = importlib.util.spec_from_file_location("_mpamd_rccl", native.RCCL_LIB)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            VERSION = mod.load(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
            _MOD = mod
        return _MOD


def available() -> bool:
    try:
        module()
        return True
    except Exception:  # noqa: BLE001 - no compiler / no librccl: callers keep torch's groups
        return False


def _stream(stream) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class RcclComm:
    def __init__(self, store, prefix: str, rank: int, world: int, device, timeout_s: float = 120.0):
        mod = module()
        self.rank, self.world = int(rank), int(world)
        self.device = torch.device(device)
        # a generation per (prefix, rank): every rank counts its own communicators under this
        # prefix, so a communicator re-created under the same prefix (a rebuilt channel) never
        # reads the unique id of its predecessor
        gen = int(store.add(f"{prefix}/rccl_gen/{self.rank}", 1))
        key = f"{prefix}/rccl_uid/{gen}"
        if self.rank == 0:
            uid = mod.unique_id()
            store.set(key, uid)
        else:
            store.wait([key], datetime.timedelta(seconds=float(timeout_s)))
            uid = store.get(key)
        torch.cuda.set_device(self.device)
        self._c = mod.Comm(self.world, self.rank, bytes(uid))
        self._mod = mod
        _LIVE.add(self)

    def _dt(self, t: torch.Tensor) -> int:
        if not t.is_contiguous():
            raise ValueError("RCCL buffers must be contiguous")
        try:
            return getattr(self._mod, _DTYPES[t.dtype])
        except KeyError:
            raise TypeError(f"RCCL: unsupported dtype {t.dtype}") from None

    def all_reduce(self, t: torch.Tensor, stream=None) -> torch.Tensor:
        """In-place sum over the communicator."""
        self._c.all_reduce(t.data_ptr(), t.numel(), self._dt(t), self._mod.SUM, _stream(stream))
        return t

    def all_gather(self, src: torch.Tensor, dst: torch.Tensor, stream=None) -> torch.Tensor:
        if dst.numel() != src.numel() * self.world:
            raise ValueError("all_gather: dst must hold world x src")
        self._c.all_gather(src.data_ptr(), dst.data_ptr(), src.numel(), self._dt(src), _stream(stream))
        return dst

    def send(self, t: torch.Tensor, peer: int, stream=None) -> None:
        self._c.send(t.data_ptr(), t.numel(), self._dt(t), int(peer), _stream(stream))

    def recv(self, t: torch.Tensor, peer: int, stream=None) -> torch.Tensor:
        self._c.recv(t.data_ptr(), t.numel(), self._dt(t), int(peer), _stream(stream))
        return t

    def send_recv(self, send: Optional[torch.Tensor], dst: int, recv: Optional[torch.Tensor], src: int,
                  stream=None) -> None:
        """One grouped send + receive (peers may be equal, or this rank itself)."""
        ref = send if send is not None else recv
        if send is not None and recv is not None and send.dtype != recv.dtype:
            raise TypeError("send_recv: one dtype per group")
        self._c.send_recv(send.data_ptr() if send is not None else 0, send.numel() if send is not None else 0,
                          int(dst) if send is not None else -1, recv.data_ptr() if recv is not None else 0,
                          recv.numel() if recv is not None else 0, int(src) if recv is not None else -1,
                          self._dt(ref), _stream(stream))

    def async_error(self) -> int:
        return int(self._c.async_error())

    @property
    def alive(self) -> bool:
        return bool(self._c.alive)

    def abort(self) -> None:
        self._c.abort()

    def close(self) -> None:
        self._c.destroy()
