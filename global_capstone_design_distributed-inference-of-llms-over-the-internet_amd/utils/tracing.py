"""roctx ranges + a per-phase timing registry (SURVEY §5 "Tracing / profiling").

The reference has only ``time.perf_counter()`` around prefill/decode (src/main.py:138-153,213-225)
and per-hop client RTT lists that are never printed (src/rpc_transport.py:98-103). Here:

* ``trace_range(name)`` pushes a roctx range (``librocprofiler-sdk-roctx`` / ``libroctx64``,
  loaded with ctypes). Under ``rocprofv3 --marker-trace`` the stage steps, handler batches and
  pipeline ticks then show up as named ranges around their kernels. It costs nothing unless
  ``MPAMD_TRACE=1`` (or :func:`enable`) is set.
* ``PhaseTimer`` accumulates host wall time per phase name (count / total / max). The stage
  handler exposes it through ``rpc_info``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
import time
from typing import Dict, Optional

_LIB = None
_ENABLED = os.environ.get("MPAMD_TRACE", "0") not in ("", "0")
_CANDIDATES = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")


def _load():
    global _LIB
    if _LIB is not None:
        return _LIB or None
    _LIB = False
    for name in _CANDIDATES:
        for path in (name, os.path.join("/opt/rocm/lib", name)):
            try:
                lib = ctypes.CDLL(path)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _LIB = lib
                return lib
            except (OSError, AttributeError):
                continue
    return None


def enable(flag: bool = True) -> bool:
    """Turn roctx ranges on/off; returns whether a roctx library is available."""
    global _ENABLED
    _ENABLED = bool(flag)
    return _load() is not None


def available() -> bool:
    return _load() is not None


@contextlib.contextmanager
def trace_range(name: str):
    lib = _load() if _ENABLED else None
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _load() if _ENABLED else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


class PhaseTimer:
    """Thread-safe wall-time accumulator: ``with timer("decode"): ...``."""

    def __init__(self):
        self._lock = threading.Lock()
        self.stats: Dict[str, Dict[str, float]] = {}

    @contextlib.contextmanager
    def __call__(self, name: str, trace: bool = True):
        t0 = time.perf_counter()
        with (trace_range(name) if trace else contextlib.nullcontext()):
            yield
        dt = time.perf_counter() - t0
        with self._lock:
            s = self.stats.setdefault(name, {"count": 0, "total_s": 0.0, "max_s": 0.0})
            s["count"] += 1
            s["total_s"] += dt
            s["max_s"] = max(s["max_s"], dt)

    def summary(self, prefix: Optional[str] = None) -> Dict[str, Dict[str, float]]:
        with self._lock:
            return {k: {**v, "mean_ms": 1000 * v["total_s"] / max(v["count"], 1)}
                    for k, v in self.stats.items() if prefix is None or k.startswith(prefix)}

    def reset(self) -> None:
        with self._lock:
            self.stats.clear()
