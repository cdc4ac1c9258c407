"""Native (C++) host runtime: KV page allocator, batch-metadata builder, wire framing.

Built in-tree by ``build()`` (g++ + pybind11) into ``native/_mpamd_runtime*.so``.  A
numpy implementation with identical semantics is kept for hosts without a compiler;
``BACKEND`` says which one is live.
"""
from __future__ import annotations

import hashlib
import os
import struct
import subprocess
import sys
import sysconfig

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "runtime.cpp")
SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
LIB = os.path.join(HERE, "_mpamd_runtime" + SUFFIX)
# direct RCCL communicators (rccl.cpp; dlopens torch's librccl at run time, links no ROCm library)
RCCL_SRC = os.path.join(HERE, "rccl.cpp")
RCCL_LIB = os.path.join(HERE, "_mpamd_rccl" + SUFFIX)


def _build_one(src: str, lib: str, force: bool, libs=()) -> str:
    import pybind11

    with open(src, "rb") as f:
        tag = hashlib.sha256(f.read()).hexdigest()
    stamp = lib + ".stamp"
    if not force and os.path.exists(lib) and os.path.exists(stamp) and open(stamp).read().strip() == tag:
        return lib
    inc = [pybind11.get_include(), sysconfig.get_paths()["include"]]
    cmd = ["g++", "-O3", "-shared", "-fPIC", "-std=c++17", "-fvisibility=hidden"] + [f"-I{p}" for p in inc] + [
        src, "-o", lib + ".tmp"] + list(libs)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode:
        raise RuntimeError(f"native build of {os.path.basename(src)} failed:\n" + r.stdout)
    os.replace(lib + ".tmp", lib)
    with open(stamp, "w") as f:
        f.write(tag)
    return lib


def build(force: bool = False) -> str:
    """Build the host runtime and the direct-RCCL module; returns the runtime's path."""
    _build_one(RCCL_SRC, RCCL_LIB, force, libs=("-ldl",))
    return _build_one(SRC, LIB, force)


_mod = None
BACKEND = "python"
try:
    if HERE not in sys.path:
        pass
    import importlib.util

    if not os.path.exists(LIB):
        try:
            build()
        except Exception:
            pass
    if os.path.exists(LIB):
        spec = importlib.util.spec_from_file_location("_mpamd_runtime", LIB)
        _mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(_mod)
        BACKEND = "native"
except Exception:  # pragma: no cover
    _mod = None
    BACKEND = "python"


class _PyPageAllocator:
    def __init__(self, n):
        self.n = n
        self.free_list = list(range(n - 1, -1, -1))
        self.used = bytearray(n)

    def free_count(self):
        return len(self.free_list)

    def capacity(self):
        return self.n

    def alloc(self, k):
        if k > len(self.free_list):
            return None
        out = [self.free_list.pop() for _ in range(k)]
        for p in out:
            self.used[p] = 1
        return out

    def free(self, pages):
        for p in pages:
            if p < 0 or p >= self.n:
                raise IndexError("page id out of range")
            if not self.used[p]:
                raise RuntimeError(f"double free of KV page {p}")
            self.used[p] = 0
            self.free_list.append(p)


def make_page_allocator(n: int):
    return _mod.PageAllocator(n) if _mod is not None else _PyPageAllocator(n)


def _py_build_meta(rows, starts, ntoks, block_table, page_size, positions, slots, q_seq, q_ctx, last_rows):
    T = int(ntoks.sum())
    t = 0
    for i in range(len(rows)):
        n = int(ntoks[i])
        p = np.arange(starts[i], starts[i] + n, dtype=np.int64)
        pages = block_table[rows[i], p // page_size].astype(np.int64)
        if (pages < 0).any():
            raise RuntimeError("unallocated KV page")
        positions[t:t + n] = p
        slots[t:t + n] = pages * page_size + (p & (page_size - 1))
        q_seq[t:t + n] = rows[i]
        q_ctx[t:t + n] = p + 1
        t += n
        last_rows[i] = t - 1
    return T


def build_meta(rows, starts, ntoks, block_table, page_size, positions, slots, q_seq, q_ctx, last_rows) -> int:
    if _mod is not None:
        return _mod.build_meta(rows, starts, ntoks, block_table, page_size, positions, slots, q_seq, q_ctx, last_rows)
    return _py_build_meta(rows, starts, ntoks, block_table, page_size, positions, slots, q_seq, q_ctx, last_rows)


MAGIC = 0x3146504D


def pack_prefix(header: bytes, payload_lens) -> bytes:
    if _mod is not None:
        return _mod.pack_prefix(header, [int(x) for x in payload_lens])
    return struct.pack("<III", MAGIC, len(header), len(payload_lens)) + b"".join(
        struct.pack("<Q", int(x)) for x in payload_lens) + header


def unpack_fixed(prefix12: bytes):
    if _mod is not None:
        return tuple(_mod.unpack_fixed(prefix12))
    magic, hl, n = struct.unpack("<III", prefix12)
    if magic != MAGIC:
        raise RuntimeError("bad frame magic")
    if hl > (64 << 20) or n > 4096:
        raise RuntimeError("frame header too large")
    return hl, n
