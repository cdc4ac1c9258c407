"""Wire format of the TCP data/control plane.

Replaces hivemind's protobuf ``ExpertRequest``/``ExpertResponse`` + ``serialize_torch_tensor``
+ msgpack metadata (reference src/rpc_transport.py:519-585, src/rpc_handler.py:405-464).

A frame is::

    [magic u32 "MPF1"][header_len u32][n_payloads u32][payload_len u64 x n]
    [header: msgpack {"m": metadata, "t": [[dtype, shape], ...], ...}]
    [payload 0 raw bytes][payload 1 raw bytes] ...

Tensors travel as their raw little-endian bytes (no protobuf copy, no per-element
encoding); the prefix is built by the native runtime (``native.pack_prefix``).
"""
from __future__ import annotations

import asyncio
import dataclasses
from typing import Any, Dict, List, Optional, Tuple

import msgpack
import numpy as np
import torch

from .. import native

_DT = {
    torch.float32: "f32", torch.float16: "f16", torch.bfloat16: "bf16", torch.int64: "i64", torch.int32: "i32",
    torch.uint8: "u8", torch.int8: "i8", torch.bool: "b1",
}
_DT_INV = {v: k for k, v in _DT.items()}
MAX_FRAME = 4 << 30


@dataclasses.dataclass
class Message:
    """metadata (msgpack-able dict) + tensors."""
    metadata: Dict[str, Any] = dataclasses.field(default_factory=dict)
    tensors: List[torch.Tensor] = dataclasses.field(default_factory=list)
    kind: str = "req"          # req | resp | err | stream
    name: str = ""             # handler name (requests)
    rid: int = 0               # request id (multiplexing)


def _tensor_bytes(t: torch.Tensor) -> memoryview:
    t = t.detach()
    if t.device.type != "cpu":
        t = t.cpu()
    t = t.contiguous()
    if t.dtype == torch.bfloat16:
        arr = t.view(torch.int16).numpy()
    elif t.dtype == torch.bool:
        arr = t.to(torch.uint8).numpy()
    else:
        arr = t.numpy()
    return memoryview(arr).cast("B")


def encode(msg: Message) -> List[bytes]:
    """Frame -> list of buffers for ``writer.writelines`` (payloads are not copied)."""
    specs = []
    bufs = []
    for t in msg.tensors:
        if t.dtype not in _DT:
            raise TypeError(f"unsupported tensor dtype {t.dtype}")
        specs.append([_DT[t.dtype], list(t.shape)])
        bufs.append(_tensor_bytes(t))
    header = msgpack.packb({"m": msg.metadata, "t": specs, "k": msg.kind, "n": msg.name, "r": msg.rid},
                           use_bin_type=True)
    prefix = native.pack_prefix(header, [len(b) for b in bufs])
    return [prefix] + bufs


def _decode_tensor(spec, raw: bytes) -> torch.Tensor:
    dt_name, shape = spec
    dt = _DT_INV[dt_name]
    if dt == torch.bfloat16:
        arr = np.frombuffer(raw, dtype=np.int16).copy()
        return torch.from_numpy(arr).view(torch.bfloat16).reshape(shape)
    if dt == torch.bool:
        return torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(torch.bool).reshape(shape)
    npdt = {torch.float32: np.float32, torch.float16: np.float16, torch.int64: np.int64, torch.int32: np.int32,
            torch.uint8: np.uint8, torch.int8: np.int8}[dt]
    return torch.from_numpy(np.frombuffer(raw, dtype=npdt).copy()).reshape(shape)


async def read_message(reader: asyncio.StreamReader) -> Message:
    prefix = await reader.readexactly(12)
    hl, n = native.unpack_fixed(prefix)
    lens_raw = await reader.readexactly(8 * n) if n else b""
    lens = np.frombuffer(lens_raw, dtype="<u8").tolist() if n else []
    if sum(lens) > MAX_FRAME:
        raise ValueError("frame too large")
    header = msgpack.unpackb(await reader.readexactly(hl), raw=False)
    tensors = []
    for spec, ln in zip(header.get("t", []), lens):
        tensors.append(_decode_tensor(spec, await reader.readexactly(ln)))
    return Message(metadata=header.get("m") or {}, tensors=tensors, kind=header.get("k", "req"),
                   name=header.get("n", ""), rid=int(header.get("r", 0)))


async def write_message(writer: asyncio.StreamWriter, msg: Message) -> None:
    writer.writelines(encode(msg))
    await writer.drain()


def split_for_streaming(t: torch.Tensor, max_bytes: int) -> List[torch.Tensor]:
    """Chunk a tensor along dim 0 (the reference's ``split_for_streaming``, rpc_transport.py:551-562)."""
    if t.numel() * t.element_size() <= max_bytes or t.shape[0] <= 1:
        return [t]
    row = max(1, t[0].numel() * t.element_size())
    per = max(1, max_bytes // row)
    return list(torch.split(t, per, dim=0))


# ---------------------------------------------------------------- addresses
def parse_peer_address(addr: str) -> Tuple[str, int, Optional[str]]:
    """``/ip4/H/tcp/P[/p2p/ID]`` (multiaddr, like the reference), ``host:port`` or ``tcp://host:port``."""
    a = addr.strip()
    if a.startswith("/"):
        parts = [p for p in a.split("/") if p]
        host, port, pid = None, None, None
        for i in range(0, len(parts) - 1, 2):
            k, v = parts[i], parts[i + 1]
            if k in ("ip4", "ip6", "dns", "dns4", "dns6"):
                host = v
            elif k == "tcp":
                port = int(v)
            elif k == "p2p":
                pid = v
        if host is None or port is None:
            raise ValueError(f"bad multiaddr {addr!r}")
        return host, port, pid
    if a.startswith("tcp://"):
        a = a[len("tcp://"):]
    if ":" not in a:
        raise ValueError(f"bad peer address {addr!r} (want host:port or /ip4/.../tcp/...)")
    host, port = a.rsplit(":", 1)
    return host, int(port), None


def make_maddr(host: str, port: int, peer_id: Optional[str] = None) -> str:
    s = f"/ip4/{host}/tcp/{port}"
    return s + (f"/p2p/{peer_id}" if peer_id else "")
