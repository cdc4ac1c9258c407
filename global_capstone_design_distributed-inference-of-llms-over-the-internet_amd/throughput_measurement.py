"""Server throughput for load balancing: min(compute, network x (1 - relay penalty)).

Reference: src/throughput_measurement.py:15-263 measures the compute rate of the whole
served span with 2 warm-up + 10 timed ``[1,1,H]`` forwards and ``torch.cuda.synchronize``,
estimates the network rate as ``bandwidth_bps / (H * elt_size)`` (default 100 Mbit/s) times
``1 - 0.2`` (relay penalty), takes the minimum, and falls back to 10.0 rps.

Here the compute probe is a real decode step of the stage executor on a probe session
(paged KV, hipGraph replay where available), timed with HIP events; the network term can
also be *measured* on a live link (``measure_link_bandwidth``: round trips of an H-sized
activation over the framework's TCP transport) instead of assumed.

Upstream Petals (petals/server/throughput.py) additionally measures a
prefill rate (``forward_rps``, 1024-token forwards) and caches measurements in a JSON file
under a system-wide ``flock`` so restarts and co-located servers do not re-measure:
``measure_forward_throughput`` and ``ThroughputCache`` / ``get_server_throughput(cache=...)``.
"""
from __future__ import annotations

import contextlib
import fcntl
import json
import logging
import os
import time
import uuid
from typing import Optional

import torch

logger = logging.getLogger(__name__)

DEFAULT_NETWORK_MBPS = 100.0
RELAY_PENALTY = 0.2
FALLBACK_THROUGHPUT = 10.0


def measure_compute_throughput(executor, n_warmup: int = 2, n_steps: int = 10, batch: int = 1,
                               rounds: int = 3) -> float:
    """Decode steps per second of this stage's whole span (``batch`` probe sessions): the best of
    ``rounds`` timed rounds of ``n_steps`` steps (a server process also runs its registry and RPC
    threads; one round on a busy host under-reports a short span by 2x)."""
    H = executor.cfg.hidden_size
    dev = executor.device
    sids = [f"__probe_{uuid.uuid4().hex[:8]}_{i}" for i in range(batch)]
    # the probe shares the executor (scratch buffers, graphs, session table, stream) with the
    # served steps of the RPC handler / device-channel threads: it runs under their lock
    lock = getattr(executor, "exec_lock", None) or contextlib.nullcontext()
    with lock:
        return _measure_compute(executor, sids, batch, n_warmup, n_steps, rounds, H, dev)


def _measure_compute(executor, sids, batch, n_warmup, n_steps, rounds, H, dev) -> float:
    try:
        if executor.is_first:
            x = torch.randint(0, executor.cfg.vocab_size, (batch,), device=dev)
        else:
            x = torch.randn(batch, H, device=dev).to(executor.dtype)
        seqs = [(s, 1) for s in sids]
        for _ in range(n_warmup):
            executor.forward(seqs, x)
        best = float("inf")
        for _ in range(max(1, rounds)):
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(n_steps):
                    executor.forward(seqs, x)
                e1.record()
                e1.synchronize()
                dt = e0.elapsed_time(e1) / 1000.0
            else:
                t0 = time.perf_counter()
                for _ in range(n_steps):
                    executor.forward(seqs, x)
                dt = time.perf_counter() - t0
            best = min(best, dt)
        return n_steps / max(best, 1e-9)
    finally:
        for s in sids:
            executor.sessions.close(s)


def measure_forward_throughput(executor, n_tokens: int = 1024, n_steps: int = 3) -> float:
    """Prefill rate: tokens/s of ``n_tokens``-token forwards through the whole span (upstream
    ``forward_rps`` x tokens).  Each step is a fresh probe session (prefill from position 0)."""
    H = executor.cfg.hidden_size
    dev = executor.device
    n_tokens = int(min(n_tokens, executor.max_tokens, executor.max_seq_len))
    if executor.is_first:
        x = torch.randint(0, executor.cfg.vocab_size, (n_tokens,), device=dev)
    else:
        x = torch.randn(n_tokens, H, device=dev).to(executor.dtype)
    sid = f"__probe_fwd_{uuid.uuid4().hex[:8]}"
    lock = getattr(executor, "exec_lock", None) or contextlib.nullcontext()
    with lock:
        return _measure_forward(executor, sid, x, n_tokens, n_steps, dev)


def _measure_forward(executor, sid, x, n_tokens, n_steps, dev) -> float:
    try:
        executor.forward([(sid, n_tokens)], x, reset=[True])
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n_steps):
            executor.forward([(sid, n_tokens)], x, reset=[True])
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        return n_steps * n_tokens / max(time.perf_counter() - t0, 1e-9)
    finally:
        executor.sessions.close(sid)


class ThroughputCache:
    """JSON file of past measurements keyed by (model, span, dtype, device), guarded by an
    exclusive ``flock`` (upstream: one system-wide lock + ``throughput_v2.json``)."""

    def __init__(self, path: Optional[str] = None):
        self.path = path or os.path.join(os.path.expanduser(os.environ.get("MPAMD_CACHE_DIR", "~/.cache/mpamd")),
                                         "throughput_v1.json")

    @contextlib.contextmanager
    def _locked(self):
        os.makedirs(os.path.dirname(self.path), exist_ok=True)
        with open(self.path + ".lock", "w") as lf:
            fcntl.flock(lf, fcntl.LOCK_EX)
            try:
                yield
            finally:
                fcntl.flock(lf, fcntl.LOCK_UN)

    def _read(self) -> dict:
        try:
            with open(self.path) as f:
                return json.load(f)
        except (OSError, ValueError):
            return {}

    @staticmethod
    def key(executor, batch: int = 1) -> str:
        dev = executor.device
        name = torch.cuda.get_device_name(dev) if dev.type == "cuda" else "cpu"
        return f"{executor.cfg.name}|{executor.start}-{executor.end}|{executor.dtype}|{name}|b{int(batch)}"

    def get(self, key: str) -> Optional[dict]:
        with self._locked():
            return self._read().get(key)

    def put(self, key: str, value: dict) -> None:
        with self._locked():
            d = self._read()
            d[key] = value
            tmp = self.path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(d, f, indent=1, sort_keys=True)
            os.replace(tmp, self.path)


def estimate_network_throughput(hidden_size: int, dtype_bytes: int = 2,
                                bandwidth_mbps: Optional[float] = None) -> float:
    """Requests/s the link can carry for one [1, 1, H] activation (reference :157-190)."""
    mbps = DEFAULT_NETWORK_MBPS if bandwidth_mbps is None else float(bandwidth_mbps)
    bits_per_request = hidden_size * dtype_bytes * 8
    return (mbps * 1e6) / bits_per_request


def get_server_throughput(executor, network_bandwidth_mbps: Optional[float] = None,
                          relay_penalty: float = RELAY_PENALTY, n_warmup: int = 2, n_steps: int = 10,
                          cache: Optional[ThroughputCache] = None, force_eval: bool = False, batch: int = 1) -> float:
    """min(compute, network x (1 - relay penalty)) in tokens/s.

    ``batch``: the compute term is measured as ``batch`` concurrent one-token decode steps
    (tokens/s = batch x steps/s): a stage serves many sessions at once, and batch 1 (the
    reference's probe) under-reports an MI355X span by an order of magnitude.  The network term
    is per token too, so the two stay comparable.  ``network_bandwidth_mbps`` is the MEASURED
    link rate when the caller has one (``measure_link_bandwidth``), else the 100 Mbit/s
    assumption of the reference."""
    key = ThroughputCache.key(executor, batch) if cache is not None else None
    cached = cache.get(key) if (cache is not None and not force_eval) else None
    if cached and "compute_rps" in cached:
        compute = float(cached["compute_rps"])
        logger.info(f"Server throughput: cached compute={compute:.2f} rps ({key})")
    else:
        try:
            compute = batch * measure_compute_throughput(executor, n_warmup, n_steps, batch=batch)
        except Exception as e:
            logger.warning(f"compute throughput probe failed ({e!r}); using fallback {FALLBACK_THROUGHPUT}")
            return FALLBACK_THROUGHPUT
        if cache is not None:
            cache.put(key, {"compute_rps": compute, "measured_at": time.time()})
    elt = torch.tensor([], dtype=executor.dtype).element_size()
    network = estimate_network_throughput(executor.cfg.hidden_size, elt, network_bandwidth_mbps) * (1 - relay_penalty)
    final = min(compute, network)
    logger.info(f"Server throughput: compute={compute:.2f} rps, network={network:.2f} rps, final={final:.2f} rps")
    return float(final)


def measure_link_bandwidth(rpc_call, payload_bytes: int, rounds: int = 5) -> float:
    """Mbit/s measured with ``rpc_call(bytes)`` round trips (echo handler on the peer): the
    measured replacement of the reference's speedtest / 100 Mbit/s constant
    (src/throughput_measurement.py:157-190, petals/server/throughput.py:147-187)."""
    rpc_call(payload_bytes)
    t0 = time.perf_counter()
    for _ in range(rounds):
        rpc_call(payload_bytes)
    dt = (time.perf_counter() - t0) / rounds
    return 2 * payload_bytes * 8 / dt / 1e6


def measure_peer_bandwidth(maddrs, hidden_size: int, dtype=torch.bfloat16, tokens: int = 256, rounds: int = 4,
                           timeout: float = 10.0) -> Optional[float]:
    """Measured Mbit/s to the first reachable address in ``maddrs``: ``rpc_echo`` round trips of
    a [1, tokens, H] activation (a prefill-sized message, so the number is bandwidth rather than
    RPC latency).  None if no address answers."""
    from .comm.rpc import RpcClient, get_loop
    from .comm.wire import Message

    loop = get_loop()
    client = RpcClient()
    x = torch.zeros(1, tokens, hidden_size, dtype=dtype)
    try:
        for addr in maddrs:
            def call(nbytes, addr=addr):
                loop.run(client.call(addr, "StageConnectionHandler.rpc_echo", Message({"bw": True}, [x]), timeout),
                         timeout=timeout + 1)
            try:
                return measure_link_bandwidth(call, x.numel() * x.element_size(), rounds)
            except Exception as e:  # noqa: BLE001 - try the next address
                logger.info(f"bandwidth probe to {addr} failed: {e!r}")
        return None
    finally:
        try:
            loop.run(client.close(), timeout=2)
        except Exception:  # noqa: BLE001
            pass
