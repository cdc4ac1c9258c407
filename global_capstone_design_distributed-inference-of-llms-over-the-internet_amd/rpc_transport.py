"""Client transport (``RpcTransport``): routes a session's activations through the swarm.

Same public API as the reference (src/rpc_transport.py:45-863): ``send_prefill``,
``send_decode_step``, ``recv_token``, ``shutdown``, per-hop timings in
``last_prefill_stage_times`` / ``last_decode_stage_times`` / ``decode_stage_history``,
``routing="stage"`` (fixed ``mini_petals:stage1..N`` keys) or ``routing="module"`` (greedy
cover of blocks [start_block, total_blocks) from ``petals:module:*`` records: pick the
candidate with the largest end block, ties by throughput, pin the route per session).

Fault tolerance (Petals-style, reference :587-712) with the reference's defects fixed:

* the per-hop input history is appended only AFTER a hop succeeded, so a replay never
  contains the step being retried (reference: :741, :805 append first -> duplicate step);
* a failed hop is re-routed from ITS start block: the replacement may have a different
  span (module routing), so the route tail is recomputed and the session's history is
  replayed hop-by-hop through the new tail (each replayed hop's outputs become the next
  new hop's history) - the reference re-discovers under the same key and may pick a peer
  with a different end block (:270-353);
* recovery success is not reported as failure on the last attempt (reference :659-661).

``push=True`` switches the data path to server-to-server forwarding (upstream Petals
``rpc_push``): the client sends the step to the first hop with the rest of the route in
``next_hops``; each server forwards its output to the next and the final token comes back
along the chain together with every hop's output, so the client still records the per-hop
history it needs for replay.  One client round trip per token instead of one per stage;
a downstream failure comes back as ``push_failed_at`` and is recovered like a star-mode
failure of that hop.

``hidden`` may be a GPU tensor; only the CPU copy crosses the wire.
"""
from __future__ import annotations

import asyncio
import logging
import os
import random
import time
from typing import Any, Dict, List, Optional, Sequence, Set, Tuple

import torch

from .comm.registry import DHT, get_dht_time
from .comm.rpc import DEFAULT_MAX_MSG_SIZE, MAX_UNARY_PAYLOAD_SIZE, RemoteError, RpcClient, get_loop
from .comm.wire import Message
from .dht_utils import get_module_entries, get_stage_key

logger = logging.getLogger(__name__)

HANDLER = "StageConnectionHandler.rpc_forward"
HANDLER_STREAM = "StageConnectionHandler.rpc_forward_stream"
RECOVERABLE = (asyncio.TimeoutError, ConnectionError, OSError, RemoteError)


class Hop:
    """One hop of a route: a peer serving blocks [start, end) (``key`` names the record it came from)."""

    def __init__(self, key: str, peer_id: str, maddrs: List[str], start: int, end: int, final: bool,
                 info: Optional[dict] = None):
        self.key, self.peer_id, self.maddrs = key, peer_id, list(maddrs)
        self.start, self.end, self.final = start, end, final
        self.info = dict(info or {})  # the registry record (channel_host / device for device channels)

    @property
    def expect_hidden(self) -> bool:
        return not self.final

    def __repr__(self):
        return f"Hop({self.key}, {self.peer_id[:8]}, [{self.start},{self.end}), final={self.final})"


class RpcTransport:
    def __init__(self, device, stage: int, dht_initial_peers: Sequence[str], dht_port: int = 8000,
                 rpc_port: int = 8001, timeout: float = 30.0, temperature: float = 1.0, top_p: float = 0.92,
                 top_k: int = 50, stage_keys: Optional[List[str]] = None, routing: str = "stage",
                 model_name: str = "default", total_blocks: Optional[int] = None, start_block: int = 0,
                 dht: Optional[DHT] = None, repetition_penalty: Optional[float] = None, max_recovery_attempts: int = 3,
                 push: bool = False):
        self.device = device
        self.stage = stage
        self.dht_port, self.rpc_port = dht_port, rpc_port
        self.timeout = timeout
        self.routing = routing
        self.model_name = model_name
        self.total_blocks = total_blocks
        self.start_block = start_block
        self.stage_keys = stage_keys or [get_stage_key(i) for i in (1, 2, 3)]
        self.sampling: Dict[str, Any] = {"temperature": float(temperature), "top_p": float(top_p), "top_k": int(top_k)}
        if repetition_penalty is not None:
            self.sampling["repetition_penalty"] = float(repetition_penalty)
        self.max_recovery_attempts = max_recovery_attempts
        self.push = bool(push)
        self._last_token: Optional[int] = None
        self.last_prefill_stage_times: List[Tuple[str, float]] = []
        self.last_prefill_total: Optional[float] = None
        self.last_decode_stage_times: List[Tuple[str, float]] = []
        self.last_decode_total: Optional[float] = None
        self.decode_stage_history: List[List[Tuple[str, float]]] = []
        self.decode_total_times: List[float] = []
        self.failed_peers: Dict[str, Set[str]] = {}
        self.session_routes: Dict[str, List[Hop]] = {}
        # history[session][hop_start_block] = list of inputs successfully sent to the hop at that block
        self.client_cache: Dict[str, Dict[int, List[torch.Tensor]]] = {}
        self._own_dht = dht is None
        self.dht = dht or DHT(start=True, initial_peers=list(dht_initial_peers or []))
        self.loop = get_loop()
        self.client = RpcClient()
        self.peer_id = self.dht.peer_id
        logger.info(f"RpcTransport initialized: stage={stage}, routing={routing}")

    # ------------------------------------------------------------------ sync helpers
    def _run(self, coro):
        return self.loop.run(coro)

    # ------------------------------------------------------------------ discovery
    def _candidates(self, key: str, block: Optional[int] = None) -> List[dict]:
        """Live records under ``key`` (stage keys) or covering ``block`` (module keys)."""
        if block is not None:
            ents = list(get_module_entries(self.dht, block, self.model_name).values())
            return [e for e in ents if e.get("start_block") is not None and e.get("end_block") is not None
                    and int(e["start_block"]) <= block < int(e["end_block"])]
        res = self.dht.get(key, latest=True)
        if res is None:
            return []
        val = res.value
        if isinstance(val, dict) and "peer_id" in val and "p2p_maddrs" in val:
            return [val]
        out = []
        if isinstance(val, dict):
            for sk, raw in val.items():
                e = raw.value if hasattr(raw, "value") else raw
                if isinstance(e, dict):
                    e = dict(e)
                    e.setdefault("peer_id", str(sk))
                    out.append(e)
        return out

    def _discover_peer(self, key: str, exclude: Set[str] = frozenset(), block: Optional[int] = None,
                       max_retries: int = 10, retry_delay: float = 1.0) -> dict:
        for attempt in range(max_retries):
            cands = [e for e in self._candidates(key, block) if str(e.get("peer_id")) not in exclude]
            if cands:
                cands.sort(key=lambda e: float(e.get("timestamp", 0.0)), reverse=True)
                return random.choice(cands[:5])
            time.sleep(retry_delay)
        raise RuntimeError(f"no live peer for {key} (excluded {len(exclude)})")

    def _stage_hop(self, i: int, exclude: Set[str] = frozenset(), retries: int = 10, delay: float = 1.0) -> Hop:
        key = self.stage_keys[i]
        e = self._discover_peer(key, exclude, max_retries=retries, retry_delay=delay)
        final = i == len(self.stage_keys) - 1
        return Hop(key, str(e["peer_id"]), e.get("p2p_maddrs") or [], int(e.get("start_block", i)),
                   int(e.get("end_block", i + 1)), final, e)

    def _module_route(self, cur: int, exclude: Set[str] = frozenset()) -> List[Hop]:
        if self.total_blocks is None:
            raise ValueError("total_blocks is required when routing='module'")
        hops: List[Hop] = []
        while cur < self.total_blocks:
            cands = [e for e in self._candidates("", cur) if str(e.get("peer_id")) not in exclude]
            if not cands:
                raise RuntimeError(f"[module routing] no server covers block={cur}")
            cands.sort(key=lambda e: (int(e["end_block"]), float(e.get("throughput") or 0.0)), reverse=True)
            e = cands[0]
            end = int(e["end_block"])
            final = end >= self.total_blocks
            if final and not bool(e.get("final_stage", False)):
                raise RuntimeError("[module routing] last hop server is not a final stage (needs lm_head)")
            hops.append(Hop(f"petals:module:{self.model_name}:block_{cur}", str(e["peer_id"]),
                            e.get("p2p_maddrs") or [], cur, end, final, e))
            cur = end
            if len(hops) > self.total_blocks + 5:
                raise RuntimeError("[module routing] route did not converge")
        logger.info(f"[module routing] route: {hops}")
        return hops

    def _get_route(self, session_id: str) -> List[Hop]:
        if session_id not in self.session_routes:
            if self.routing == "module":
                self.session_routes[session_id] = self._module_route(int(self.start_block))
            else:
                self.session_routes[session_id] = [self._stage_hop(i) for i in range(len(self.stage_keys))]
        return self.session_routes[session_id]

    def _route_tail(self, route: List[Hop], k: int, exclude: Set[str]) -> List[Hop]:
        if self.routing == "module":
            return self._module_route(route[k].start, exclude)
        return [self._stage_hop(i, exclude if i == k else frozenset(), retries=5, delay=0.5)
                for i in range(k, len(self.stage_keys))]

    # ------------------------------------------------------------------ calls
    async def _call(self, hop: Hop, x: torch.Tensor, md: dict) -> Message:
        if not hop.maddrs:
            raise ConnectionError(f"peer {hop.peer_id[:8]} announced no addresses")
        nbytes = x.numel() * x.element_size()
        last_err = None
        for addr in hop.maddrs:
            try:
                if nbytes > MAX_UNARY_PAYLOAD_SIZE // 2:
                    return await self.client.call(addr, HANDLER_STREAM, Message(md, [x]), self.timeout,
                                                  stream_chunk_bytes=DEFAULT_MAX_MSG_SIZE)
                return await self.client.call(addr, HANDLER, Message(md, [x]), self.timeout)
            except (ConnectionError, OSError) as e:
                last_err = e
                continue
        raise last_err if last_err else ConnectionError("no address reachable")

    @staticmethod
    def _token_of(resp: Message) -> int:
        if resp.metadata.get("token_id") is not None:
            return int(resp.metadata["token_id"])
        return int(resp.tensors[0].reshape(-1)[0])

    async def _replay_tail(self, session_id: str, route: List[Hop], k: int, base_md: dict) -> None:
        """Rebuild KV on hops route[k:] by replaying the history recorded at hop k's start block."""
        hist = self.client_cache.get(session_id, {})
        inputs = list(hist.get(route[k].start, []))
        if not inputs:
            return
        new_hist: Dict[int, List[torch.Tensor]] = {}
        for j in range(k, len(route)):
            hop = route[j]
            new_hist[hop.start] = list(inputs)
            outs = []
            cum = 0
            for idx, x in enumerate(inputs):
                cum += int(x.shape[1])
                md = dict(base_md, session_id=session_id, seq_len=int(x.shape[1]), cur_len=cum,
                          is_prefill=idx == 0, is_replay=True)
                resp = await self._call(hop, x, md)
                if hop.expect_hidden:
                    outs.append(resp.tensors[0])
            inputs = outs
            if not hop.expect_hidden:
                break
        hist.update(new_hist)
        self.client_cache[session_id] = hist

    def _record(self, session_id: str, hop: Hop, x: torch.Tensor) -> None:
        self.client_cache.setdefault(session_id, {}).setdefault(hop.start, []).append(x.clone())

    async def _send(self, session_id: str, hidden: torch.Tensor, md: dict, which: str):
        t_all = time.perf_counter()
        x = hidden.detach().to("cpu")
        if x.dim() == 2:
            x = x.unsqueeze(0)
        route = self.session_routes[session_id]  # resolved by the caller (outside the event loop)
        times: List[Tuple[str, float]] = []
        k = 0
        attempts = 0
        while k < len(route):
            hop = route[k]
            t0 = time.perf_counter()
            failed_exc: Optional[BaseException] = None
            resp = None
            push = self.push and k + 1 < len(route)
            try:
                call_md = md
                if push:
                    call_md = dict(md, next_hops=[{"key": h.key, "peer_id": h.peer_id, "maddrs": h.maddrs}
                                                  for h in route[k + 1:]])
                resp = await self._call(hop, x, call_md)
            except RECOVERABLE as e:
                failed_exc = e
            if resp is not None and push:
                # chain reply: outputs of hops k.. (+ token if the chain completed)
                pf = resp.metadata.get("push_failed_at")
                final = pf is None
                hiddens = list(resp.tensors[1:] if final else resp.tensors)
                j = len(route) if final else k + int(pf)
                inp = x
                for i in range(k, j):
                    self._record(session_id, route[i], inp)
                    if i - k < len(hiddens):
                        inp = hiddens[i - k]
                        if inp.dim() == 2:
                            inp = inp.unsqueeze(0)
                times.append((f"push:{hop.key}", time.perf_counter() - t0))
                if final:
                    return self._finish(which, times, t_all, resp)
                x, k, hop = inp, j, route[j]
                failed_exc = ConnectionError(resp.metadata.get("push_error", "push failed"))
            if failed_exc is not None:
                attempts += 1
                logger.warning(f"hop {hop} failed ({type(failed_exc).__name__}: {failed_exc}); recovery {attempts}/"
                               f"{self.max_recovery_attempts}")
                self.failed_peers.setdefault(hop.key, set()).add(hop.peer_id)
                self.client.drop(hop.maddrs[0]) if hop.maddrs else None
                if attempts > self.max_recovery_attempts:
                    raise RuntimeError(f"failed to recover {hop.key} after {self.max_recovery_attempts} attempts") \
                        from failed_exc
                exclude = set().union(*self.failed_peers.values())
                try:
                    tail = await asyncio.get_running_loop().run_in_executor(None, self._route_tail, route, k, exclude)
                    route = route[:k] + tail
                    self.session_routes[session_id] = route
                    base = {kk: v for kk, v in md.items() if kk not in ("seq_len", "cur_len", "is_prefill")}
                    await self._replay_tail(session_id, route, k, base)
                except RECOVERABLE + (RuntimeError,) as re:
                    logger.error(f"recovery attempt failed: {re}")
                    await asyncio.sleep(0.5)
                continue
            times.append((hop.key, time.perf_counter() - t0))
            self._record(session_id, hop, x)
            if hop.expect_hidden:
                x = resp.tensors[0]
                if x.dim() == 2:
                    x = x.unsqueeze(0)
                k += 1
                continue
            return self._finish(which, times, t_all, resp)
        raise RuntimeError("No final stage returned a token")

    def _finish(self, which: str, times, t_all: float, resp: Message) -> int:
        total = time.perf_counter() - t_all
        if which == "prefill":
            self.last_prefill_stage_times, self.last_prefill_total = times, total
        else:
            self.last_decode_stage_times, self.last_decode_total = times, total
            self.decode_stage_history.append(times)
            self.decode_total_times.append(total)
        return self._token_of(resp)

    # ------------------------------------------------------------------ public API
    def send_prefill(self, L: int, hidden: torch.Tensor, session_id: str, max_length: int):
        if self.stage != 0:
            raise RuntimeError("send_prefill should only be called by stage0")
        self.client_cache.pop(session_id, None)
        md = {"session_id": session_id, "seq_len": int(L), "cur_len": int(L), "is_prefill": True,
              "max_length": int(max_length), **self.sampling}
        self._get_route(session_id)
        self._last_token = self._run(self._send(session_id, hidden, md, "prefill"))

    def send_decode_step(self, cur_len: int, hidden: torch.Tensor, session_id: str, max_length: int,
                         generated_tokens: Optional[List[int]] = None):
        if self.stage != 0:
            raise RuntimeError("send_decode_step should only be called by stage0")
        md = {"session_id": session_id, "seq_len": 1, "cur_len": int(cur_len), "is_prefill": False,
              "max_length": int(max_length), "generated_tokens": list(generated_tokens or [])[-50:], **self.sampling}
        self._get_route(session_id)
        self._last_token = self._run(self._send(session_id, hidden, md, "decode"))

    def send_steps(self, steps: Sequence[Tuple[str, torch.Tensor, int, int, int, Optional[List[int]]]]) -> List[int]:
        """Concurrent sessions over TCP: one step (prefill when ``seq_len == cur_len``, else
        decode) for each ``(session_id, hidden, seq_len, cur_len, max_length, generated)``,
        all in flight at once so each server's batching window (rpc_handler ``_drain``) runs
        them as one ragged step.  Returns the sessions' next tokens, in order.  Per-session
        recovery is unchanged (every ``_send`` excludes, re-routes and replays on its own)."""
        if self.stage != 0:
            raise RuntimeError("send_steps should only be called by stage0")

        async def _all():
            coros = []
            for sid, hidden, L, cur, mx, gen in steps:
                pre = int(L) == int(cur)
                if pre:
                    self.client_cache.pop(sid, None)
                md = {"session_id": sid, "seq_len": int(L), "cur_len": int(cur), "is_prefill": pre,
                      "max_length": int(mx), **self.sampling}
                if not pre:
                    md["generated_tokens"] = list(gen or [])[-50:]
                coros.append(self._send(sid, hidden, md, "prefill" if pre else "decode"))
            return await asyncio.gather(*coros)

        for sid, *_ in steps:
            self._get_route(sid)
        return [int(t) for t in self._run(_all())]

    def recv_token(self) -> int:
        if self.stage != 0:
            raise RuntimeError("recv_token should only be called by stage0")
        if self._last_token is None:
            raise RuntimeError("No token received. Call send_prefill or send_decode_step first.")
        t, self._last_token = self._last_token, None
        return int(t)

    def close_session(self, session_id: str) -> None:
        """Free the session's KV pages on every hop (not in the reference: its caches leak)."""
        route = self.session_routes.pop(session_id, [])
        self.client_cache.pop(session_id, None)

        async def _close():
            for hop in route:
                for addr in hop.maddrs[:1]:
                    try:
                        await self.client.call(addr, "StageConnectionHandler.rpc_close_session",
                                               Message({"session_id": session_id}), timeout=5.0)
                    except Exception:
                        pass

        try:
            self._run(_close())
        except Exception:
            pass

    # ------------------------------------------------------------------ same-node device channel
    def device_channel_possible(self, route: List[Hop], device) -> bool:
        """GPU client and every hop announced a device channel on THIS machine.  (CPU swarms stay
        on the TCP RPC path: BASELINE config 1 is "rpc_transport over localhost"; ``--device_channel
        on`` forces the channel anyway, over gloo.)"""
        from .parallel.channel import host_id

        me = host_id()
        return torch.device(device).type == "cuda" and bool(route) and route[-1].final and \
            all(h.info.get("channel_host") == me for h in route)

    def channel_routes(self, device, max_routes: Optional[int] = None, exclude: Set[str] = frozenset(),
                       same_node: bool = True, wait_s: float = 10.0) -> List[List[Hop]]:
        """Disjoint complete routes for device channels: the node's pipeline replicas.

        Every server hosts at most one route (a server's stage executor serves any number of
        channels, but two replicas on one GPU would just share it).  With ``same_node`` only
        servers that announced a device channel on this machine qualify.  Stage routing takes
        one server per ``mini_petals:stage{k}`` key, newest record first; module routing
        covers [start_block, total_blocks) greedily (largest end block, then throughput), as
        ``_module_route`` does.  Waits up to ``wait_s`` for the FIRST route to appear."""
        from .parallel.channel import host_id

        me = host_id()
        used = set(exclude) | set().union(*self.failed_peers.values()) if self.failed_peers else set(exclude)

        def ok(e) -> bool:
            return str(e.get("peer_id")) not in used and (not same_node or e.get("channel_host") == me)

        def one() -> Optional[List[Hop]]:
            hops: List[Hop] = []
            if self.routing == "module":
                cur = int(self.start_block)
                while cur < int(self.total_blocks):
                    cands = [e for e in self._candidates("", cur) if ok(e)]
                    if not cands:
                        return None
                    cands.sort(key=lambda e: (int(e["end_block"]), float(e.get("throughput") or 0.0)), reverse=True)
                    e = cands[0]
                    end = int(e["end_block"])
                    final = end >= int(self.total_blocks)
                    if final and not bool(e.get("final_stage", False)):
                        return None
                    hops.append(Hop(f"petals:module:{self.model_name}:block_{cur}", str(e["peer_id"]),
                                    e.get("p2p_maddrs") or [], cur, end, final, e))
                    cur = end
                return hops
            for i, key in enumerate(self.stage_keys):
                cands = [e for e in self._candidates(key) if ok(e)]
                if not cands:
                    return None
                cands.sort(key=lambda e: (-float(e.get("timestamp", 0.0)), str(e.get("peer_id"))))
                e = cands[0]
                hops.append(Hop(key, str(e["peer_id"]), e.get("p2p_maddrs") or [], int(e.get("start_block", i)),
                                int(e.get("end_block", i + 1)), i == len(self.stage_keys) - 1, e))
            return hops

        routes: List[List[Hop]] = []
        t0 = time.monotonic()
        while max_routes is None or len(routes) < max_routes:
            r = one()
            if r is None:
                if routes or time.monotonic() - t0 > wait_s:
                    break
                time.sleep(0.25)
                continue
            routes.append(r)
            used |= {h.peer_id for h in r}
        return routes

    def replacement_hop(self, dead: Hop, device, exclude: Set[str] = frozenset(), same_node: bool = True,
                        wait_s: float = 10.0) -> Optional[Hop]:
        """A server that can take the place of ``dead`` in a device-channel route: the same stage
        key (stage routing) or exactly the same block span [start, end) (module routing - a
        different span would shift every later stage), not in ``exclude`` nor failed, on this
        machine if ``same_node``; newest record first.  Stage-local recovery swaps only this hop
        (``_run_rank0_channel``'s ``recover``).  Waits up to ``wait_s``; None if nothing qualifies."""
        from .parallel.channel import host_id

        me = host_id()
        used = set(exclude) | set().union(*self.failed_peers.values()) if self.failed_peers else set(exclude)
        used.add(dead.peer_id)
        t0 = time.monotonic()
        while True:
            if self.routing == "module":
                cands = [e for e in self._candidates("", dead.start) if int(e["end_block"]) == dead.end]
            else:
                cands = list(self._candidates(dead.key))
            cands = [e for e in cands if str(e.get("peer_id")) not in used and
                     (not same_node or e.get("channel_host") == me) and
                     (not dead.final or bool(e.get("final_stage", dead.final)))]
            if cands:
                cands.sort(key=lambda e: (-float(e.get("timestamp", 0.0)), str(e.get("peer_id"))))
                e = cands[0]
                return Hop(dead.key, str(e["peer_id"]), e.get("p2p_maddrs") or [], dead.start, dead.end, dead.final, e)
            if time.monotonic() - t0 > wait_s:
                return None
            time.sleep(0.25)

    def hop_alive(self, hop: Hop, timeout: float = 2.0) -> bool:
        """Does the hop's server still answer (``rpc_echo`` over TCP)?  Failure detection for
        device-channel routes: a channel error names no culprit, the TCP control plane does."""
        async def ping():
            for addr in hop.maddrs:
                try:
                    await self.client.call(addr, "StageConnectionHandler.rpc_echo", Message({"ping": True}), timeout)
                    return True
                except Exception:  # noqa: BLE001 - any failure = not alive on this address
                    self.client.drop(addr)
            return False

        try:
            return bool(self._run(ping()))
        except Exception:  # noqa: BLE001
            return False

    def open_device_channel(self, route: List[Hop], device, *, n_slots: int = 1, batch: int = 64,
                            timeout: float = 60.0, idle_timeout: float = 3600.0, timing: bool = False,
                            data_backend: Optional[str] = None, replay_cache: bool = False,
                            resume_prefix: Optional[str] = None):
        """Rendezvous a ``parallel.channel.Channel`` with every hop of ``route``: this client
        is rank 0 (head), hop i is rank i + 1, the final hop the tail.  The TCP RPC carries
        only this handshake; afterwards hidden states move GPU -> GPU (RCCL over xGMI) and the
        tail returns token ids on the channel.  Payloads are staged through gloo when two
        participants share a GPU (RCCL refuses duplicate devices) or on CPU.  ``data_backend``
        (``--channel_data``) picks the GPU data plane: "nccl" (ProcessGroupNCCL, default) or "rccl"
        (the framework's own communicators, ``parallel/rccl.py``; ``MPAMD_GRAPH_HOP=1`` then records
        the hop inside the decode graphs); None reads ``MPAMD_CHANNEL_DATA``.  ``replay_cache``
        makes every non-tail server keep its output rows for stage-local recovery; ``resume_prefix``
        (the failed channel's name) lets the servers of a replacement channel adopt that channel's
        sessions (``PipelineServingEngine.resume_sessions``)."""
        import uuid

        from .parallel.channel import Channel, free_port, host_id, make_store

        world = len(route) + 1
        devs = [str(torch.device(device))] + [str(h.info.get("device", "")) for h in route]
        gpu = torch.device(device).type == "cuda"
        want = data_backend or os.environ.get("MPAMD_CHANNEL_DATA") or "nccl"
        data = want if gpu and len(set(devs)) == len(devs) and want in ("nccl", "rccl") else "gloo"
        port = free_port("127.0.0.1")
        store = make_store("127.0.0.1", port, world, True, timeout_s=timeout)
        prefix = f"chan-{uuid.uuid4().hex[:12]}"

        async def _open():
            for i, hop in enumerate(route):
                md = {"store_host": "127.0.0.1", "store_port": port, "prefix": prefix, "rank": i + 1, "world": world,
                      "timeout": timeout, "idle_timeout": idle_timeout, "data_backend": data, "n_slots": n_slots,
                      "batch": batch, "host_id": host_id(), "timing": bool(timing),
                      "replay_cache": bool(replay_cache), "resume_prefix": resume_prefix}
                r = await self._call_hop(hop, "rpc_channel_open", [], md)
                if not r.metadata.get("ok"):
                    raise ConnectionError(f"{hop}: device channel refused: {r.metadata.get('error')}")

        self._run(_open())
        ch = Channel(store, prefix, 0, world, device, timeout_s=timeout, data_backend=data)
        ch._store = store  # the client hosts the rendezvous store: keep it alive with the channel
        logger.info(f"device channel {prefix}: {world} ranks, data over {data}")
        return ch

    # ------------------------------------------------------------------ fine-tuning (stateless)
    def _fresh_route(self) -> List[Hop]:
        if self.routing == "module":
            return self._module_route(int(self.start_block))
        return [self._stage_hop(i) for i in range(len(self.stage_keys))]

    def _prompt_slice(self, prompts: Optional[torch.Tensor], hop: Hop) -> List[torch.Tensor]:
        if prompts is None:
            return []
        a, b = hop.start - int(self.start_block), hop.end - int(self.start_block)
        return [prompts[a:b].contiguous()]

    async def _call_hop(self, hop: Hop, name: str, tensors: List[torch.Tensor], md: dict) -> Message:
        last_err = None
        for addr in hop.maddrs:
            try:
                return await self.client.call(addr, "StageConnectionHandler." + name, Message(md, tensors),
                                              self.timeout * 4)
            except (ConnectionError, OSError) as e:
                last_err = e
        raise last_err if last_err else ConnectionError(f"peer {hop.peer_id[:8]} announced no addresses")

    def _stateless_hop(self, route: List[Hop], k: int, name: str, tensors_of, md: dict) -> Tuple[Message, List[Hop]]:
        """Call hop k; on failure re-route from its start block (stateless: nothing to replay)."""
        for attempt in range(self.max_recovery_attempts + 1):
            hop = route[k]
            try:
                return self._run(self._call_hop(hop, name, tensors_of(hop), md)), route
            except RECOVERABLE as e:
                if attempt == self.max_recovery_attempts:
                    raise
                logger.warning(f"[stateless] {name} failed at {hop}: {e!r}; re-routing")
                self.failed_peers.setdefault("__stateless__", set()).add(hop.peer_id)
                tail = self._route_tail(route, k, self.failed_peers["__stateless__"])
                if tail[0].start != hop.start:
                    raise
                route = route[:k] + tail
        raise RuntimeError("unreachable")

    def forward_stateless(self, hidden: torch.Tensor, prompts: Optional[torch.Tensor] = None,
                          route: Optional[List[Hop]] = None):
        """Run [B, T, H] hidden states through every remote block without a session (upstream
        ``rpc_forward`` as the training client uses it). ``prompts`` are deep prompts for the
        remote blocks, ``[total_blocks - start_block, B|1, P, H]``; each hop receives its own
        slice. Returns ``(output, per_hop_inputs, route)``; keep the last two for
        :meth:`backward_stateless`."""
        x = hidden.detach().to("cpu")
        if x.dim() == 2:
            x = x.unsqueeze(0)
        p = prompts.detach().to("cpu") if prompts is not None else None
        route = list(route or self._fresh_route())
        md = {"stateless": True, "has_prompts": p is not None}
        inputs = []
        k = 0
        while k < len(route):
            cur = x
            resp, route = self._stateless_hop(route, k, "rpc_forward", lambda h: [cur] + self._prompt_slice(p, h), md)
            inputs.append(x)
            x = resp.tensors[0]
            k += 1
        return x, inputs, route

    def backward_stateless(self, inputs: List[torch.Tensor], route: List[Hop], grad_output: torch.Tensor,
                           prompts: Optional[torch.Tensor] = None):
        """Backward through the route of a :meth:`forward_stateless` call, last hop first
        (upstream ``rpc_backward``). Returns ``(grad_hidden, grad_prompts or None)``."""
        g = grad_output.detach().to("cpu")
        if g.dim() == 2:
            g = g.unsqueeze(0)
        p = prompts.detach().to("cpu") if prompts is not None else None
        gp = torch.zeros_like(p) if p is not None else None
        md = {"stateless": True, "has_prompts": p is not None}
        route = list(route)
        for k in range(len(route) - 1, -1, -1):
            cur_g, inp = g, inputs[k]
            resp, route = self._stateless_hop(route, k, "rpc_backward",
                                              lambda h: [inp, cur_g] + self._prompt_slice(p, h), md)
            g = resp.tensors[0]
            if gp is not None:
                a, b = route[k].start - int(self.start_block), route[k].end - int(self.start_block)
                gp[a:b] += resp.tensors[1]
        return g, gp

    def remote_blocks(self, hidden: torch.Tensor, prompts: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Differentiable call of the remote blocks: gradients flow to ``hidden`` and ``prompts``
        (client-side prompt tuning, as with upstream ``RemoteSequential``)."""
        return _RemoteBlocks.apply(hidden, prompts if prompts is not None else torch.empty(0), self)

    def shutdown(self):
        try:
            self._run(self.client.close())
        except Exception:
            pass
        if self._own_dht:
            self.dht.shutdown()


class _RemoteBlocks(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hidden, prompts, tx):
        p = prompts if prompts.numel() else None
        out, inputs, route = tx.forward_stateless(hidden, p)
        ctx.tx, ctx.inputs, ctx.route, ctx.has_p = tx, inputs, route, p is not None
        ctx.hshape, ctx.hdtype, ctx.hdev = hidden.shape, hidden.dtype, hidden.device
        ctx.save_for_backward(prompts)
        return out.to(hidden.device, hidden.dtype).reshape(hidden.shape)

    @staticmethod
    def backward(ctx, grad):
        (prompts,) = ctx.saved_tensors
        gh, gp = ctx.tx.backward_stateless(ctx.inputs, ctx.route, grad, prompts if ctx.has_p else None)
        gh = gh.to(ctx.hdev, ctx.hdtype).reshape(ctx.hshape)
        gp = gp.to(prompts.device, prompts.dtype) if gp is not None else None
        return gh, gp, None
