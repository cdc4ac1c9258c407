"""Stage server RPC handler (``StageConnectionHandler``).

Reference: src/rpc_handler.py:43-464 - a hivemind ConnectionHandler whose
``rpc_forward`` / ``rpc_forward_stream`` handlers run the stage on one session's hidden
states, keep that session's KV tuple in a dict forever, and (final stage) sample the next
token server-side.  This implementation keeps the handler names, request metadata and
reply format, and changes the engine underneath:

* the stage is a ``StageExecutor`` (HIP kernels, paged KV in HBM, hipGraph decode);
* **continuous batching**: requests from different sessions that arrive together are
  executed as ONE ragged step (``batch_window_ms``), on a single GPU worker thread so the
  asyncio loop never blocks on the device;
* KV sessions have ``max_length`` enforced and expire after a TTL (no leak);
* position bookkeeping is idempotent: a decode step carries ``cur_len``, so a retried or
  replayed step overwrites its own slot instead of appending twice (the reference's replay
  duplicates the current step);
* extra handlers beyond the reference, from the upstream Petals server surface the reference
  vendors (petals/server/handler.py): ``rpc_info`` (free cache
  tokens), ``rpc_inference`` (per-step session API with ``step_id`` de-duplication and
  ``start_from_position`` rewind), server-to-server **push** (a request carrying
  ``next_hops`` is forwarded by this server to the next one, upstream ``rpc_push``: the
  client pays one round trip per token instead of one per stage), task priorities (decode
  steps before prefills, upstream ``TaskPrioritizer``), KV allocation that waits for pages
  to be freed up to ``alloc_timeout`` (upstream ``MemoryCache``), ``rpc_close_session``,
  ``rpc_echo`` and ``rpc_check_reachability``.

Metadata keys: session_id, seq_len, cur_len, is_prefill, is_replay, max_length, temperature,
top_p, top_k, repetition_penalty (default 1.5), generated_tokens.  Final-stage replies carry
``token_id`` (and an int64 [[token]] tensor); others return hidden [1, T, H].
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import dataclasses
import logging
import threading
import time
from typing import Dict, List, Optional

import torch

from .comm.rpc import RemoteError, RpcClient, RpcServer
from .comm.wire import Message
from .runtime.kv_cache import AllocationFailed
from .runtime.sampler import BatchSampler, SamplingParams, session_seed
from .utils.tracing import PhaseTimer

logger = logging.getLogger(__name__)

HANDLER_PREFIX = "StageConnectionHandler."


class TaskPrioritizer:
    """Upstream Petals ``DummyTaskPrioritizer`` (petals/server/task_prioritizer.py:6-20):
    inference (one-token decode) steps first, everything else (prefill / forward) after.
    Lower value = served first; ties in arrival order."""

    def prioritize(self, n_tokens: int, is_prefill: bool, **kwargs) -> float:
        return 1.0 if (n_tokens == 1 and not is_prefill) else 2.0


@dataclasses.dataclass
class _Req:
    sid: str
    x: torch.Tensor          # [T, H] hidden (or [T] ids for a first stage)
    start: int               # first position of these tokens
    reset: bool
    params: SamplingParams
    generated: List[int]
    max_length: Optional[int]
    fut: asyncio.Future
    t0: float
    priority: float = 2.0
    prompts: Optional[torch.Tensor] = None  # deep prompts [n_blocks, P, H] for this step


class StageConnectionHandler:
    def __init__(self, dht, stage_model, device=None, request_timeout: float = 30.0, final_stage: bool = False,
                 batch_window_ms: float = 0.5, max_batch_tokens: Optional[int] = None, seed: int = 0,
                 alloc_timeout: float = 5.0, prioritizer: Optional[TaskPrioritizer] = None):
        self.dht = dht
        self.executor = stage_model
        self.device = torch.device(device) if device is not None else stage_model.device
        self.request_timeout = request_timeout
        self.final_stage = final_stage
        self.batch_window = batch_window_ms / 1000.0
        self.max_batch_tokens = max_batch_tokens or stage_model.max_tokens
        self.seed = seed
        self._default = SamplingParams(0.8, 0.9, 0, 1.5)  # reference handler defaults (:71-73, :164)
        self._pending: List[_Req] = []
        self._draining = False
        # sessions seen recently (sid -> last arrival): the collection window only waits while
        # some of them have not sent this step's request yet - a lone session (the reference
        # client's mode) never pays it
        self._recent: Dict[str, float] = {}
        self._worker = concurrent.futures.ThreadPoolExecutor(1, thread_name_prefix="stage-gpu")
        self._sampler = BatchSampler(self.device) if final_stage else None
        self.alloc_timeout = alloc_timeout
        self.prioritizer = prioritizer or TaskPrioritizer()
        self._client: Optional[RpcClient] = None  # for push forwarding (created on the server loop)
        self._steps: Dict[str, Dict[str, Message]] = {}  # session -> step_id -> reply (dedup, rpc_inference)
        # device-channel engines by channel name: a channel that failed stays here (its sessions
        # parked, its replay cache alive) until a replacement channel adopts it (stage-local recovery)
        self._chan_engines: Dict[str, object] = {}
        self._chan_lock = threading.Lock()
        self.stats = {"requests": 0, "batches": 0, "tokens": 0, "pushed": 0}
        self.timer = PhaseTimer()  # host wall time per phase (+ roctx ranges when MPAMD_TRACE=1)

    # ------------------------------------------------------------------ registration
    def add_p2p_handlers(self, server: RpcServer) -> None:
        server.add_handler(HANDLER_PREFIX + "rpc_forward", self.rpc_forward)
        server.add_handler(HANDLER_PREFIX + "rpc_forward_stream", self.rpc_forward_stream)
        server.add_handler(HANDLER_PREFIX + "rpc_info", self.rpc_info)
        server.add_handler(HANDLER_PREFIX + "rpc_close_session", self.rpc_close_session)
        server.add_handler(HANDLER_PREFIX + "rpc_echo", self.rpc_echo)
        server.add_handler(HANDLER_PREFIX + "rpc_inference", self.rpc_inference)
        server.add_handler(HANDLER_PREFIX + "rpc_push", self.rpc_push)
        server.add_handler(HANDLER_PREFIX + "rpc_check_reachability", self.rpc_check_reachability)
        server.add_handler(HANDLER_PREFIX + "rpc_backward", self.rpc_backward)
        server.add_handler(HANDLER_PREFIX + "rpc_backward_stream", self.rpc_backward_stream)
        server.add_handler(HANDLER_PREFIX + "rpc_channel_open", self.rpc_channel_open)

    # ------------------------------------------------------------------ handlers
    async def rpc_forward(self, msg: Message) -> Message:
        if msg.metadata.get("stateless"):
            return await self._stateless(msg, backward=False)
        return await self._handle(msg)

    async def rpc_forward_stream(self, msg: Message) -> Message:
        return await self.rpc_forward(msg)

    async def rpc_backward(self, msg: Message) -> Message:
        """Gradients w.r.t. the span's input hidden states and deep prompts (upstream
        ``rpc_backward``, petals/server/handler.py:434-459; ``run_rpc_backward``,
        block_functions.py:84-141). Tensors: ``[hidden [B,T,H], grad_output [B,T,H], prompts?]``,
        where ``prompts`` is ``[n_blocks, B|1, P, H]`` when ``metadata["has_prompts"]``. The reply is
        ``[grad_hidden]`` or ``[grad_hidden, grad_prompts]``. Stateless: no session and no KV cache."""
        return await self._stateless(msg, backward=True)

    async def rpc_backward_stream(self, msg: Message) -> Message:
        return await self.rpc_backward(msg)

    def _autograd_stage(self):
        if getattr(self, "_ag", None) is None:
            from .runtime.autograd_stage import AutogradStage

            ex = self.executor
            self._ag = AutogradStage(ex.cfg, ex.w, ex.device, ex.dtype)
        return self._ag

    async def _stateless(self, msg: Message, backward: bool) -> Message:
        """Upstream ``run_rpc_forward`` / ``run_rpc_backward``. These run on the GPU worker thread,
        so they serialise with inference batches, which are submitted first."""
        if self.executor.is_first:
            raise ValueError("stateless forward/backward takes hidden states; this span starts with the embedding")
        md, ts = msg.metadata, list(msg.tensors)
        has_prompts = bool(md.get("has_prompts", False))
        need = (2 if backward else 1) + int(has_prompts)
        if len(ts) != need:
            raise ValueError(f"expected {need} tensors, got {len(ts)}")
        hidden = ts[0] if ts[0].dim() == 3 else ts[0].unsqueeze(0)
        prompts = ts[-1] if has_prompts else None

        def run():
            ag = self._autograd_stage()
            if not backward:
                with torch.no_grad():
                    return [ag.forward(hidden, prompts).to("cpu")]
            g = ts[1] if ts[1].dim() == 3 else ts[1].unsqueeze(0)
            gh, gp = ag.backward(hidden, g, prompts)
            out = [gh.to("cpu", hidden.dtype)]
            if gp is not None:
                out.append(gp.to("cpu", prompts.dtype))
            return out

        self.stats["backward" if backward else "forward_stateless"] = \
            self.stats.get("backward" if backward else "forward_stateless", 0) + 1
        outs = await asyncio.wait_for(asyncio.get_running_loop().run_in_executor(self._worker, run),
                                      self.request_timeout * 4)
        return Message({"session_id": md.get("session_id")}, outs)

    async def rpc_channel_open(self, msg: Message) -> Message:
        """Join a same-node device channel (``parallel.channel``): the client found every hop
        of its route on its own machine and asks this server to take rank ``rank`` of a
        pipeline whose rank 0 is the client.  Hidden states then hop GPU -> GPU over RCCL
        (xGMI) and token ids come back on the channel; this TCP RPC only carries the
        rendezvous.  The serving loop runs on its own thread (``PipelineServingEngine.serve``)
        until the client's STOP or a peer failure; TCP requests keep being served meanwhile."""
        md = msg.metadata
        import threading

        from .parallel.channel import host_id

        if md.get("host_id") not in (None, host_id()):
            return Message({"ok": False, "error": "not on the same host"})
        rank, world = int(md["rank"]), int(md["world"])
        if (rank == world - 1) != bool(self.final_stage):
            return Message({"ok": False, "error": f"rank {rank}/{world} does not match final_stage={self.final_stage}"})
        t = threading.Thread(target=self._channel_serve, args=(dict(md),), daemon=True,
                             name=f"channel-{md.get('prefix')}")
        t.start()
        self.stats["channels"] = self.stats.get("channels", 0) + 1
        return Message({"ok": True, "start_block": self.executor.start, "end_block": self.executor.end})

    def _channel_serve(self, md: dict) -> None:
        from .parallel.channel import Channel, make_store
        from .parallel.engine import PipelineFailure, PipelineServingEngine

        ex = self.executor
        ch = eng = None
        name = str(md.get("prefix", "chan"))
        try:
            store = make_store(md["store_host"], int(md["store_port"]), int(md["world"]), False,
                               timeout_s=float(md.get("timeout", 60.0)))
            ch = Channel(store, name, int(md["rank"]), int(md["world"]), ex.device,
                         timeout_s=float(md.get("timeout", 60.0)), data_backend=md.get("data_backend"))
            resume = None
            old = md.get("resume_prefix")
            if old:
                with self._chan_lock:
                    prev = self._chan_engines.pop(str(old), None)
                if prev is not None:
                    # the replaced channel has failed even if its thread has not noticed yet (it may
                    # be blocked on a payload from the dead stage): abort it so that wait returns now
                    # and its serving loop ends, then free the executor's graph hook
                    if prev.ch is not None:
                        prev.ch.abort()
                    prev.release()
                resume = {"prefix": str(old), "cache": getattr(prev, "replay", None)}
                if prev is not None:
                    prev.replay = None  # the new engine owns it now and drops it once adopted
            eng = PipelineServingEngine(ex, ch, n_slots=int(md.get("n_slots", 1)), batch=int(md.get("batch", 64)),
                                        name=name, replay_cache=bool(md.get("replay_cache", False)), resume=resume)
            with self._chan_lock:
                self._chan_engines[name] = eng
            logger.info(f"device channel {name}: open as rank {int(md['rank'])} of {int(md['world'])}"
                        + (f", resuming {old}" if old else ""))
            eng.idle_timeout_s = float(md.get("idle_timeout", 3600.0))
            eng.timing = bool(md.get("timing", False))  # per-stage ms for the client's STATS gathers
            ch.timing = eng.timing
            with torch.inference_mode():
                eng.serve()
            logger.info(f"device channel {name}: stopped after {eng.steps_run} steps")
        except (PipelineFailure, RuntimeError) as e:
            logger.warning(f"device channel {name} failed: {e}")
        finally:
            if eng is not None:
                eng.release()  # no graph of this channel's hop survives it (TCP steps, probes, next channel)
                with self._chan_lock:
                    if eng.failed is None or not eng.park_on_fail:
                        self._chan_engines.pop(name, None)
                    if eng.failed is not None:
                        eng.failed_at = time.monotonic()
                    self._prune_failed_channels()
            with ex.exec_lock:  # (parked sessions - ``park:`` keys - wait for adoption or the session TTL)
                for sid in [k for k in ex.sessions.sessions if k.startswith(name + ":")]:
                    ex.sessions.close(sid)
            if ch is not None:
                ch.close()

    # failed, not-yet-adopted channels keep their replay cache (max_handles x max_len x hidden in HBM,
    # outside the KV capacity exchange) for the client's stage-local recovery: bounded by age and bytes
    replay_keep_s = 300.0
    replay_keep_bytes = 8 << 30

    def _prune_failed_channels(self, now: Optional[float] = None) -> None:
        """Drop the replay caches of failed channels nobody adopted: older than ``replay_keep_s``,
        then the oldest ones while the kept caches exceed ``replay_keep_bytes`` (several clients
        failing close together each keep theirs up to that budget).  Caller holds ``_chan_lock``."""
        now = time.monotonic() if now is None else now
        dead = sorted(((getattr(e, "failed_at", now), k) for k, e in self._chan_engines.items()
                       if getattr(e, "failed", None) is not None), reverse=True)  # newest first
        kept = 0
        for at, k in dead:
            e = self._chan_engines[k]
            rc = getattr(e, "replay", None)
            n = rc.buf.numel() * rc.buf.element_size() if rc is not None else 0
            if now - at > self.replay_keep_s or kept + n > self.replay_keep_bytes:
                self._chan_engines.pop(k).replay = None
            else:
                kept += n

    async def rpc_push(self, msg: Message) -> Message:
        """Server-to-server hop of a pushed chain (upstream ``rpc_push``); same body as rpc_forward."""
        return await self._handle(msg)

    async def rpc_inference(self, msg: Message) -> Message:
        """Upstream Petals per-step inference API (petals/server/handler.py ``rpc_inference``).

        Metadata: ``session_id``, ``step_id`` (a repeated step id returns the cached reply
        instead of running twice), optional ``start_from_position`` (rewind the session to
        that position before this step), optional ``fork_from`` (beam search: this session
        first becomes a copy of that one, the per-session form of upstream ``hypo_ids``),
        ``max_length``; otherwise as ``rpc_forward``.
        """
        md = dict(msg.metadata)
        sid, step_id = md.get("session_id"), md.get("step_id")
        src = md.pop("fork_from", None)
        # the dedup check comes first: a retried step that already ran (fork included) must
        # neither fork again (that would reset sid's KV to src's length) nor recompute
        if sid is not None and step_id is not None:
            cached = self._steps.get(sid, {}).get(str(step_id))
            if cached is not None:
                return cached
        if src is not None and sid is not None:  # beam search: continue from another hypothesis
            await asyncio.get_running_loop().run_in_executor(self._worker, self.executor.sessions.fork, str(src),
                                                             str(sid))
        x = msg.tensors[0] if msg.tensors else None
        if x is not None and "cur_len" not in md:
            T = x.shape[-2] if x.dim() >= 2 and not self.executor.is_first else x.reshape(-1).shape[0]
            sess = self.executor.sessions.get(sid) if sid is not None else None
            start = md.get("start_from_position")
            base = int(start) if start is not None else (sess.length if sess is not None else 0)
            md["cur_len"] = base + int(T)
            md.setdefault("is_prefill", sess is None or base == 0)
        reply = await self._handle(Message(md, list(msg.tensors)))
        if sid is not None and step_id is not None:
            steps = self._steps.setdefault(sid, {})
            steps[str(step_id)] = reply
            while len(steps) > 64:
                steps.pop(next(iter(steps)))
        return reply

    async def rpc_check_reachability(self, msg: Message) -> Message:
        """Probe whether ``target`` (a multiaddr) is reachable from THIS server (upstream
        petals/server/reachability.py: peers check each other's direct reachability)."""
        target = msg.metadata.get("target")
        if not target:
            return Message({"ok": False, "error": "no target"})
        t0 = time.perf_counter()
        try:
            if self._client is None:
                self._client = RpcClient()
            await self._client.call(target, HANDLER_PREFIX + "rpc_echo", Message({"ping": True}),
                                    timeout=float(msg.metadata.get("timeout", 5.0)))
            return Message({"ok": True, "rtt_s": time.perf_counter() - t0})
        except Exception as e:  # noqa: BLE001 - any failure means "not reachable"
            return Message({"ok": False, "error": f"{type(e).__name__}: {e}"})

    async def _handle(self, msg: Message) -> Message:
        reply = await asyncio.wait_for(self._submit(msg), self.request_timeout)
        hops = msg.metadata.get("next_hops")
        if not hops or self.final_stage or msg.metadata.get("has_prompts"):  # upstream: no push with prompts
            return reply
        return await self._push(msg.metadata, reply, list(hops))

    async def _push(self, md: dict, reply: Message, hops: List[dict]) -> Message:
        """Forward this stage's output to the next server of the chain and return the
        downstream reply with this hop's output prepended (the client keeps every hop's
        input for failover replay).  A downstream failure returns this hop's output with
        ``push_failed_at`` = index (relative to this server) of the hop that failed."""
        out = reply.tensors[0]
        nxt, rest = hops[0], hops[1:]
        fwd = {k: v for k, v in md.items() if k != "next_hops"}
        if rest:
            fwd["next_hops"] = rest
        if self._client is None:
            self._client = RpcClient()
        self.stats["pushed"] += 1
        err = None
        for addr in nxt.get("maddrs") or []:
            try:
                down = await self._client.call(addr, HANDLER_PREFIX + "rpc_push", Message(fwd, [out]),
                                               timeout=self.request_timeout * (1 + len(rest)))
                dmd = dict(down.metadata)
                if "push_failed_at" in dmd:
                    dmd["push_failed_at"] = int(dmd["push_failed_at"]) + 1
                    return Message(dmd, [out] + list(down.tensors))
                # final reply: [token, hiddens...] -> [token, out, hiddens...]
                if "token_id" in dmd:
                    return Message(dmd, [down.tensors[0], out] + list(down.tensors[1:]))
                return Message(dmd, [out] + list(down.tensors))
            except (ConnectionError, OSError, asyncio.TimeoutError, RemoteError) as e:
                err = e
                self._client.drop(addr)
        return Message({"session_id": md.get("session_id"), "push_failed_at": 1,
                        "push_error": f"{type(err).__name__}: {err}" if err else "no address"}, [out])

    async def rpc_info(self, msg: Message) -> Message:
        ex = self.executor
        return Message({"cache_tokens_left": ex.sessions.cache_tokens_left(), "sessions": len(ex.sessions.sessions),
                        "start_block": ex.start, "end_block": ex.end, "final_stage": self.final_stage,
                        "phases": self.timer.summary(), **self.stats})

    async def rpc_close_session(self, msg: Message) -> Message:
        sid = msg.metadata.get("session_id")
        if sid is not None:
            self._steps.pop(sid, None)
            await asyncio.get_running_loop().run_in_executor(self._worker, self.executor.sessions.close, sid)
        return Message({"ok": True})

    async def rpc_echo(self, msg: Message) -> Message:
        return Message(dict(msg.metadata), list(msg.tensors))

    # ------------------------------------------------------------------ request parsing
    def _parse(self, msg: Message) -> _Req:
        md = msg.metadata
        sid = md.get("session_id")
        if sid is None:
            raise ValueError("request.metadata must contain session_id")
        if not msg.tensors:
            raise ValueError("request carries no tensor")
        x = msg.tensors[0]
        if x.dim() == 3:
            x = x.reshape(-1, x.shape[-1])
        elif x.dim() == 2 and self.executor.is_first and x.dtype in (torch.int64, torch.int32):
            x = x.reshape(-1)
        T = x.shape[0]
        is_prefill = bool(md.get("is_prefill", False))
        is_replay = bool(md.get("is_replay", False))
        cur_len = int(md.get("cur_len", T))
        sess = self.executor.sessions.get(sid)
        if is_prefill:
            start, reset = 0, True
        elif sess is None:
            if not is_replay:
                raise ValueError(f"Missing past_key_values for session_id={sid}. This may indicate a server "
                                 f"restart or cache loss. If this is a replay scenario, ensure is_replay=True.")
            start, reset = 0, True  # first replayed request on a fresh server
        else:
            want = cur_len - T
            if 0 <= want <= sess.length:
                start = want  # idempotent: a retried / replayed step overwrites its own slot
            else:
                logger.warning(f"[{sid[:8]}] past len mismatch: cache={sess.length} cur_len={cur_len} T={T}")
                start = sess.length
            reset = False
        params = SamplingParams(float(md.get("temperature", self._default.temperature)),
                                float(md.get("top_p", self._default.top_p)), int(md.get("top_k", self._default.top_k)),
                                float(md.get("repetition_penalty", self._default.repetition_penalty)))
        prompts = None
        if md.get("has_prompts") and len(msg.tensors) > 1:
            # upstream layout [n_blocks, B(=1), P, H]; one session per request here
            prompts = msg.tensors[1]
            if prompts.dim() == 4:
                prompts = prompts[:, 0]
        return _Req(sid, x, start, reset, params, list(md.get("generated_tokens", []) or []),
                    md.get("max_length"), None, time.perf_counter(), prompts=prompts)

    async def _submit(self, msg: Message) -> Message:
        req = self._parse(msg)
        req.priority = self.prioritizer.prioritize(int(req.x.shape[0]), bool(req.reset))
        req.fut = asyncio.get_running_loop().create_future()
        self._recent[req.sid] = req.t0
        self._pending.append(req)
        self.stats["requests"] += 1
        if not self._draining:
            self._draining = True
            asyncio.ensure_future(self._drain())
        return await req.fut

    # ------------------------------------------------------------------ continuous batching
    async def _drain(self):
        loop = asyncio.get_running_loop()
        try:
            while self._pending:
                if self.batch_window > 0 and self._expect_more():
                    await asyncio.sleep(self.batch_window)
                batch, rest, seen, ntok = [], [], set(), 0
                # priority order (decode steps first), arrival order within a priority
                self._pending.sort(key=lambda r: (r.priority, r.t0))
                for r in self._pending:
                    n = r.x.shape[0]
                    if r.sid in seen or (batch and ntok + n > self.max_batch_tokens):
                        rest.append(r)
                        continue
                    batch.append(r)
                    seen.add(r.sid)
                    ntok += n
                self._pending = rest
                try:
                    outs = await self._run_with_alloc_wait(loop, batch)
                except Exception as e:  # one bad request must not take the batch down: retry singly
                    if len(batch) == 1:
                        if not batch[0].fut.done():
                            batch[0].fut.set_exception(e)
                        continue
                    outs = []
                    for r in batch:
                        try:
                            outs.append((await loop.run_in_executor(self._worker, self._run_batch, [r]))[0])
                        except Exception as e1:
                            outs.append(e1)
                for r, o in zip(batch, outs):
                    if r.fut.done():
                        continue
                    if isinstance(o, Exception):
                        r.fut.set_exception(o)
                    else:
                        r.fut.set_result(o)
        finally:
            self._draining = False

    def _expect_more(self, horizon_s: float = 1.0) -> bool:
        """Are sessions active within ``horizon_s`` missing from the pending queue?  Only then can
        the collection window merge more requests into this step."""
        now = time.perf_counter()
        if len(self._recent) > 4 * len(self._pending) + 64:  # prune sessions gone quiet
            self._recent = {k: t for k, t in self._recent.items() if now - t < horizon_s}
        pending = {r.sid for r in self._pending}
        return any(now - t < horizon_s and sid not in pending for sid, t in self._recent.items())

    async def _run_with_alloc_wait(self, loop, batch: List[_Req]):
        """Run a batch; when the KV cache is full, evict expired sessions and wait (up to
        ``alloc_timeout``) for pages to be freed - upstream MemoryCache semantics
        (petals/server/memory_cache.py: allocation waits, then ``AllocationFailed``)."""
        deadline = time.perf_counter() + self.alloc_timeout
        while True:
            try:
                return await loop.run_in_executor(self._worker, self._run_batch, batch)
            except AllocationFailed:
                await loop.run_in_executor(self._worker, self.executor.sessions.evict_expired)
                if time.perf_counter() >= deadline:
                    raise
                await asyncio.sleep(0.05)

    def _run_batch(self, batch: List[_Req]) -> List[Message]:
        ex = self.executor
        seqs = [(r.sid, r.x.shape[0]) for r in batch]
        if ex.is_first:
            x = torch.cat([r.x.reshape(-1).to(torch.long) for r in batch]).to(ex.device)
        else:
            x = torch.cat([r.x for r in batch]).to(ex.device, ex.dtype)
        ml = max((int(r.max_length) for r in batch if r.max_length), default=None)
        phase = "handler.prefill" if any(r.x.shape[0] > 1 for r in batch) else "handler.decode"
        prompts = [r.prompts for r in batch] if any(r.prompts is not None for r in batch) else None
        with torch.inference_mode(), self.timer(phase), ex.exec_lock:
            out = ex.forward(seqs, x, reset=[r.reset for r in batch], starts=[r.start for r in batch], max_length=ml,
                             prompts=prompts)
            self.stats["batches"] += 1
            self.stats["tokens"] += int(x.shape[0])
            if self.final_stage:
                seeds = [session_seed(r.sid, r.start + r.x.shape[0], self.seed) for r in batch]
                toks = self._sampler(out, [r.params for r in batch], [r.generated for r in batch], seeds).tolist()
                return [Message({"token_id": int(t), "session_id": r.sid}, [torch.tensor([[int(t)]], dtype=torch.long)])
                        for r, t in zip(batch, toks)]
            if out.is_cuda and out.numel():
                # the |x| check of the reference's warning runs on the device, and the hidden
                # states leave through pinned memory (torch's caching host allocator): one
                # stream sync for both instead of a pageable copy plus a host-side reduction
                amax_dev = out.abs().amax(-1).float()
                out_cpu = torch.empty(out.shape, dtype=out.dtype, pin_memory=True)
                amaxes = torch.empty(amax_dev.shape, dtype=torch.float32, pin_memory=True)
                out_cpu.copy_(out, non_blocking=True)
                amaxes.copy_(amax_dev, non_blocking=True)
                torch.cuda.current_stream(out.device).synchronize()
            else:
                out_cpu = out.to("cpu", non_blocking=False)
                amaxes = out_cpu.float().abs().amax(-1) if out_cpu.numel() else out_cpu
        res, off = [], 0
        for r in batch:
            n = r.x.shape[0]
            h = out_cpu[off:off + n]
            amax = float(amaxes[off:off + n].max()) if n else 0.0
            off += n
            if amax > 100:
                logger.warning(f"[{r.sid[:8]}] large activation values detected (|x|max={amax:.2f})")
            res.append(Message({"session_id": r.sid}, [h.unsqueeze(0)]))
        return res

    def shutdown(self):
        self._worker.shutdown(wait=False)
