"""Continuous-batching pipeline serving engine over a device ``Channel``.

Reference dataflow: the Stage-0 client embeds, runs its blocks, then drives ONE session
token by token through the remote stages (star topology, one hop at a time, a
``generated_tokens`` list and the sampling parameters in every request's metadata; the
last stage samples and replies with the token id), stopping on EOS, ``max_new_tokens`` or
5 consecutive repeats (reference src/main.py:62-227, src/rpc_transport.py:718-842,
src/rpc_handler.py:149-325).

Here the same roles run as a chain of stage ranks, one process per GPU:

    head (rank 0: embedding + blocks [0, s0) + SCHEDULER)
      -> stage 1 -> ... -> tail (blocks + norm + lm_head + SAMPLER)
      -> token ids back to the head

* The head owns the request queue.  Sessions are admitted into one of ``M`` micro-batch
  slots (at most ``batch`` sessions each) whenever there is room, prefill and decode rows
  mix in one ragged step (chunked prefill caps the prompt tokens per step), and finished
  sessions are retired in the very next step of their slot: continuous batching.
* Every step is announced by a header on the host control group (sessions, token counts,
  positions, closes, admissions with sampling parameters and repetition history) that a
  stage forwards to its successor before computing; the payload (hidden states) follows on
  RCCL.  Stage k therefore never waits on a host round trip of stage k-1's compute.
* The tail samples with per-session parameters and a device-resident repetition history
  (reference semantics, ``ops.sample``), seeded by (session seed, position): the random draw
  of a session never depends on which micro-batch, replica or batch mix it runs in.  The
  LOGITS do, in their last bits, on the GPU: the decode GEMM form (and so its reduction order)
  is chosen per row bucket, and a failed-over session's KV is rebuilt by a prefill (hipBLASLt
  + FA2) where the original came from decode steps.  Exactness contract: on the CPU path
  (fp32 reference ops) a re-placed session's logits agree to fp32 rounding and its tokens equal
  the uninterrupted run's (``tests/test_channel_failover.py``, ``tests/test_failover_drill.py``);
  on the GPU the tokens generated before a failure are identical and, after re-placement, the
  teacher-forced logits agree within bf16 tolerance (``tests/test_failover_gpu.py``), so a
  sampled token can differ only where two candidates are within that tolerance of each other.
* Stop conditions are checked on the head from a pinned copy of each step's tokens one
  round later, so the decode loop never blocks the host on the device: the next step's
  inputs are gathered on the device from the previous step's sampled tokens.  A finished
  session costs one discarded extra decode row.
* ``M >= stages + 1`` slots keep every stage busy and leave a slot of slack for the token
  return hop; every rank runs the same number of rounds x slots, so ``run_rounds(k)`` is a
  lock-step unit (the benchmark times exactly k of them) and a serving stage simply loops
  until the head's STOP header.
* Failures: every host receive has a timeout and a dead peer surfaces as a connection
  error; the head additionally polls its token events with a deadline (an RCCL receive from
  a dead rank never completes).  The channel is aborted and the failure reported with the
  affected requests' token histories (``PipelineFailure``), which the replica router
  (``parallel.router``) re-places on surviving replicas by re-prefilling prompt + generated
  tokens (recompute-from-tokens).
"""
from __future__ import annotations

import collections
import dataclasses
import gc
import logging
import os
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from ..runtime.executor import StageExecutor
from ..runtime.sampler import RECENT, SamplingParams
from ..utils.tracing import trace_range
from .channel import Channel, ChannelError, wait_event

logger = logging.getLogger(__name__)

KIND_STEP, KIND_STOP, KIND_STATS, KIND_REPLAY = 0, 1, 2, 3
REPLAY_REC = 3   # new handle, replayed length L, handle in the failed channel
F_RESET, F_SAMPLE = 1, 2
HDR = 8          # kind, slot, n_seq, T, n_close, n_admit, round, reserved
SEQ_REC = 5      # handle, n_tok, start, flags, seed
ADM_REC = 6 + RECENT  # handle, temp, top_p, top_k, rep_pen, hist_len, hist[RECENT]
_M64 = (1 << 64) - 1


class PipelineFailure(RuntimeError):
    """The pipeline lost a stage; ``requests`` are the unfinished ones (with the tokens
    generated so far) to be re-placed elsewhere."""

    def __init__(self, msg: str, requests: Sequence["Request"] = ()):
        super().__init__(msg)
        self.requests = list(requests)


@dataclasses.dataclass
class Request:
    prompt: List[int]
    max_new_tokens: int = 64
    params: SamplingParams = dataclasses.field(default_factory=lambda: SamplingParams(1.0, 0.92, 50, 1.5))
    eos_token_id: Optional[int] = None
    stop_on_repeat: int = 5  # reference run_rank0: stop after 5 consecutive repeats (0 = off)
    seed: int = 0
    rid: Optional[str] = None
    generated: List[int] = dataclasses.field(default_factory=list)
    done: bool = False
    finish_reason: Optional[str] = None
    t_submit: float = 0.0
    t_first: Optional[float] = None
    t_done: Optional[float] = None
    _repeat: int = 0

    @property
    def tokens(self) -> List[int]:
        return list(self.prompt) + list(self.generated)


def _f2i(x: float) -> int:
    return int(np.float64(x).view(np.int64))


def _i2f(x) -> float:
    return float(np.int64(x).view(np.float64))


def mix_seeds(base: np.ndarray, pos: np.ndarray) -> np.ndarray:
    """splitmix64(base ^ pos * golden): per (session seed, position) sampling seeds."""
    with np.errstate(over="ignore"):
        z = (base.astype(np.uint64) ^ (pos.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)))
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(0x7FFFFFFFFFFFFFFF)).astype(np.int64)


def repeat_run(generated: Sequence[int]) -> int:
    """The client's consecutive-repeat counter after ``generated`` (reference src/main.py:160,
    197-205: ``last_token`` starts as None, so the first token - the prefill's - is never
    compared; every later token equal to its predecessor extends the run, any other resets it)."""
    n = 0
    for i in range(len(generated) - 1, 1, -1):
        if generated[i] != generated[i - 1]:
            break
        n += 1
    return n


_HEAP_FROZEN = False


def settle_heap() -> bool:
    """Once per PROCESS, before a driver's first serving step: collect, then freeze every object
    alive now (model, buffers, graphs, channels) into the interpreter's permanent generation.  The
    serving loop allocates small objects every step; without this each full collection it triggers
    (every few dozen steps) walks the whole setup heap and stalls the step loop for milliseconds.
    Only drivers call it (engines with ``freeze_heap``): frozen objects are never collected, so a
    server that builds an engine per client channel must not freeze each one's transient state.
    Returns True if this call froze the heap."""
    global _HEAP_FROZEN
    if _HEAP_FROZEN:
        return False
    _HEAP_FROZEN = True
    gc.collect()
    gc.freeze()
    return True


def request_seed(seed: int, rid: str) -> int:
    import hashlib

    h = hashlib.blake2b(f"{seed}:{rid}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") & 0x7FFFFFFFFFFFFFFF


# ====================================================================== tail sampler
class TailSampler:
    """Per-session sampling state resident on the tail's device: parameters set at
    admission, the last RECENT generated ids (repetition penalty, reference
    src/rpc_handler.py:348-372) updated in place by the sampling kernel."""

    def __init__(self, device, max_handles: int, vocab: int):
        dev = self.device = torch.device(device)
        H = max_handles
        self.temp = torch.zeros(H, dtype=torch.float32, device=dev)
        self.top_p = torch.ones(H, dtype=torch.float32, device=dev)
        self.top_k = torch.zeros(H, dtype=torch.int32, device=dev)
        self.rp = torch.ones(H, dtype=torch.float32, device=dev)
        self.hist = torch.zeros(H, RECENT, dtype=torch.int32, device=dev)
        self.hist_len = torch.zeros(H, dtype=torch.int32, device=dev)
        self.temp_host = np.zeros(H, dtype=np.float64)
        self.seed_host = np.zeros(H, dtype=np.int64)
        self._ws = None
        self.vocab = vocab
        pin = dev.type == "cuda"
        self._pin_i64 = [torch.empty(4 * 256, dtype=torch.int64, pin_memory=pin) for _ in range(2)]
        self._pin_ev = [None, None]
        self._pk = 0
        # working set of the last sampled batch: in steady decode the same handles come back
        # in the same order every step, so their parameters / history stay gathered
        self._cur_key: Optional[bytes] = None
        self._cur: Optional[dict] = None

    def warm(self, rows: int) -> None:
        """First-call costs of the serving path's sampler bookkeeping (admission scatter, history
        gather / write-back, the staged seed copy, the sampling kernel at ``rows`` rows) paid at
        start-up on scratch records for handles 0..rows-1, which every real admission overwrites."""
        n = min(int(rows), self.temp.shape[0])
        if n <= 0 or self.device.type != "cuda":
            return
        recs = np.zeros((n, ADM_REC), dtype=np.int64)
        recs[:, 0] = np.arange(n)
        recs[:, 1], recs[:, 2], recs[:, 3], recs[:, 4] = _f2i(1.0), _f2i(0.92), 50, _f2i(1.5)
        self.admit(recs)
        logits = torch.zeros(n, self.vocab, dtype=torch.bfloat16, device=self.device)
        self.sample(logits, np.arange(n, dtype=np.int64), np.zeros(n, dtype=np.int64))
        self._writeback()
        self.hist_len.zero_()
        self.hist.zero_()
        torch.cuda.synchronize(self.device)

    def _writeback(self) -> None:
        if self._cur is not None:
            c = self._cur
            self.hist.index_copy_(0, c["rows"], c["recent"])
            self.hist_len.index_copy_(0, c["rows"], c["rlen"])
        self._cur, self._cur_key = None, None

    def admit(self, recs: np.ndarray) -> None:
        """recs: [n, ADM_REC] admission records."""
        if not len(recs):
            return
        self._writeback()
        h = recs[:, 0].astype(np.int64)
        f = np.stack([recs[:, 1], recs[:, 2], recs[:, 4]]).astype(np.int64).view(np.float64)
        self.temp_host[h] = f[0]
        hl = np.minimum(recs[:, 5], RECENT).astype(np.int32)
        hist = recs[:, 6:6 + RECENT].astype(np.int32)
        idx = torch.from_numpy(h).to(self.device)
        self.temp[idx] = torch.from_numpy(f[0].astype(np.float32)).to(self.device)
        self.top_p[idx] = torch.from_numpy(f[1].astype(np.float32)).to(self.device)
        self.rp[idx] = torch.from_numpy(f[2].astype(np.float32)).to(self.device)
        self.top_k[idx] = torch.from_numpy(recs[:, 3].astype(np.int32)).to(self.device)
        self.hist[idx] = torch.from_numpy(hist).to(self.device)
        self.hist_len[idx] = torch.from_numpy(hl).to(self.device)

    def _stage(self, arrs: Sequence[np.ndarray]) -> List[torch.Tensor]:
        """Async H2D of small int64 vectors through a double-buffered pinned area."""
        n = sum(len(a) for a in arrs)
        if self.device.type != "cuda" or n > self._pin_i64[0].numel():
            return [torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).to(self.device) for a in arrs]
        self._pk ^= 1
        ev = self._pin_ev[self._pk]
        if ev is not None:
            ev.synchronize()
        buf = self._pin_i64[self._pk]
        host = buf.numpy()
        off, outs = 0, []
        for a in arrs:
            host[off:off + len(a)] = a
            outs.append((off, len(a)))
            off += len(a)
        dev = buf[:n].to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pin_ev[self._pk] = ev
        return [dev[o:o + k] for o, k in outs]

    def sample(self, logits: torch.Tensor, handles: np.ndarray, positions: np.ndarray,
               sample_rows: Optional[np.ndarray] = None) -> torch.Tensor:
        """Tokens [n] (int64, device) for the rows of ``logits``; rows not in ``sample_rows``
        get -1 and leave the history untouched (intermediate prefill chunks)."""
        n = logits.shape[0]
        if sample_rows is not None and len(sample_rows) < n:
            out = torch.full((n,), -1, dtype=torch.long, device=logits.device)
            if len(sample_rows):
                sel = torch.from_numpy(sample_rows.astype(np.int64)).to(logits.device)
                sub = self.sample(logits.index_select(0, sel), handles[sample_rows], positions[sample_rows])
                out.index_copy_(0, sel, sub)
            return out
        if n == 0:
            return torch.empty(0, dtype=torch.long, device=logits.device)
        if (self.temp_host[handles] <= 0).all():
            return ops.argmax(logits)  # greedy: no penalty, no history (reference temp <= 0 branch)
        handles = np.ascontiguousarray(handles, dtype=np.int64)
        seeds_h = mix_seeds(self.seed_host[handles], positions)
        key = handles.tobytes()
        if key != self._cur_key:
            self._writeback()
            rows, seeds = self._stage([handles, seeds_h])
            self._cur = dict(rows=rows, recent=self.hist.index_select(0, rows),
                             rlen=self.hist_len.index_select(0, rows), temp=self.temp.index_select(0, rows),
                             top_p=self.top_p.index_select(0, rows), top_k=self.top_k.index_select(0, rows),
                             rp=self.rp.index_select(0, rows))
            self._cur_key = key
        else:
            (seeds,) = self._stage([seeds_h])
        c = self._cur
        ws = None
        if logits.device.type == "cuda":
            if self._ws is None or self._ws.numel() < n * logits.shape[1]:
                self._ws = torch.empty(max(n, 64) * logits.shape[1], dtype=torch.float32, device=logits.device)
            ws = self._ws
        return ops.sample(logits, c["temp"], c["top_p"], c["top_k"], c["rp"], c["recent"], c["rlen"], seeds,
                          workspace=ws, update_history=True)


# ====================================================================== stage-local recovery
class ReplayCache:
    """A non-tail stage's OUTPUT hidden states per session and position, in HBM - the reference
    client's per-hop input cache (src/rpc_transport.py:741,805; replayed to a replacement server
    by ``_replay_past_inputs`` :670-712) kept where the data already is.  When the next stage dies
    and a spare takes over its blocks, this stage replays the cached rows of every unfinished
    session to the spare, which rebuilds its KV with one prefill; every other surviving stage keeps
    its KV (adopted into the new channel) and does no work.  One ``index_copy_`` per step."""

    def __init__(self, max_handles: int, max_len: int, hidden: int, dtype, device):
        self.max_len = int(max_len)
        self.buf = torch.zeros(int(max_handles) * self.max_len, hidden, dtype=dtype, device=device)
        pin = self.buf.is_cuda
        self._pin = [torch.empty(1 << 14, dtype=torch.int64, pin_memory=pin) for _ in range(2)]
        self._pin_ev: List[Optional[object]] = [None, None]
        self._k = 0

    def _to_device(self, a: np.ndarray) -> torch.Tensor:
        """Row indices to the device without a host block (double-buffered pinned staging)."""
        if not self.buf.is_cuda or len(a) > self._pin[0].numel():
            return torch.from_numpy(a).to(self.buf.device)
        self._k ^= 1
        if self._pin_ev[self._k] is not None:
            self._pin_ev[self._k].synchronize()
        host = self._pin[self._k]
        host.numpy()[: len(a)] = a
        dev = host[: len(a)].to(self.buf.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pin_ev[self._k] = ev
        return dev

    def store(self, recs, out: torch.Tensor) -> None:
        """``recs``: the step's (handle, n_tokens, start, ...) records, ``out`` its [T, H] rows."""
        idx, keep, off = [], [], 0
        for r in recs:
            h, n, st = int(r[0]), int(r[1]), int(r[2])
            pos = np.arange(st, st + n)
            ok = pos < self.max_len
            idx.append(h * self.max_len + pos[ok])
            keep.append(off + np.nonzero(ok)[0])
            off += n
        if not idx:
            return
        idx, keep = np.concatenate(idx).astype(np.int64), np.concatenate(keep).astype(np.int64)
        src = out[: len(keep)] if np.array_equal(keep, np.arange(len(keep))) else \
            out.index_select(0, self._to_device(keep))
        self.buf.index_copy_(0, self._to_device(idx), src)

    def rows(self, handle: int, n: int) -> torch.Tensor:
        return self.buf[int(handle) * self.max_len: int(handle) * self.max_len + int(n)]


# ====================================================================== head-side state
@dataclasses.dataclass
class _Live:
    req: Request
    handle: int
    slot: int
    fed: int = 0                      # tokens fed into the KV cache (issued steps)
    pending: List[int] = dataclasses.field(default_factory=list)  # prompt tokens not yet fed
    admitted: bool = False            # admission record sent
    retired: bool = False
    last_row: int = -1                # its row in the slot's previous step (decode feed)


@dataclasses.dataclass
class _Step:
    slot: int
    rows: List[Tuple[_Live, int, bool]]  # (session, n_tokens, samples)
    tok_dev: Optional[torch.Tensor] = None
    waiter: Optional[Callable] = None
    tok_host: Optional[torch.Tensor] = None
    event: Optional[object] = None
    consumed: bool = False
    booked: bool = False
    t_issue: float = 0.0


class PipelineServingEngine:
    """One stage rank of a serving pipeline.  Rank 0 (the head) also schedules."""

    def __init__(self, executor: StageExecutor, channel: Optional[Channel], *, n_slots: Optional[int] = None,
                 batch: int = 64, max_step_tokens: Optional[int] = None, prefill_chunk: Optional[int] = None,
                 timeout_s: float = 120.0, max_handles: Optional[int] = None, timing: bool = False,
                 name: str = "pipe", warmup: Optional[bool] = None, replay_cache: bool = False,
                 resume: Optional[dict] = None):
        self.ex = executor
        self.ch = channel
        self.rank = channel.rank if channel is not None else 0
        self.S = channel.world if channel is not None else 1
        self.is_head = self.rank == 0
        self.is_tail = self.rank == self.S - 1
        self.dev = executor.device
        self.H = executor.cfg.hidden_size
        self.M = int(n_slots or (self.S + 1 if self.S > 1 else 1))
        self.B = int(batch)
        self.timeout_s = float(timeout_s)
        self.max_step_tokens = int(max_step_tokens or executor.max_tokens)
        self.prefill_chunk = int(prefill_chunk or self.max_step_tokens)
        self.name = name
        self.max_handles = int(max_handles or executor.sessions.max_sessions)
        self.timing = timing
        self._events = collections.deque(maxlen=8192)  # (start, end) HIP events of timed steps
        self.stopped = False
        self.failed: Optional[str] = None
        self.rounds = 0
        self.steps_run = 0
        # decode-step hops received straight into the static input of the graph the step replays
        # (``StageExecutor.graph_input``; every channel backend honours it) vs a receive slab + copy:
        # ``MPAMD_RECV_INTO=0`` (or ``recv_into = False``) keeps the copy path.  Counted per engine.
        self.recv_into = os.environ.get("MPAMD_RECV_INTO", "1") != "0"
        self.recvs = self.recvs_into = 0
        if self.is_tail:
            self.sampler = TailSampler(self.dev, self.max_handles, executor.cfg.vocab_size)
        if self.is_head:
            self.queue: List[Request] = []
            self.slots: List[List[_Live]] = [[] for _ in range(self.M)]
            self.inflight: List[Optional[_Step]] = [None] * self.M
            self.booking: List[Optional[_Step]] = [None] * self.M
            self.closes: List[List[int]] = [[] for _ in range(self.M)]
            self.free_handles = list(range(self.max_handles - 1, -1, -1))
            self.live: Dict[str, _Live] = {}
            self.finished: List[Request] = []
            self.on_token: Optional[Callable[[Request, int], None]] = None
            self.on_finish: Optional[Callable[[Request], None]] = None
            self._rid = 0
            self._pin = [torch.empty(max(self.B, 1) * 4, dtype=torch.int64, pin_memory=self.dev.type == "cuda")
                         for _ in range(2 * self.M + 2)]
            self._pin_k = 0
            self.capacity_tokens: Optional[int] = None
            self.reserved_tokens = 0
            self.tokens_generated = 0
        self._exchange_capacity()
        # stage-local recovery (opt-in): park KV on failure, keep a replay cache of the outputs
        self.park_on_fail = bool(replay_cache)
        self.replay = (ReplayCache(self.max_handles, self.max_len, self.H, executor.dtype, self.dev)
                       if replay_cache and not self.is_tail else None)
        self.resume = dict(resume or {})  # {"prefix": failed channel's engine name, "cache": its ReplayCache}
        self.failed_sessions: Dict[str, Tuple[int, Request]] = {}  # head: rid -> (handle, request) at failure
        if warmup is None:
            warmup = self.dev.type == "cuda" and os.environ.get("MPAMD_WARMUP", "1") != "0"
        if warmup:
            # the first steps' real shapes (a batch-wide ragged prefill, the decode graph of the
            # batch bucket, the sampler at batch rows): the first request pays no first-call costs
            self.ex.warmup_serving(self.B, max(1, min(self.max_step_tokens // max(self.B, 1), 512)))
            if self.is_tail:
                self.sampler.warm(self.B)

    # ------------------------------------------------------------------ setup
    def _exchange_capacity(self) -> None:
        """All-gather (free KV tokens, max sessions, page size) over the channel: the head
        admits only what EVERY stage can hold (stages with more blocks hold fewer tokens)."""
        ex = self.ex
        want_hop = (self.ch is not None and getattr(self.ch, "data_backend", "") == "rccl" and
                    os.environ.get("MPAMD_GRAPH_HOP", "0") == "1" and ex.graph_hook_free(self))
        mine = [float(ex.sessions.cache_tokens_left()), float(ex.sessions.max_sessions), float(ex.cache.page_size),
                float(ex.max_seq_len), float(want_hop), float(bool(ex.use_graphs)), float(ex.graph_max_batch)]
        allv = self.ch.all_gather_floats(mine) if self.ch is not None else [mine]
        self.stage_capacity = allv
        cap = int(min(v[0] for v in allv))
        self.max_handles = min(self.max_handles, int(min(v[1] for v in allv)))
        self.page = int(max(v[2] for v in allv))
        self.max_len = int(min(v[3] for v in allv))
        # graph hop (opt-in, MPAMD_GRAPH_HOP=1 on the direct-RCCL data plane): every stage's
        # decode graph ends with its hidden-state send, recorded into the graph on the compute
        # stream; a receiver must then know the row count of every hop from the header alone,
        # so all stages need identical graph settings (else no stage uses it)
        self.graph_hop = (self.S > 1 and all(v[4] == 1.0 for v in allv) and all(v[5] == 1.0 for v in allv) and
                          len({v[6] for v in allv}) == 1)
        if self.graph_hop and not self.is_tail:
            nxt = self.rank + 1
            ex.set_graph_hook(lambda out: self.ch.send_on_stream(nxt, out), owner=self)
        if self.is_head:
            self.capacity_tokens = cap
            self.free_handles = list(range(self.max_handles - 1, -1, -1))

    # ------------------------------------------------------------------ head API
    def submit(self, req: Request) -> Request:
        if not self.is_head:
            raise RuntimeError("submit() is a head (rank 0) operation")
        if req.rid is None:
            req.rid = f"{self.name}-{self._rid}"
            self._rid += 1
        if not req.prompt:
            raise ValueError("empty prompt")
        need = self._need(req)
        if need > self.max_len:
            raise ValueError(f"request needs {need} tokens > max_seq_len {self.max_len}")
        req._repeat = repeat_run(req.generated)  # a re-placed session resumes its stop counter
        req.t_submit = req.t_submit or time.perf_counter()
        self.queue.append(req)
        return req

    @property
    def idle(self) -> bool:
        return self.is_head and not self.queue and not self.live

    def _key(self, h: int) -> str:
        return f"{self.name}:{h}"

    @staticmethod
    def _need(req: Request) -> int:
        """KV tokens a request can ever hold: ``max_new_tokens`` is the TOTAL generation budget,
        so tokens a failed-over session already generated are part of it, not extra."""
        return len(req.prompt) + max(req.max_new_tokens, len(req.generated)) + 2

    def _reserve(self, req: Request) -> int:
        n = self._need(req)
        return self.page * ((n + self.page - 1) // self.page)

    def _admit(self, m: int, budget: int) -> List[Tuple[_Live, int]]:
        """Move queued requests into slot m while there is room (sessions, handles, KV
        tokens on every stage, this step's prefill token budget).  Returns (session, first
        chunk length) pairs; the first admission of a step always gets at least one chunk."""
        out: List[Tuple[_Live, int]] = []
        while self.queue and len(self.slots[m]) < self.B and self.free_handles:
            if self.ex.sessions.free_rows() - len(out) <= 0:
                break  # the head's executor is shared by several replica engines: no row left
            req = self.queue[0]
            res = self._reserve(req)
            if self.reserved_tokens + res > self.capacity_tokens and self.live:
                break  # wait for retirements
            feed = list(req.prompt) + list(req.generated)  # failover re-prefill: prompt + generated
            take = min(len(feed), self.prefill_chunk, max(budget, 0))
            if take <= 0:
                if out:
                    break
                take = min(len(feed), self.prefill_chunk)
            self.queue.pop(0)
            lv = _Live(req, self.free_handles.pop(), m, pending=feed)
            self.reserved_tokens += res
            self.slots[m].append(lv)
            self.live[req.rid] = lv
            out.append((lv, take))
            budget -= take
        return out

    def _retire(self, lv: _Live, reason: str) -> None:
        if lv.retired:
            return
        lv.retired = True
        req = lv.req
        req.done = True
        req.finish_reason = req.finish_reason or reason
        req.t_done = time.perf_counter()
        self.slots[lv.slot].remove(lv)
        self.closes[lv.slot].append(lv.handle)
        self.free_handles.append(lv.handle)
        self.live.pop(req.rid, None)
        self.reserved_tokens -= self._reserve(req)
        self.ex.sessions.close(self._key(lv.handle))
        self.finished.append(req)
        if self.on_finish is not None:
            self.on_finish(req)

    def _accept(self, lv: _Live, tok: int) -> None:
        """Reference client stop rules (src/main.py:190-205): EOS is not emitted, a token
        repeated ``stop_on_repeat`` times in a row ends generation, max_new_tokens."""
        req = lv.req
        if req.done:
            return
        if req.t_first is None:
            req.t_first = time.perf_counter()
        if req.eos_token_id is not None and tok == req.eos_token_id:
            self._retire(lv, "eos")
            return
        if req.stop_on_repeat and req.generated and tok == req.generated[-1] and len(req.generated) > 1:
            req._repeat += 1
            if req._repeat >= req.stop_on_repeat:
                self._retire(lv, "repeat")
                return
        else:
            req._repeat = 0
        req.generated.append(int(tok))
        self.tokens_generated += 1
        if self.on_token is not None:
            self.on_token(req, int(tok))
        if len(req.generated) >= req.max_new_tokens:
            self._retire(lv, "length")

    def _book(self, step: Optional[_Step]) -> None:
        """Host bookkeeping of a step's tokens (pinned copy issued a round ago)."""
        if step is None or step.booked:
            return
        step.booked = True
        if not step.consumed:
            self._consume(step)
        wait_event(step.event, self.timeout_s, "token copy")
        toks = step.tok_host[: len(step.rows)].tolist() if step.tok_host is not None else []
        for (lv, n, samples), t in zip(step.rows, toks):
            if samples and not lv.retired and t >= 0:
                self._accept(lv, int(t))

    def _consume(self, step: _Step) -> None:
        """Make the step's tokens usable on the device and start their async host copy."""
        if step.consumed:
            return
        step.consumed = True
        if step.waiter is not None:
            step.tok_dev = step.waiter()
        n = len(step.rows)
        if n == 0 or step.tok_dev is None:
            return
        self._pin_k = (self._pin_k + 1) % len(self._pin)
        host = self._pin[self._pin_k]
        if host.numel() < n:
            host = self._pin[self._pin_k] = torch.empty(2 * n, dtype=torch.int64,
                                                        pin_memory=self.dev.type == "cuda")
        host[:n].copy_(step.tok_dev[:n], non_blocking=True)
        step.tok_host = host
        if self.dev.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            step.event = ev

    # ------------------------------------------------------------------ one head step
    def _head_step(self, m: int) -> None:
        prev2, prev = self.booking[m], self.inflight[m]
        self._book(prev2)                       # tokens of two steps ago: stop checks
        if prev is not None:
            self._consume(prev)                 # tokens of the last step: device feed
        # (a session retired just now still had a row in ``prev``: that token is ignored)
        budget = self.max_step_tokens
        dec: List[_Live] = [lv for lv in self.slots[m] if not lv.pending]
        budget -= len(dec)
        chunks: List[Tuple[_Live, int]] = []
        for lv in self.slots[m]:
            if lv.pending and lv.admitted and budget > 0:
                take = min(len(lv.pending), self.prefill_chunk, budget)
                chunks.append((lv, take))
                budget -= take
        admitted = self._admit(m, budget)
        chunks.extend(admitted)
        rows: List[Tuple[_Live, int, bool]] = [(lv, 1, True) for lv in dec]
        recs = [(lv.handle, 1, lv.fed, F_SAMPLE, lv.req.seed) for lv in dec]
        ids_host: List[int] = []
        for lv, take in chunks:
            last = take == len(lv.pending)
            flags = (F_RESET if lv.fed == 0 else 0) | (F_SAMPLE if last else 0)
            recs.append((lv.handle, take, lv.fed, flags, lv.req.seed))
            rows.append((lv, take, last))
            ids_host.extend(lv.pending[:take])
        closes = self.closes[m]
        self.closes[m] = []
        hdr = self._header(m, recs, closes, [lv for lv, _ in admitted])
        for lv, _ in admitted:
            lv.admitted = True
        step = _Step(m, rows, t_issue=time.perf_counter())
        if self.S > 1:
            self.ch.send_msg(1, hdr)
        if rows:
            # inputs: decode tokens gathered on the device from the last step + prompt chunk ids
            parts = []
            if dec:
                src_rows = [lv.last_row for lv in dec]
                if src_rows == list(range(prev.tok_dev.shape[0])):
                    parts.append(prev.tok_dev)  # steady decode: same sessions, same order
                else:
                    idx = torch.tensor(src_rows, dtype=torch.long)
                    parts.append(prev.tok_dev.index_select(0, idx.to(self.dev, non_blocking=True)))
            if ids_host:
                parts.append(torch.tensor(ids_host, dtype=torch.long).to(self.dev, non_blocking=True))
            x = parts[0] if len(parts) == 1 else torch.cat(parts)
            out = self._compute(recs, x, m)
            for r, (lv, n, _) in enumerate(rows):
                lv.fed += n
                lv.last_row = r
                if lv.pending:
                    del lv.pending[:n]
            if self.S == 1:
                step.tok_dev = self._sample_tail(hdr, out)
            else:
                self._hop_send(1, out)
                _, step.waiter = self.ch.recv(self.S - 1, (len(rows),), torch.long, which="ret")
        self.booking[m] = prev
        self.inflight[m] = step
        self.steps_run += 1

    # ------------------------------------------------------------------ hidden-state hop
    def _hop_rows(self, T: int, is_decode: bool) -> int:
        """Rows a hop of a T-token step carries: T, or with the graph hop the sender's batch
        bucket when its step replays a graph (the send recorded in it moves the whole static
        output)."""
        if self.graph_hop:
            return self.ex.graph_rows(T, is_decode) or T
        return T

    def _hop_send(self, dst: int, out: torch.Tensor) -> None:
        if not self.graph_hop:
            self.ch.send(dst, out)
        elif self.ex.last_hooked:  # the send ran inside the replay
            self.ch.count_send(self.ex.graph_rows(out.shape[0], True) * out.shape[1] * out.element_size())
        else:  # eager steps: the same compute stream, so the communicator sees one op order
            self.ch.send_on_stream(dst, out.contiguous())

    def _header(self, m: int, recs, closes: List[int], admitted: List[_Live]) -> np.ndarray:
        hdr = np.zeros(HDR + SEQ_REC * len(recs) + len(closes) + ADM_REC * len(admitted), dtype=np.int64)
        T = sum(int(r[1]) for r in recs)
        hdr[:HDR] = (KIND_STEP, m, len(recs), T, len(closes), len(admitted), self.rounds, 0)
        off = HDR
        if recs:
            hdr[off:off + SEQ_REC * len(recs)] = np.asarray(recs, dtype=np.int64).reshape(-1)
            off += SEQ_REC * len(recs)
        if closes:
            hdr[off:off + len(closes)] = closes
            off += len(closes)
        for lv in admitted:
            p = lv.req.params
            hist = list(lv.req.generated)[-RECENT:]
            hdr[off:off + 6] = (lv.handle, _f2i(p.temperature), _f2i(p.top_p), int(p.top_k),
                                _f2i(p.repetition_penalty), len(hist))
            hdr[off + 6:off + 6 + len(hist)] = hist
            off += ADM_REC
        return hdr

    # ------------------------------------------------------------------ shared compute
    def _compute(self, seq_recs, x, m: int):
        ex = self.ex
        seqs = [(self._key(int(h)), int(n)) for h, n, _, _, _ in seq_recs]
        reset = [bool(int(f) & F_RESET) for _, _, _, f, _ in seq_recs]
        starts = [int(s) for _, _, s, _, _ in seq_recs]
        e0 = e1 = None
        if self.timing and self.dev.type == "cuda":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        with trace_range(f"pp.rank{self.rank}.slot{m}"):
            out = ex.forward(seqs, x, reset=reset, starts=starts, max_length=self.max_len, hook_owner=self)
        if self.replay is not None:
            self.replay.store(seq_recs, out)
        if e1 is not None:
            e1.record()
            self._events.append((e0, e1))
        return out

    def _sample_tail(self, hdr: np.ndarray, logits: torch.Tensor) -> torch.Tensor:
        n_seq, n_close, n_adm = int(hdr[2]), int(hdr[4]), int(hdr[5])
        recs = hdr[HDR:HDR + SEQ_REC * n_seq].reshape(n_seq, SEQ_REC)
        off = HDR + SEQ_REC * n_seq + n_close
        adm = hdr[off:off + ADM_REC * n_adm].reshape(n_adm, ADM_REC)
        if n_adm:
            self.sampler.admit(adm)
        handles = recs[:, 0]
        self.sampler.seed_host[handles] = recs[:, 4]
        positions = recs[:, 2] + recs[:, 1]  # index of the token being sampled
        samples = (recs[:, 3] & F_SAMPLE) != 0
        rows = None if samples.all() else np.nonzero(samples)[0]
        return self.sampler.sample(logits, handles, positions, rows)

    # ------------------------------------------------------------------ non-head stage
    def _stage_step(self) -> bool:
        """Receive one header (+ payload), compute, forward.  False on STOP."""
        hdr = self.ch.recv_msg(self.rank - 1, timeout_s=self.idle_timeout_s)
        kind = int(hdr[0])
        if kind == KIND_STOP:
            if not self.is_tail:
                self.ch.send_msg(self.rank + 1, hdr)
            return False
        if kind == KIND_STATS:
            if not self.is_tail:
                self.ch.send_msg(self.rank + 1, hdr)
            self.ch.all_gather_floats(self._stats_row())
            return True
        if kind == KIND_REPLAY:
            if not self.is_tail:
                self.ch.send_msg(self.rank + 1, hdr)
            self._replay_step(hdr)
            self.steps_run += 1
            return True
        m, n_seq, T, n_close = int(hdr[1]), int(hdr[2]), int(hdr[3]), int(hdr[4])
        if not self.is_tail:
            self.ch.send_msg(self.rank + 1, hdr)  # the successor plans while we compute
        recs = hdr[HDR:HDR + SEQ_REC * n_seq].reshape(n_seq, SEQ_REC)
        closes = hdr[HDR + SEQ_REC * n_seq:HDR + SEQ_REC * n_seq + n_close]
        x = waiter = None
        rows = T
        if n_seq:
            # the payload's HOST wait happens outside exec_lock: a predecessor that dies between its
            # header and its payload leaves this thread blocked here until the channel times out or
            # is aborted, and the executor must stay usable meanwhile (stage-local recovery adopts
            # this channel's sessions into a new one, the TCP handler keeps serving).  Everything
            # that touches the device (stream waits, staging copies) runs under the lock: another
            # thread may be capturing a decode graph.
            is_dec = bool((recs[:, 1] == 1).all())
            rows = self._hop_rows(T, is_dec)
            into = None
            if is_dec and (self.recv_into or self.graph_hop) and self.ex.graph_rows(T, True) is not None:
                # straight into the static input of the decode graph this step replays (every
                # backend: no receive slab, no copy into the graph input)
                got = self.ex.graph_input(T, int((recs[:, 2] + recs[:, 1]).max()), owner=self)
                if got is not None:
                    into = (got[0][:rows], got[1])
            # (posting the receive stays outside the lock too: a first RCCL receive can block on its
            # peer's connection set-up; decode graphs are captured in thread-local mode, so this
            # thread's stream calls never invalidate another thread's capture)
            t, waiter = self.ch.recv(self.rank - 1, (rows, self.H), self.ex.dtype, into=into)
            self.recvs += 1
            self.recvs_into += int(into is not None and t is into[0])
            hw = getattr(waiter, "host_wait", None)
            if hw is not None:
                hw()
        if self.ch.closed:
            raise ChannelError("channel aborted while waiting for a payload")
        with self.ex.exec_lock:
            if waiter is not None:
                x = waiter()
                if x is not None and rows != T:
                    x = x[:T]
            for c in closes:  # before the compute: a closed handle may be re-admitted in this very step
                self.ex.sessions.close(self._key(int(c)))
            if n_seq:
                out = self._compute(recs.tolist(), x, m)
                if self.is_tail:
                    tok = self._sample_tail(hdr, out)
                    self.ch.send(0, tok, which="ret")
                else:
                    self._hop_send(self.rank + 1, out)
        self.steps_run += 1
        return True

    idle_timeout_s: Optional[float] = None  # None: the channel timeout
    # driver processes (bench.py, the CLI client) set this: the first engine of the process freezes
    # the setup heap (``settle_heap``); long-lived servers, which build an engine per client
    # channel, leave the collector alone
    freeze_heap: bool = False

    # ------------------------------------------------------------------ driving
    def _settle_heap(self) -> None:
        if self.freeze_heap:
            settle_heap()

    def release(self) -> None:
        """Give the executor back: remove this engine's graph hook and the graphs that recorded its
        send (idempotent; stop / failure / end of ``serve`` call it, so a shared executor never
        replays a send on a closed communicator)."""
        self.ex.clear_graph_hook(self)
        self.ex.release_owner(self)

    def run_rounds(self, n: int) -> None:
        """n rounds x M slot-steps on every rank (lock-step unit of the benchmark)."""
        self._settle_heap()
        try:
            for _ in range(n):
                for m in range(self.M):
                    if self.is_head:
                        self._head_step(m)
                    elif not self._stage_step():
                        self.stopped = True
                        self.release()
                        return
                self.rounds += 1
        except ChannelError as e:
            self._fail(str(e))

    def serve(self) -> None:
        """Non-head ranks: process steps until the head's STOP."""
        self._settle_heap()
        try:
            while self._stage_step():
                pass
            self.stopped = True
        except ChannelError as e:
            self._fail(str(e))
        finally:
            self.release()

    def run_until_idle(self, max_rounds: Optional[int] = None) -> List[Request]:
        """Head: run rounds until every submitted request has finished."""
        k = 0
        while not self.idle:
            self.run_rounds(1)
            k += 1
            if max_rounds is not None and k >= max_rounds:
                break
        self.drain()
        return self.finished

    def drain(self) -> None:
        """Head: book every outstanding step (end of a run)."""
        if not self.is_head:
            return
        try:
            for m in range(self.M):
                self._book(self.booking[m])
                self.booking[m] = None
            for m in range(self.M):
                self._book(self.inflight[m])
                self.inflight[m] = None
            for m in range(self.M):  # rows decided finished at this point: nothing in flight anymore
                for lv in list(self.slots[m]):
                    if lv.req.done:
                        self._retire(lv, lv.req.finish_reason or "done")
        except ChannelError as e:
            self._fail(str(e))

    def stop(self) -> None:
        """Head: close every session downstream and stop the serving ranks."""
        if not self.is_head or self.ch is None or self.failed:
            return
        try:
            hdr = np.zeros(HDR, dtype=np.int64)
            hdr[0] = KIND_STOP
            self.ch.send_msg(1, hdr)
            self.ch.flush(timeout_s=self.timeout_s)
        except (ChannelError, RuntimeError) as e:
            logger.warning(f"stop: {e}")
        finally:
            self.release()

    def _fail(self, why: str) -> None:
        self.failed = why
        logger.error(f"[{self.name} rank {self.rank}] pipeline failure: {why}")
        self.release()
        if self.ch is not None:
            self.ch.abort()
        if self.is_head:
            pend = [lv.req for m in range(self.M) for lv in self.slots[m] if not lv.req.done] + list(self.queue)
            with self.ex.exec_lock:  # the head's rows / pages go back to the (shared) executor
                for m in range(self.M):
                    for lv in self.slots[m]:
                        if not lv.req.done:
                            self.failed_sessions[lv.req.rid] = (lv.handle, lv.req)
                        if not self.park_on_fail:
                            self.ex.sessions.close(self._key(lv.handle))
                    self.slots[m] = []
                self.live.clear()
                self.queue = []
            if self.park_on_fail:
                self.park_sessions()
            raise PipelineFailure(why, pend)
        if self.park_on_fail:
            self.park_sessions()
        raise PipelineFailure(why)

    # ------------------------------------------------------------------ stage-local recovery
    def park_sessions(self) -> int:
        """Keep this engine's KV past its channel's failure under ``park:<name>:<handle>`` keys (the
        session TTL still evicts them) so a replacement channel can adopt them."""
        pre, n = self.name + ":", 0
        with self.ex.exec_lock:
            for sid in [k for k in self.ex.sessions.sessions if k.startswith(pre)]:
                self.ex.sessions.rename(sid, "park:" + sid)
                n += 1
        return n

    def _adopt(self, handle: int, length: int, old_handle: int) -> Tuple[bool, bool]:
        """Take over the failed channel's session ``old_handle`` as ``handle``: its KV (truncated to
        ``length``: a step in flight at the failure may have reached some stages) and its replay
        rows.  The failed engine's keys are ``<old>:<handle>`` (its thread may not have noticed
        the failure yet) or, parked, ``park:<old>:<handle>``.  Returns (KV found, rows found)."""
        old = self.resume.get("prefix")
        if old is None:
            return False, False
        s = None
        for key in (f"{old}:{int(old_handle)}", f"park:{old}:{int(old_handle)}"):
            s = self.ex.sessions.rename(key, self._key(int(handle)))
            if s is not None:
                s.length = min(s.length, int(length))
                break
        cache = self.resume.get("cache")
        rows = (self.replay is not None and cache is not None and 0 < length <= cache.max_len and
                length <= self.replay.max_len)
        if rows:
            self.replay.rows(handle, length).copy_(cache.rows(old_handle, length))
        return s is not None, rows

    def _replay_step(self, hdr: np.ndarray) -> None:
        """REPLAY header: adopt the listed sessions; the stage before ``target`` sends its cached
        output rows, the ``target`` (the replacement) prefills them (rebuilding its KV), everyone
        else only adopts; the tail also admits the sessions' sampling state.  A survivor that lost
        a session's KV (evicted) or the source's rows fails the channel loudly: the front end then
        re-places the sessions by re-prefill."""
        n, T, target, n_adm = int(hdr[2]), int(hdr[3]), int(hdr[4]), int(hdr[5])
        recs = hdr[HDR:HDR + REPLAY_REC * n].reshape(n, REPLAY_REC)
        adm = hdr[HDR + REPLAY_REC * n:HDR + REPLAY_REC * n + ADM_REC * n_adm].reshape(n_adm, ADM_REC)
        with self.ex.exec_lock:
            lost = 0
            for h, L, oh in recs:
                kv, rows = self._adopt(int(h), int(L), int(oh))
                lost += int(self.rank != target and not kv) + int(self.rank == target - 1 and not rows)
            self.resume.pop("cache", None)  # every row is copied: the failed channel's cache can go
            if lost:
                self._fail(f"replay: {lost} session state(s) missing on rank {self.rank}")
            if self.rank == target - 1:
                self._replay_send(torch.cat([self.replay.rows(int(h), int(L)) for h, L, _ in recs]))
            elif self.rank == target:
                _, waiter = self.ch.recv(self.rank - 1, (T, self.H), self.ex.dtype)
                x = waiter()
                out = self.ex.forward([(self._key(int(h)), int(L)) for h, L, _ in recs], x, reset=[True] * n,
                                      max_length=self.max_len)
                if self.replay is not None:
                    self.replay.store([(int(h), int(L), 0) for h, L, _ in recs], out)
            if self.is_tail and n_adm:
                self.sampler.admit(adm)
        logger.info(f"[{self.name} rank {self.rank}] replay: " +
                    (f"rebuilt the KV of {n} session(s) from {T} replayed rows" if self.rank == target
                     else f"adopted {n} session(s)"))

    def _replay_send(self, x: torch.Tensor) -> None:
        """Replayed rows to the next rank, in the same op order as the data plane's hidden-state
        hops (with the graph hop those go on the compute stream, not the channel's side stream)."""
        if self.graph_hop:
            self.ch.send_on_stream(self.rank + 1, x.contiguous())
        else:
            self.ch.send(self.rank + 1, x)

    def resume_sessions(self, items: Sequence[Tuple[Request, int, int]], target: int) -> List[Request]:
        """Head of the channel that replaced a failed one (same surviving servers, a spare in
        position ``target``): continue ``items`` = (request, its handle in the failed channel, L =
        tokens every stage had processed: prompt + all generated but the last) without
        re-prefilling - the survivors adopt their KV, the stage before ``target`` replays its cached
        outputs to the spare, and decoding resumes by feeding each session's last token at position
        L.  Returns the requests resumed (the rest should be re-placed the usual way)."""
        if not self.is_head or self.ch is None or not (0 < target < self.S):
            return []
        done: List[Tuple[_Live, int]] = []
        with self.ex.exec_lock:
            for req, oh, L in items:
                if L <= 0 or not req.generated or not self.free_handles or L > self.max_len:
                    continue
                m = min(range(self.M), key=lambda k: len(self.slots[k]))
                if len(self.slots[m]) >= self.B:
                    continue
                res = self._reserve(req)
                if self.reserved_tokens + res > self.capacity_tokens:
                    continue
                h = self.free_handles.pop()
                kv, rows = self._adopt(h, int(L), int(oh))
                if not kv or (target == 1 and not rows):
                    self.ex.sessions.close(self._key(h))
                    self.free_handles.append(h)
                    continue  # the head lost it: re-placed by re-prefill instead
                lv = _Live(req, h, m, fed=int(L), pending=[int(req.generated[-1])], admitted=True)
                self.reserved_tokens += res
                self.slots[m].append(lv)
                self.live[req.rid] = lv
                req._repeat = repeat_run(req.generated)
                done.append((lv, int(oh)))
        self.resume.pop("cache", None)  # adopted rows are in this engine's own cache now
        if not done:
            return []
        recs = np.asarray([(lv.handle, lv.fed, oh) for lv, oh in done], dtype=np.int64)
        hdr = np.zeros(HDR + REPLAY_REC * len(done) + ADM_REC * len(done), dtype=np.int64)
        hdr[:HDR] = (KIND_REPLAY, 0, len(done), int(recs[:, 1].sum()), int(target), len(done), self.rounds, 0)
        hdr[HDR:HDR + REPLAY_REC * len(done)] = recs.reshape(-1)
        off = HDR + REPLAY_REC * len(done)
        for lv, _ in done:
            p = lv.req.params
            hist = list(lv.req.generated)[-RECENT:]  # what the sampler held when the last token was drawn
            hdr[off:off + 6] = (lv.handle, _f2i(p.temperature), _f2i(p.top_p), int(p.top_k),
                                _f2i(p.repetition_penalty), len(hist))
            hdr[off + 6:off + 6 + len(hist)] = hist
            off += ADM_REC
        try:
            self.ch.send_msg(1, hdr)
            if target == 1:
                self._replay_send(torch.cat([self.replay.rows(lv.handle, lv.fed) for lv, _ in done]))
        except ChannelError as e:
            self._fail(str(e))
        logger.info(f"[{self.name}] stage-local recovery: {len(done)} session(s) resumed, stage {target} "
                    f"rebuilt from {sum(lv.fed for lv, _ in done)} replayed rows")
        return [lv.req for lv, _ in done]

    def _stats_row(self) -> List[float]:
        st = self.ch.stats(reset=True) if self.ch is not None else {"recv_wait_ms": 0.0, "bytes_sent": 0}
        n = len(self._events)
        ms = self.stage_ms() if self.dev.type == "cuda" else None
        return [float(ms or 0.0), float(n), float(st["recv_wait_ms"]), float(st["bytes_sent"]),
                float(self.ex.end - self.ex.start)]

    def gather_stage_stats(self) -> List[dict]:
        """Head: per-stage timing of the steps since the last gather, every rank's row gathered
        over the ctrl group (a STATS header walks the chain first): mean compute ms per
        micro-batch step (HIP events), timed steps, mean ms the stage's stream waited for its
        payload, hop bytes sent, blocks.  The pipeline analogue of the reference client's
        per-hop ``last_decode_stage_times`` (src/rpc_transport.py:98-103, 824-839)."""
        if not self.is_head:
            raise RuntimeError("gather_stage_stats() is a head operation")
        if self.ch is None:
            rows = [self._stats_row()]
        else:
            hdr = np.zeros(HDR, dtype=np.int64)
            hdr[0] = KIND_STATS
            try:
                self.ch.send_msg(1, hdr)
                rows = self.ch.all_gather_floats(self._stats_row())
            except ChannelError as e:
                self._fail(str(e))
        keys = ("compute_ms", "steps", "recv_wait_ms", "bytes_sent", "blocks")
        return [dict(zip(keys, r), stage=k) for k, r in enumerate(rows)]

    def stage_ms(self) -> Optional[float]:
        if not self._events:
            return None
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in self._events]
        self._events.clear()
        return sum(ms) / len(ms)
