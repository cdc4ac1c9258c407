"""Single-node pipeline-parallel serving over RCCL point-to-point (xGMI).

Reference: the Stage-0 client sends hidden states to each remote stage in turn over
hivemind RPC in a star topology and gets a token back from the last stage
(reference src/rpc_transport.py:738-766, :802-833; src/main.py:164-211), one session at a
time.  On one MI355X node the same dataflow becomes a chain of RCCL send/recv over the
direct xGMI link between neighbouring GPUs:

    rank 0 (embed + blocks [0,s0)) -> rank 1 -> ... -> rank N-1 (blocks + norm + lm_head + sampler)
         ^                                                                       |
         +----------------------- token ids int64[B] ----------------------------+

* M micro-batches of B sessions are in flight (M >= N keeps every stage busy); every
  "step" advances all M*B sessions by one token.
* Receives are pre-posted one micro-batch ahead so the hop overlaps compute; outputs are
  copied into a ring of send buffers so a pending send never aliases the hipGraph output.
* Sampling happens on the last stage (reference semantics) with the repetition-penalty
  history kept ON DEVICE (no host round trip per token).
* gloo carries the identical protocol on CPU (tests).
* Replicas (data parallel over pipelines, BASELINE config "4 stages x 2 replicas"): with
  ``stages=S < world`` the node runs R = world / S independent pipelines, replica r on ranks
  [r*S, (r+1)*S), each with its own RCCL sub-communicator (``dist.new_group``) so the
  replicas' hops never share a communicator.  Sessions are assigned to replicas by
  ``assign_sessions`` (throughput-proportional, the load_balancing.py rule re-expressed
  for replicas of a whole pipeline).
* The token return hop (last stage -> stage 0) runs on its OWN communicator per replica
  (``make_token_groups``).  RCCL serialises the P2P operations of one communicator on one
  stream, so with 2 stages the forward hidden send (0 -> 1) and the token receive (1 -> 0)
  would share a stream: stage 0's send of micro-batch m+1 would sit in front of the receive
  of token m, and the pipeline would only make progress while RCCL can complete the small
  token send eagerly.  Two communicators make the two directions independent streams.
"""
from __future__ import annotations

import dataclasses
import time
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import ops
from ..runtime.executor import StageExecutor
from ..runtime.sampler import RECENT, SamplingParams
from ..utils.tracing import trace_range


@dataclasses.dataclass
class MicroBatch:
    sids: List[str]
    tokens: Optional[torch.Tensor] = None      # stage 0: next input ids [B] (device)
    recent: Optional[torch.Tensor] = None      # last stage: [B, RECENT] int32
    recent_len: Optional[torch.Tensor] = None  # last stage: [B] int32
    step: int = 0
    index: int = 0


def assign_sessions(n_sessions: int, throughputs: Sequence[float]) -> List[int]:
    """Replica index for each of ``n_sessions`` new sessions, proportional to replica
    throughput (largest-remainder rounding; ties to the lower index)."""
    tp = [max(float(t), 0.0) for t in throughputs]
    tot = sum(tp)
    if tot <= 0:
        tp, tot = [1.0] * len(tp), float(len(tp))
    quota = [n_sessions * t / tot for t in tp]
    base = [int(q) for q in quota]
    rem = n_sessions - sum(base)
    order = sorted(range(len(tp)), key=lambda i: (-(quota[i] - base[i]), i))
    for i in order[:rem]:
        base[i] += 1
    out: List[int] = []
    for r, n in enumerate(base):
        out.extend([r] * n)
    return out


def make_replica_groups(world: int, stages: int):
    """One sub-communicator per replica (every rank creates every group, same order)."""
    if stages >= world:
        return None
    return [dist.new_group(list(range(r * stages, (r + 1) * stages))) for r in range(world // stages)]


def make_token_groups(world: int, stages: int):
    """One extra communicator per replica for the last -> first token hop (see module doc).
    Collective: every rank calls it, after ``make_replica_groups``, in the same order."""
    if stages <= 1 or not dist.is_initialized():
        return None
    return [dist.new_group(list(range(r * stages, (r + 1) * stages))) for r in range(world // stages)]


class PipelineEngine:
    def __init__(self, executor: StageExecutor, rank: int, world: int, sampling: SamplingParams,
                 n_micro: int, batch: int, seed: int = 0, send_ring: int = 4, timing: bool = False,
                 stages: Optional[int] = None, groups=None, tp: int = 1, tok_groups=None):
        """``tp`` > 1: consecutive groups of ``tp`` lanes (pipelines) are the tensor-parallel
        shards of one replica; they sample with the same seeds so their tokens agree."""
        self.ex = executor
        self.rank, self.world = rank, world
        S = int(stages or world)
        if world % S:
            raise ValueError(f"world size {world} is not a multiple of stages={S}")
        self.S, self.R = S, world // S
        self.replica, self.stage = rank // S, rank % S
        self.base = self.replica * S
        self.group = groups[self.replica] if groups else None
        self.tok_group = tok_groups[self.replica] if tok_groups else self.group
        self.dev = executor.device
        self.sp = sampling
        self.B, self.M = batch, n_micro
        self.seed = seed
        self.tp = max(1, int(tp))
        self.first = self.stage == 0
        self.last = self.stage == S - 1
        H = executor.cfg.hidden_size
        self.H = H
        self.mbs = [MicroBatch([f"r{self.replica}s{m}_{b}" for b in range(batch)], index=m) for m in range(n_micro)]
        # send ring (hidden for mid stages, tokens for the last stage)
        self._ring = [None] * send_ring
        self._ring_work = [None] * send_ring
        self._ring_k = 0
        self._pending_recv = None  # (tag, work, buffer)
        self.timing = timing
        self._events: List = []
        self.record = False  # rank 0: keep every received token (tests / generation API)
        self.tokens_out: List[List[torch.Tensor]] = [[] for _ in range(n_micro)]
        if self.last:
            dev = self.dev
            B = batch
            self._temps = torch.full((B,), sampling.temperature, dtype=torch.float32, device=dev)
            self._topp = torch.full((B,), sampling.top_p, dtype=torch.float32, device=dev)
            self._topk = torch.full((B,), sampling.top_k, dtype=torch.int32, device=dev)
            self._rp = torch.full((B,), sampling.repetition_penalty, dtype=torch.float32, device=dev)
            self._arange = torch.arange(B, dtype=torch.int64, device=dev)
            for mb in self.mbs:
                mb.recent = torch.zeros(B, RECENT, dtype=torch.int32, device=dev)
                mb.recent_len = torch.zeros(B, dtype=torch.int32, device=dev)

    # ------------------------------------------------------------------ comm helpers
    def _send(self, t: torch.Tensor, dst: int, group=None):
        k = self._ring_k
        self._ring_k = (k + 1) % len(self._ring)
        w = self._ring_work[k]
        if w is not None:
            w.wait()
        buf = self._ring[k]
        if buf is None or buf.shape != t.shape or buf.dtype != t.dtype:
            buf = torch.empty_like(t)
            self._ring[k] = buf
        buf.copy_(t)
        self._ring_work[k] = dist.isend(buf, dst, group=group or self.group)

    def _post_recv(self, shape, dtype, src, group=None):
        buf = torch.empty(shape, dtype=dtype, device=self.dev)
        return dist.irecv(buf, src, group=group or self.group), buf

    def _flush_sends(self):
        for i, w in enumerate(self._ring_work):
            if w is not None:
                w.wait()
                self._ring_work[i] = None

    # ------------------------------------------------------------------ sampling on the last stage
    def _sample(self, mb: MicroBatch, logits: torch.Tensor) -> torch.Tensor:
        """One fused kernel per micro-batch: penalty + top-k/top-p draw (or argmax at T <= 0)
        and the device-side history update (no host round trip, no extra device ops)."""
        B = logits.shape[0]
        seeds = (self._arange[:B] + (self.seed * 1000003 + mb.step * 7919 + mb.index * 104729
                                     + (self.replica // self.tp) * 15485863) * 4096)
        tok = ops.sample(logits, self._temps[:B], self._topp[:B], self._topk[:B], self._rp[:B], mb.recent,
                         mb.recent_len, seeds, update_history=True)
        mb.step += 1
        return tok

    # ------------------------------------------------------------------ one micro-batch on this stage
    def _compute(self, mb: MicroBatch, x: torch.Tensor, n_tokens: int, reset: bool):
        seqs = [(sid, n_tokens) for sid in mb.sids]
        if self.timing and self.dev.type == "cuda":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        with trace_range(f"pp.stage{self.stage}.mb{mb.index}"):
            out = self.ex.forward(seqs, x, reset=[reset] * len(seqs))
        if self.timing and self.dev.type == "cuda":
            e1.record()
            self._events.append((e0, e1))
        return out

    def _input_shape(self, n_tokens):
        return (self.B * n_tokens, self.H)

    def run_round(self, n_tokens: int, prompts: Optional[Sequence[torch.Tensor]] = None, reset: bool = False):
        """Advance every micro-batch by one step (``n_tokens`` per session; prompts for prefill)."""
        M = self.M
        dt = self.ex.dtype
        for m, mb in enumerate(self.mbs):
            # ---------------- input
            if self.first:
                if prompts is not None:
                    x = prompts[m].to(self.dev).view(-1)
                elif self.S == 1:
                    x = mb.tokens
                else:
                    w, buf = self._tok_recv[m]
                    w.wait()
                    x = buf
                    if self.record:
                        self.tokens_out[m].append(buf.clone())
            else:
                if self._pending_recv is None:
                    self._pending_recv = self._post_recv(self._input_shape(n_tokens), dt, self.rank - 1)
                w, x = self._pending_recv
                w.wait()
                self._pending_recv = None
                if m + 1 < M:  # pre-post the next micro-batch's receive (overlaps this compute)
                    self._pending_recv = self._post_recv(self._input_shape(n_tokens), dt, self.rank - 1)
            # ---------------- compute
            out = self._compute(mb, x, n_tokens, reset)
            # ---------------- output
            if self.last:
                tok = self._sample(mb, out)
                if self.S == 1:
                    mb.tokens = tok
                    if self.record:
                        self.tokens_out[m].append(tok.clone())
                else:
                    self._send(tok, self.base, group=self.tok_group)
            else:
                self._send(out, self.rank + 1)
        if self.first and self.S > 1:
            # receive this round's tokens (posted after all sends of the round, in micro-batch order)
            self._tok_recv = [self._post_recv((self.B,), torch.long, self.base + self.S - 1, group=self.tok_group)
                              for _ in range(M)]

    def prefill(self, prompts: Sequence[torch.Tensor]):
        """prompts[m]: int64 [B, L] token ids for micro-batch m (stage 0 only reads them)."""
        L = int(prompts[0].shape[1]) if prompts is not None else 0
        self.run_round(L, prompts=prompts if self.first else None, reset=True)

    def decode(self, n_steps: int):
        for _ in range(n_steps):
            self.run_round(1)

    def finish(self):
        self._flush_sends()
        if self.first and self.S > 1:
            # tokens of the final round are still in flight; consume them
            for m, (w, buf) in enumerate(getattr(self, "_tok_recv", [])):
                w.wait()
                if self.record:
                    self.tokens_out[m].append(buf.clone())
            self._tok_recv = []
            self._tok_recv_consumed = True

    def generated(self) -> List[List[List[int]]]:
        """rank 0: tokens[m][b] generated so far (needs ``record=True`` before the run)."""
        out = []
        for m in range(self.M):
            if not self.tokens_out[m]:
                out.append([[] for _ in range(self.B)])
                continue
            t = torch.stack(self.tokens_out[m], 1).cpu()
            out.append(t.tolist())
        return out

    def stage_ms(self) -> Optional[float]:
        if not self._events:
            return None
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in self._events]
        self._events.clear()
        return sum(ms) / len(ms)
