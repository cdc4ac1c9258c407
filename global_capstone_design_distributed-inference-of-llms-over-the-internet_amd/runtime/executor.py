"""StageExecutor: one pipeline stage (a contiguous block range) on one device.

Replaces the reference's Stage0 / StageSegment / StageLast modules
(reference src/llama_partition.py:76-474) and the optimized HF layer they wrap
(petals/llama/block.py:39-248) with an MI355X-first step function:

* weights resident in HBM (no per-forward CPU<->GPU layer streaming),
* a paged KV cache written in place by the fused RoPE kernel,
* ragged batches: any mix of sessions, each contributing ``n_tokens`` (prefill chunks,
  decode steps, replays) executed as ONE forward over the concatenated tokens,
* per layer 7 launches on the decode path: add+RMSNorm, QKV GEMM, RoPE+KV write,
  paged attention, O GEMM, add+RMSNorm, gate/up GEMM with fused SwiGLU, down GEMM,
* decode steps replayed from hipGraphs captured per (batch bucket, context bucket);
* the last stage applies the final norm and ``lm_head`` to the LAST token of each
  sequence only (the reference projects every prefill position, src/llama_partition.py:470).

Attention is causal for prefill (the reference's optimized layer gets no mask and is
NOT causal: src/llama_partition.py:118 -> petals/llama/block.py:136-137).
"""
from __future__ import annotations

import dataclasses
import logging
import math
import os
import threading
import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import native, ops
from ..ops import moe
from ..models.config import ModelConfig
from ..models.weights import StageWeights
from .kv_cache import PagedKVCache
from .session import SessionManager, SessionState

logger = logging.getLogger(__name__)

# per-path weight tensors a layer loop reads (what CPU offload streams)
_PACKED_FIELDS = ("input_norm", "post_norm", "qkv_p", "o_p", "gate_up_p", "down_p", "router_p")
_DENSE_FIELDS = ("input_norm", "post_norm", "qkv", "o", "gate_up", "down", "router")
_GPT2_FIELDS = ("ln1_w", "ln1_b", "attn_w", "attn_b", "proj_w", "proj_b", "ln2_w", "ln2_b", "fc_w", "fc_b",
                "fc2_w", "fc2_b")


@dataclasses.dataclass
class Plan:
    """Host-side description of one ragged step.

    ``h64`` / ``h32`` are the step's metadata in pinned host memory; the device copies
    (``meta_i64`` / ``meta_i32``) are made on first use.  A graph-replayed decode step never
    touches them: it stages the padded metadata of its batch bucket in ONE host-to-device
    copy of its own (``_DecodeGraph.replay``)."""
    sessions: List[SessionState]
    ntoks: np.ndarray
    starts: np.ndarray
    T: int
    max_ctx: int
    is_decode: bool
    h64: np.ndarray                     # [2, T] positions, slots (pinned host view)
    h32: np.ndarray                     # [2*T + S] q_seq, q_ctx, last_rows (pinned host view)
    qblocks: Optional[torch.Tensor] = None  # [2, NB] MFMA-attention query blocks (prefill steps)
    superblocks: Optional[torch.Tensor] = None  # [2, NSB] runs of <= 4 blocks (grouped prefill kernel)
    fablocks: Optional[torch.Tensor] = None  # [2, NBF] FA2 prefill workgroup blocks (csrc/attention_fa.hip)
    fa_waves: int = 4                   # waves per FA2 workgroup (ops.fa_plan)
    _dev: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
    _upload: Optional[object] = None    # callable making the device copies

    def _device(self):
        if self._dev is None:
            self._dev = self._upload()
        return self._dev

    @property
    def meta_i64(self) -> torch.Tensor:
        return self._device()[0]

    @property
    def meta_i32(self) -> torch.Tensor:
        return self._device()[1]

    @property
    def positions(self):
        return self.meta_i64[0]

    @property
    def slots(self):
        return self.meta_i64[1]

    @property
    def q_seq(self):
        return self.meta_i32[: self.T]

    @property
    def q_ctx(self):
        return self.meta_i32[self.T: 2 * self.T]

    @property
    def last_rows(self):
        return self.meta_i32[2 * self.T:]


class _Pinned:
    """Double-buffered pinned host staging for per-step metadata (async H2D without races)."""

    def __init__(self, n_i64: int, n_i32: int, device):
        self.device = torch.device(device)
        pin = self.device.type == "cuda"
        self.i64 = [torch.empty(n_i64, dtype=torch.int64, pin_memory=pin) for _ in range(2)]
        self.i32 = [torch.empty(n_i32, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.events = [None, None]
        self.k = 0

    def next(self):
        self.k ^= 1
        ev = self.events[self.k]
        if ev is not None:
            ev.synchronize()
        return self.i64[self.k], self.i32[self.k]

    def mark(self):
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            self.events[self.k] = ev


class StageExecutor:
    def __init__(self, cfg: ModelConfig, weights: StageWeights, device, *, dtype=torch.bfloat16,
                 page_size: int = 64, max_sessions: int = 256, max_seq_len: Optional[int] = None,
                 kv_cache_bytes: Optional[int] = None, kv_fraction: float = 0.9, use_graphs: Optional[bool] = None,
                 graph_max_batch: int = 256, max_tokens_per_step: int = 8192, offload: bool = False,
                 keep_layers_on_gpu: int = 0, tp=None, warmup: Optional[bool] = None):
        """``tp``: a ``parallel.tensor_parallel.TPGroup`` when ``weights`` is a tensor-parallel
        shard (``cfg`` is then the shard config); partial sums are all-reduced after the
        o and down projections."""
        cfg.validate()
        if offload and cfg.is_moe:
            # the streamed slot layers carry only the per-path projection fields; the MoE MLP
            # also reads the router and per-expert row-major weights.  Mixtral-8x7B (93 GB bf16)
            # fits one MI355X resident, so offload is rejected rather than half-supported.
            raise ValueError("CPU offload is not supported for MoE (Mixtral) models: serve them resident")
        self._tp = tp if (tp is not None and getattr(tp, "active", tp.size > 1)) else None
        self.cfg = cfg
        self.w = weights
        self.device = torch.device(device)
        self.dtype = dtype
        self.n_layers = len(weights.layers)
        self.start, self.end = weights.start, weights.end
        self.is_first = weights.has_embed
        self.is_last = weights.has_head
        self.nh, self.nkv, self.D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.D)
        self.max_seq_len = int(max_seq_len or cfg.max_position_embeddings)
        if cfg.sliding_window and self.max_seq_len > cfg.sliding_window:
            # Mistral / Mixtral sliding-window attention: sessions are capped at the window, inside
            # which sliding-window and full causal attention are the same computation
            logger.info(f"max_seq_len capped at sliding_window={cfg.sliding_window}")
            self.max_seq_len = int(cfg.sliding_window)
        self.max_tokens = max_tokens_per_step
        if cfg.model_type != "gpt2":
            self.cos, self.sin = ops.rope_cos_sin(self.D, self.max_seq_len, cfg.rope_theta, self.device,
                                                  cfg.rope_scaling)
        if kv_cache_bytes is None:
            kv_cache_bytes = PagedKVCache.auto_budget_bytes(self.device, fraction=kv_fraction)
        num_pages = PagedKVCache.pages_for_bytes(kv_cache_bytes, self.n_layers, self.nkv, self.D, page_size)
        max_useful = max_sessions * math.ceil(self.max_seq_len / page_size)
        num_pages = max(1, min(num_pages, max_useful))
        self.cache = PagedKVCache(self.n_layers, num_pages, self.nkv, self.D, page_size, dtype, self.device)
        self.sessions = SessionManager(self.cache, max_sessions, self.max_seq_len)
        self.use_graphs = (self.device.type == "cuda") if use_graphs is None else bool(use_graphs)
        self.use_graphs = self.use_graphs and self.device.type == "cuda" and cfg.model_type != "gpt2" and \
            os.environ.get("MPAMD_GRAPHS", "1") != "0"
        if self._tp is not None and not getattr(self._tp, "capturable", False):
            # torch's all-reduce (gloo, or ProcessGroupNCCL's private stream) is not replayable:
            # graphs under TP need the direct RCCL communicator (parallel/rccl.py)
            self.use_graphs = False
        self.graph_max_batch = graph_max_batch
        self._graphs: Dict[tuple, "_DecodeGraph"] = {}
        self._graph_pool = None
        # graph_input: receive graphs are per OWNER (a channel engine): two engines sharing this
        # executor never hand each other's hidden states to a replay.  Owner -> small tag (part of
        # the graph key); (tag, base key) -> last receive slot handed out; tag -> (key, graph) its
        # next step replays
        self._owner_tags = weakref.WeakKeyDictionary()
        self._owner_strong: Dict[int, tuple] = {}
        self._next_tag = 1
        self._recv_slot: Dict[tuple, int] = {}
        self._recv_pin: Dict[int, tuple] = {}
        # qkv fold per decode-graph batch bucket (_confirm_qkv_fold's end-to-end A/B on THIS executor)
        self.qkv_fold_by_bucket: Dict[int, bool] = {}
        self._pinned = _Pinned(2 * max_tokens_per_step, 2 * max_tokens_per_step + max_sessions, self.device)
        self.last_step_ms: Optional[float] = None
        # graph_hook(out): recorded at the END of every decode graph capture (the static output
        # buffer), e.g. the stage hop's RCCL send (parallel/engine.py graph hop); last_graphed
        # says whether the last step ran as a graph replay
        self.graph_hook = None
        self._hook_owner = None
        self.last_graphed = self.last_hooked = False
        # MFMA flash attention for prefill steps (csrc/attention_mfma.hip)
        self._attn_mfma_prefill = cfg.model_type != "gpt2" and cfg.head_dim in (64, 128)
        # GQA decode: the whole group of a kv head in the MFMA rows (2x the VALU kernel at nrep 8)
        # MHA decode stays on the flash-decoding kernel: forcing it onto the MFMA kernel (15 of 16
        # MFMA rows idle) measured 11005 vs 13617 tok/s at 64 sessions and 13847 vs 16248 at 128
        # (Llama-2-7B, profiles/r1_attn_mha_mfma_vs_simt/)
        self._attn_mfma_gqa = self._attn_mfma_prefill and self.nh // self.nkv >= 4
        # decode steps of GQA models on the MFMA kernel (a lab script may flip this before the
        # first decode step to A/B the flash-decoding kernel)
        self.gqa_decode_mfma = self._attn_mfma_gqa
        # prefill: up to 4 query blocks of a sequence per workgroup share each K/V step
        # (csrc/attention_mfma.hip attn_mfma_grp_kernel)
        self._attn_grouped = True
        self._cur_sb = None
        # prefill steps with a row-major attention output: the FA2 kernel on 32x32x16 MFMA with
        # transposed LDS reads of V (csrc/attention_fa.hip); other shapes keep the 16x16 one
        self._attn_fa = self._attn_mfma_prefill and \
            ops.fa_ok(cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim, page_size)
        self._cur_fb = None
        self._cur_fw = 4
        self._n_cu = torch.cuda.get_device_properties(self.device).multi_processor_count \
            if self.device.type == "cuda" else 256
        # decode steps on the flash-decoding kernel fold RoPE + the KV page write into it
        self._fuse_rope = True
        # shortest split-K context slice (ops.attention_partition): longer on the MFMA GQA kernel
        self._attn_min_part = 256 if self.gqa_decode_mfma else 64
        self._decode_qb: Dict[int, torch.Tensor] = {}
        self._moe_y: Dict[int, torch.Tensor] = {}
        self.timing = False
        # one executor may be driven by the TCP handler's GPU worker AND a device-channel
        # engine thread: every device step (incl. hipGraph capture) runs under this lock
        self.exec_lock = threading.RLock()
        # fp8 weights: W8A16 (ops.linear_w8: fp8 weights dequantized into the bf16 MFMA, bf16
        # activations, the fused-norm path below; default) or W8A8 (MPAMD_FP8_MODE=w8a8: fp8 MFMA,
        # activations quantized per row before every GEMM, RMSNorm kernels; also under TP).
        # MPAMD_FP8_MODE=mx: the W8A16 path with the o projection of <= 64-row GQA decode steps on the
        # W8A8-MX GEMM (ops.linear_mx: MX e4m3 activations, block-scaled MFMA), its input written as
        # MX by the attention kernel's epilogue (no quantizer launch); profiles/r6mx
        fp8_mode = os.environ.get("MPAMD_FP8_MODE", "w8a16")
        self._w8 = (self.device.type == "cuda" and weights.fp8 and cfg.model_type != "gpt2" and not cfg.is_moe and
                    self._tp is None and fp8_mode in ("w8a16", "mx") and
                    os.environ.get("MPAMD_FUSED_NORM", "1") != "0" and
                    all(d % 256 == 0 for d in (cfg.hidden_size, cfg.q_dim, cfg.intermediate_size)) and
                    (cfg.q_dim + 2 * cfg.kv_dim) % 32 == 0)
        self._mx = bool(self._w8 and fp8_mode == "mx")
        if self._w8:
            weights.prepare_w8a16(fold_norms=True)
        # fused-norm decode path (ops/csrc/gemm.hip EpiArgs): no RMSNorm kernels between the
        # layers' GEMMs - dense bf16 or W8A16 Llama stages without TP (MoE / W8A8 / TP keep the
        # norm kernels)
        self._fused = (self.device.type == "cuda" and cfg.model_type != "gpt2" and not cfg.is_moe and
                       self._tp is None and (not weights.fp8 or self._w8) and ops.gemm_policy() != "hipblaslt" and
                       os.environ.get("MPAMD_FUSED_NORM", "1") != "0" and
                       all(d % 128 == 0 for d in (cfg.hidden_size, cfg.q_dim, cfg.intermediate_size)))
        self._ss = ops.norm_stats_buffer(self.device, 2) if self._fused else None
        # first stage on that path: the stage-entry kernel gathers the embedding rows itself
        # (ops.embed_stage_entry; MPAMD_FUSED_ENTRY=0 keeps the separate embedding launch)
        self._fused_entry = os.environ.get("MPAMD_FUSED_ENTRY", "1") != "0"
        # unit RMSNorm weight for > 64-row decode steps over norm-folded packed weights (made
        # here, not inside a hipGraph capture)
        self._ones = torch.ones(cfg.hidden_size, dtype=self.dtype, device=self.device) if self._fused else None
        if self.device.type == "cuda":
            ops.require_native()
            if cfg.model_type != "gpt2" and ops.gemm_policy() != "hipblaslt":
                weights.pack_for_decode(fold_norms=self._fused)
                if self._fused and not all(getattr(L, "folded", False) for L in weights.layers):
                    self._fused = False  # packed before (e.g. a shared weights object): norm kernels
                ops.use_tuned_gemms()  # library GEMM solutions for the row-major shapes
                ops.gemm_workspace(self.device)  # allocated before any hipGraph capture
                ops.attention_counters(self.device)
                ops.load_kernel_table()  # the committed per-shape kernel choices (ops.KERNEL_TABLE)
                if ops.autotune_mode() != "off":
                    H, F = cfg.hidden_size, cfg.intermediate_size
                    shapes = [] if (weights.fp8 or not weights.layers) else \
                        [(cfg.q_dim + 2 * cfg.kv_dim, H, 0), (H, cfg.q_dim, 0), (2 * F, H, 1), (H, F, 0)]
                    if self._fused and shapes:
                        shapes += [(H, cfg.q_dim, 3), (H, F, 3)]
                    if cfg.is_moe and shapes:
                        shapes.append((16 * ((cfg.num_local_experts + 15) // 16), H, 0))  # router
                    if weights.lm_head_p is not None:
                        shapes.append((16 * weights.lm_head_p.shape[0], H, 0))
                    ops.autotune_gemm(shapes, self.device)
                    if self._w8 and weights.layers:
                        ops.autotune_w8([(cfg.q_dim + 2 * cfg.kv_dim, H, 0), (H, cfg.q_dim, 3), (2 * F, H, 1),
                                         (H, F, 3)], self.device)
                    if self._fused and weights.layers and self._fuse_rope:
                        # qkv as split-K partials summed in the attention kernel, per row bucket
                        ops.autotune_qkv_fold(cfg.q_dim + 2 * cfg.kv_dim, H, self.device, fp8=bool(self._w8))
                    elif weights.fp8 and weights.layers:
                        ops.autotune_fp8([(cfg.q_dim + 2 * cfg.kv_dim, H, 0), (H, cfg.q_dim, 0), (2 * F, H, 1),
                                          (H, F, 0)], self.device)
        self._streamer, self._n_stream = None, self.n_layers
        if offload and self.device.type == "cuda":
            self._setup_offload(keep_layers_on_gpu)
        if warmup is None:
            warmup = self.device.type == "cuda" and os.environ.get("MPAMD_WARMUP", "1") != "0"
        # (not under TP: a shape that fails on one rank would desynchronise the all-reduces)
        if warmup and self.device.type == "cuda" and self.n_layers and self._tp is None and self._streamer is None:
            self.warmup()
        logger.info(f"StageExecutor blocks [{self.start},{self.end}) embed={self.is_first} head={self.is_last} "
                    f"kv_pages={num_pages} x {page_size} tokens ({self.cache.nbytes / 2**30:.2f} GiB) "
                    f"graphs={self.use_graphs}")

    # ================================================================== planning
    def plan(self, seqs: Sequence[Tuple[str, int]], *, reset: Sequence[bool] = (), max_length: Optional[int] = None,
             starts: Optional[Sequence[int]] = None) -> Plan:
        """Open/extend sessions and build device metadata for a ragged step.

        ``seqs``: (session_id, n_tokens) pairs.  ``reset[i]`` clears the session first
        (prefill / replay).  ``starts[i]`` (optional) rewinds a session to that position
        (Petals' ``start_from_position``).
        """
        S = len(seqs)
        sess: List[SessionState] = []
        ntoks = np.empty(S, dtype=np.int32)
        st = np.empty(S, dtype=np.int32)
        for i, (sid, n) in enumerate(seqs):
            s = self.sessions.open(sid, max_length)
            if reset and reset[i]:
                self.sessions.reset(sid)
            if starts is not None and starts[i] is not None and starts[i] < s.length:
                s.length = int(starts[i])
            self.sessions.reserve(s, s.length + int(n))
            sess.append(s)
            ntoks[i] = n
            st[i] = s.length
        T = int(ntoks.sum())
        if T > self.max_tokens:
            raise ValueError(f"step has {T} tokens > max_tokens_per_step {self.max_tokens}")
        rows = np.fromiter((s.row for s in sess), dtype=np.int32, count=S)
        h64, h32 = self._pinned.next()
        n64 = h64[: 2 * T].numpy().reshape(2, T) if T else np.empty((2, 0), np.int64)
        n32 = h32[: 2 * T + S].numpy()
        native.build_meta(rows, st, ntoks, self.sessions.table, self.cache.page_size, n64[0], n64[1], n32[:T],
                          n32[T:2 * T], n32[2 * T:])
        self.sessions.sync_table()
        max_ctx = int((st + ntoks).max()) if S else 0
        is_decode = bool(S and (ntoks == 1).all())
        pinned = self._pinned

        def upload():
            if self.device.type == "cuda":
                d64 = h64[: 2 * T].view(2, T).to(self.device, non_blocking=True)
                d32 = h32[: 2 * T + S].to(self.device, non_blocking=True)
                pinned.mark()  # the pinned buffers are reused two plans later: after this copy
            else:
                d64 = h64[: 2 * T].view(2, T).clone()
                d32 = h32[: 2 * T + S].clone()
            return d64, d32

        qb = sb = fb = None
        fa_waves = 4
        if self.device.type == "cuda" and not is_decode and self._attn_fa:
            fbn, fa_waves = ops.fa_plan(ntoks, self.nh, self.nkv, self._n_cu)
            fb = torch.from_numpy(fbn).to(self.device, non_blocking=True)
        if self.device.type == "cuda" and not is_decode and self._attn_mfma_prefill:
            qb = torch.from_numpy(ops.query_blocks(ntoks, self.nh // self.nkv)).to(self.device, non_blocking=True)
            if self._attn_grouped:
                sb = torch.from_numpy(ops.query_superblocks(ntoks, self.nh // self.nkv)).to(self.device,
                                                                                              non_blocking=True)
        return Plan(sess, ntoks, st, T, max_ctx, is_decode, n64, n32, qb, sb, fb, fa_waves, _upload=upload)

    def commit(self, plan: Plan) -> None:
        for s, n in zip(plan.sessions, plan.ntoks):
            s.length += int(n)
            s.step += 1

    # ================================================================== execution
    def forward(self, seqs: Sequence[Tuple[str, int]], x: torch.Tensor, **plan_kw) -> torch.Tensor:
        """One ragged step.  ``x``: token ids [T] (first stage) or hidden [T, H].

        Returns hidden [T, H] (non-last stage) or last-token logits [S, V] (last stage).
        Steps larger than ``max_tokens_per_step`` run as consecutive chunks (chunked prefill,
        upstream Petals TransformerBackend.inference_step): a long prompt is split at token
        boundaries, later pieces attend to the KV the earlier pieces wrote.
        """
        T = sum(int(n) for _, n in seqs)
        prompts = plan_kw.pop("prompts", None)
        hook_owner = plan_kw.pop("hook_owner", None)
        if prompts is not None and not any(p is not None for p in prompts):
            prompts = None
        if T > self.max_tokens:
            if prompts is not None:
                raise ValueError("deep prompts need the step to fit max_tokens_per_step")
            return self._forward_chunked(seqs, x, **plan_kw)
        plan = self.plan(seqs, **plan_kw)
        out = self.run(plan, x, prompt=self._prompt_rows(seqs, prompts) if prompts is not None else None,
                       hook_owner=hook_owner)
        self.commit(plan)
        return out

    def _prompt_rows(self, seqs, prompts):
        """Deep prompts (upstream iterate_rpc_inference / TransformerBackend: before every block,
        ``hidden[:, :P] += prompt``, applied to the first P tokens of this step). ``prompts[i]`` is
        None or ``[n_layers, P, H]`` for sequence i. Returns (rows [R], values [n_layers, R, H])."""
        rows, vals, off = [], [], 0
        for (sid, n), p in zip(seqs, prompts):
            if p is not None:
                if p.dim() != 3 or p.shape[0] != self.n_layers or p.shape[2] != self.cfg.hidden_size:
                    raise ValueError(f"prompts must be [{self.n_layers}, P, {self.cfg.hidden_size}], "
                                     f"got {tuple(p.shape)}")
                k = min(int(p.shape[1]), int(n))
                rows.extend(range(off, off + k))
                vals.append(p[:, :k])
            off += int(n)
        if not rows:
            return None
        return (torch.tensor(rows, dtype=torch.long, device=self.device),
                torch.cat(vals, 1).to(self.device, self.dtype))

    def _forward_chunked(self, seqs, x, reset: Sequence[bool] = (), starts=None, max_length=None):
        C = self.max_tokens
        pieces = []  # (seq index, token offset within the seq, count, offset into x)
        xoff = 0
        for i, (sid, n) in enumerate(seqs):
            off = 0
            while off < n:
                pieces.append((i, off, min(int(n) - off, C), xoff + off))
                off += pieces[-1][2]
            xoff += int(n)
        chunks, cur, used = [], [], 0
        for pc in pieces:
            if used + pc[2] > C and cur:
                chunks.append(cur)
                cur, used = [], 0
            take = pc
            while used + take[2] > C:  # a piece longer than the room left: split it
                room = C - used
                cur.append((take[0], take[1], room, take[3]))
                chunks.append(cur)
                cur, used = [], 0
                take = (take[0], take[1] + room, take[2] - room, take[3] + room)
            cur.append(take)
            used += take[2]
        if cur:
            chunks.append(cur)
        hidden, logits = [], [None] * len(seqs)
        for ch in chunks:
            sub = [(seqs[i][0], c) for (i, off, c, _) in ch]
            sub_reset = [bool(reset[i]) if (reset and off == 0) else False for (i, off, c, _) in ch]
            sub_starts = [(starts[i] if (starts is not None and off == 0) else None) for (i, off, c, _) in ch]
            xs = torch.cat([x[xo:xo + c] for (_, _, c, xo) in ch])
            out = self.forward(sub, xs, reset=sub_reset, starts=sub_starts, max_length=max_length)
            if self.is_last:
                for r, (i, off, c, _) in enumerate(ch):
                    if off + c == int(seqs[i][1]):
                        logits[i] = out[r]
            else:
                hidden.append(out)
        if self.is_last:
            return torch.stack(logits)
        return torch.cat(hidden)

    def run(self, plan: Plan, x: torch.Tensor, prompt=None, hook_owner=None) -> torch.Tensor:
        if plan.T == 0:
            H = self.cfg.hidden_size
            return torch.empty(0, self.cfg.vocab_size if self.is_last else H, dtype=self.dtype, device=self.device)
        x = x.to(self.device)
        if not self.is_first and x.dtype != self.dtype:
            x = x.to(self.dtype)
        ev = None
        if self.timing and self.device.type == "cuda":
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        self.last_graphed = self.last_hooked = False
        if prompt is None and self.use_graphs and plan.is_decode and plan.T <= self.graph_max_batch:
            hooked = self.graph_hook is not None and hook_owner is not None and hook_owner is self._hook_owner
            out = self._run_graph(plan, x, hooked, owner=hook_owner)
            self.last_graphed, self.last_hooked = True, hooked
        elif self.cfg.model_type == "gpt2":
            out = self._forward_gpt2(plan, x, prompt=prompt)
        else:
            self._cur_sb = plan.superblocks
            self._cur_fb = plan.fablocks
            self._cur_fw = plan.fa_waves
            try:
                out = self._forward_llama(x, plan.positions, plan.slots, plan.q_seq, plan.q_ctx, plan.last_rows,
                                          plan.T, plan.max_ctx, None, qblocks=plan.qblocks, prompt=prompt,
                                          decode=plan.is_decode)
            finally:
                self._cur_sb = None
                self._cur_fb = None
        if ev is not None:
            ev[1].record()
            ev[1].synchronize()
            self.last_step_ms = ev[0].elapsed_time(ev[1])
        return out

    # ------------------------------------------------------------------ llama
    def decode_qblocks(self, T: int) -> torch.Tensor:
        """Query blocks of a decode step (one token per block); cached per batch size so
        hipGraph captures reuse the same buffer."""
        qb = self._decode_qb.get(T)
        if qb is None:
            import numpy as np

            qb = torch.from_numpy(np.stack([np.arange(T), np.ones(T)]).astype(np.int32)).to(self.device)
            self._decode_qb[T] = qb
        return qb

    def _attend(self, qkv, kc, vc, q_seq, q_ctx, out, ws, ps, np_, packed, qblocks, max_ctx):
        """Paged attention: MFMA flash attention for prefill blocks (``qblocks``) and GQA decode,
        else the flash-decoding kernel."""
        table = self.sessions.table_dev
        if qblocks is None and self.gqa_decode_mfma and self.device.type == "cuda":
            T = qkv.shape[0]
            ps2 = 128 * math.ceil(ps / 128)
            np2 = max(1, math.ceil(ps * np_ / ps2))
            return ops.attention_mfma(qkv, kc, vc, table, q_seq, q_ctx, self.decode_qblocks(T), self.nh, self.nkv,
                                      self.scale, out=out, workspace=ws, part_size=ps2, num_parts=np2,
                                      packed=packed)
        fb = getattr(self, "_cur_fb", None)
        if qblocks is not None and fb is not None and not packed:
            return ops.attention_fa(qkv, kc, vc, table, q_seq, q_ctx, fb, self.nh, self.nkv, self.scale, out=out,
                                    workspace=ws, max_ctx=max_ctx, waves=getattr(self, "_cur_fw", 4))
        if qblocks is not None:
            return ops.attention_mfma(qkv, kc, vc, table, q_seq, q_ctx, qblocks, self.nh, self.nkv, self.scale,
                                      out=out, workspace=ws, max_ctx=max_ctx, packed=packed,
                                      superblocks=getattr(self, "_cur_sb", None))
        return ops.paged_attention(qkv, kc, vc, table, q_seq, q_ctx, self.nh, self.nkv, self.scale, out=out,
                                   workspace=ws, part_size=ps, num_parts=np_, packed=packed)

    def _qkv_fold(self, T: int) -> bool:
        """Decode steps of T rows: qkv as split-K partial slabs folded into the attention kernel's
        loads - where ``_confirm_qkv_fold``'s decode-step A/B on this executor found it faster for
        the batch bucket the step replays (an unconfirmed bucket keeps the reduce launch)."""
        if not (self._fuse_rope and self._fused and self.device.type == "cuda") or \
                os.environ.get("MPAMD_QKV_FOLD", "1") == "0":
            return False
        cfg = self.cfg
        return bool(self.qkv_fold_by_bucket.get(self._bucket(T), False)) and \
            ops.rwk_split(T, cfg.q_dim + 2 * cfg.kv_dim, cfg.hidden_size, bool(self._w8)) > 0

    def _rope_attend(self, qkv, positions, slots, kc, vc, q_seq, q_ctx, out, ws, ps, np_, packed, qblocks, max_ctx,
                     decode, qkv_part=None, mx_out=None, mx_used=None):
        """RoPE + KV write + attention.  Decode steps that run on the flash-decoding kernel do all
        three in one launch (ops.paged_attention_rope); everything else keeps rope_kv_write.
        ``qkv_part``: q / k / v as the qkv GEMM's split-K slabs (decode RoPE paths only).  ``mx_out``:
        (ax, as_) MX buffers the GQA kernel writes instead of ``out`` when it can (one part, packed,
        head_dim 128); it then appends True to ``mx_used``."""
        if decode and qblocks is None and self._fuse_rope and self.gqa_decode_mfma and self.device.type == "cuda":
            T = qkv.shape[0]
            ps2 = 128 * math.ceil(ps / 128)
            np2 = max(1, math.ceil(ps * np_ / ps2))
            mx = mx_out if (mx_out is not None and np2 == 1 and packed and self.D == 128) else None
            if mx is not None and mx_used is not None:
                mx_used.append(True)
            return ops.attention_mfma_rope(qkv, kc, vc, self.sessions.table_dev, q_seq, q_ctx, self.decode_qblocks(T),
                                           positions, self.cos, self.sin, slots, self.nh, self.nkv, self.scale,
                                           out=out, workspace=ws, part_size=ps2, num_parts=np2, packed=packed,
                                           qkv_part=qkv_part, mx_out=mx)
        if decode and qblocks is None and self._fuse_rope and not (
                self.gqa_decode_mfma and self.device.type == "cuda"):
            return ops.paged_attention_rope(qkv, kc, vc, self.sessions.table_dev, q_seq, q_ctx, positions, self.cos,
                                            self.sin, slots, self.nh, self.nkv, self.scale, out=out, workspace=ws,
                                            part_size=ps, num_parts=np_, packed=packed, qkv_part=qkv_part)
        if qkv_part is not None:
            raise RuntimeError("qkv partial slabs need a fused RoPE decode attention path")
        ops.rope_kv_write(qkv, positions, self.cos, self.sin, kc, vc, slots, self.nh, self.nkv)
        return self._attend(qkv, kc, vc, q_seq, q_ctx, out, ws, ps, np_, packed, qblocks, max_ctx)

    def _forward_llama(self, x, positions, slots, q_seq, q_ctx, last_rows, T, max_ctx, attn_part,
                       bufs: Optional[dict] = None, qblocks=None, prompt=None, decode=False):
        cfg, w = self.cfg, self.w
        H, eps = cfg.hidden_size, cfg.rms_norm_eps
        dev, dt = self.device, self.dtype
        table = self.sessions.table_dev
        if bufs is None:
            bufs = {}
        e = lambda name, shape, dtype=dt: bufs.get(name) if name in bufs else torch.empty(shape, dtype=dtype, device=dev)  # noqa: E731
        fp8_dec = prompt is None and self._fp8_ok(T)
        fused_dec = (not fp8_dec and prompt is None and self._fused and self.n_layers > 0 and
                     (T <= 64 and (self._w8 or self._packed_ok(T)) or (not self._w8 and self._fused_wide_ok(T))))
        if self.is_first and not (fused_dec and self._fused_entry and x.dim() == 1 and x.is_contiguous()):
            h = ops.embedding(x, w.embed, out=e("h", (T, H)))
        elif self.is_first:
            h = None  # the fused path's stage-entry kernel gathers the embedding rows itself
        else:
            h = x
        if attn_part is None:
            attn_part = ops.attention_partition(T, self.nkv, max_ctx, min_part=self._attn_min_part)
        ps, np_ = attn_part
        ws = e("attn_ws", (max(1, T * self.nh * np_ * (self.D + 2)),), torch.float32)
        res = e("res", (T, H))
        qkv = e("qkv", (T, cfg.q_dim + 2 * cfg.kv_dim))
        o = e("o", (T, H))
        mlp = e("mlp", (T, H))
        if fp8_dec:
            # fp8 W8A8 decode path: packed bf16 activations are quantized per row right before
            # each GEMM (csrc/fp8.hip); weights stream at 1 byte per parameter
            pk = ops.packed_numel
            xn = e("xn_p", (pk(T, H),))
            F = cfg.intermediate_size
            # row-major: their only reader is the row quantization kernel (coalesced rows)
            attn = e("attn", (T, cfg.q_dim))
            act = e("act", (T, F))
            a8 = e("a8", (pk(T, max(H, cfg.q_dim, cfg.intermediate_size)),), torch.uint8)
            asc = e("a8_scale", (((T + 15) // 16) * 16 * 33,), torch.float32)
            # the two norm sites emit fp8 + row scales themselves (norm.hip a8 output): only the
            # attention output and the SwiGLU output still take a separate quantization pass
            for li, L in enumerate(w.layers):
                if li == 0:
                    ops.rmsnorm(h, L.input_norm, eps, out=xn, residual=res, mode=2, packed=True, a8=a8, a8_scale=asc)
                else:
                    ops.rmsnorm(mlp, L.input_norm, eps, out=xn, residual=res, mode=1, packed=True, a8=a8,
                                a8_scale=asc)
                ops.linear_fp8(a8, asc, L.qkv_q, L.qkv_s, T, out=qkv)
                kc, vc = self.cache.layer(li)
                self._rope_attend(qkv, positions, slots, kc, vc, q_seq, q_ctx, attn, ws, ps, np_, False, qblocks,
                                  max_ctx, decode)
                ops.quant_rows_fp8(attn, out=a8, scale=asc)
                ops.linear_fp8(a8, asc, L.o_q, L.o_s, T, out=o)
                self._ar(o)
                ops.rmsnorm(o, L.post_norm, eps, out=xn, residual=res, mode=1, packed=True, a8=a8, a8_scale=asc)
                ops.linear_fp8(a8, asc, L.gate_up_q, L.gate_up_s, T, out=act, epilogue=1)
                ops.quant_rows_fp8(act, out=a8, scale=asc)
                ops.linear_fp8(a8, asc, L.down_q, L.down_s, T, out=mlp)
                self._ar(mlp)
        elif fused_dec:
            # fused-norm decode path: 5 launches per layer (qkv, attention, o, gate/up, down).
            # The residual stream r lives row-major in ``res`` and packed in ``xr``; o / down add
            # their product into it in their epilogue and accumulate sum(r^2) per row, and qkv /
            # gate_up (norm weights folded into their packed weights) scale their rows by
            # rsqrt(mean r^2 + eps).  ss[0] / ss[1]: input- / post-attention-norm statistics;
            # each producer clears the other buffer, whose consumer has already run.
            pk = ops.packed_numel
            xr = e("xr_p", (pk(T, H),))
            attn = e("attn_p", (pk(T, cfg.q_dim),))
            act = e("act_p", (pk(T, cfg.intermediate_size),))
            ss_in, ss_post = self._ss[0], self._ss[1]
            if self._w8:  # fp8 weights (W8A16): same launches, 1 byte per weight streamed
                def gemm(a, L, name, **kw):
                    return ops.linear_w8(a, getattr(L, name + "_w8"), getattr(L, name + "_ws"), T, **kw)
            else:
                def gemm(a, L, name, **kw):
                    return ops.linear(a, None, wp=getattr(L, name + "_p"), a_rows=T, **kw)
            # decode steps whose qkv GEMM measured faster as split-K partial slabs: the attention
            # kernel sums the slabs + applies the row scale on its q / k / v loads (no reduce launch)
            fold = decode and qblocks is None and self._qkv_fold(T)
            # W8A8-MX o projection: the attention epilogue writes the MX activation (GQA decode)
            Q = cfg.q_dim
            mx_o = None
            if (self._mx and decode and qblocks is None and T <= 64 and self.gqa_decode_mfma and self._fuse_rope and
                    ops.rwk_split(T, H, Q, 2) > 0):
                mx_o = (e(f"mx_ax{Q}", (16 * ((T + 15) // 16) * Q,), torch.uint8), e(f"mx_as{Q}", (2 * Q,), torch.uint8))
            for li, L in self._iter_layers(_PACKED_FIELDS):
                if li == 0 and h is None:  # first stage: embedding lookup + stage entry in one launch
                    ops.embed_stage_entry(x, w.embed, xr, res, ss_in)
                elif li == 0:
                    ops.rmsnorm(h, L.input_norm, eps, out=xr, residual=res, mode=3, packed=True, ss=ss_in)
                qp = None
                if fold:
                    if self._w8:
                        part = ops.linear_partials(xr, T, w8=L.qkv_w8, w_scale=L.qkv_ws, out=qkv)
                    else:
                        part = ops.linear_partials(xr, T, wp=L.qkv_p, out=qkv)
                    qp = (part, ss_in, 1.0 / H, eps)
                else:
                    gemm(xr, L, "qkv", out=qkv, ss_in=ss_in, eps=eps)
                kc, vc = self.cache.layer(li)
                used = []
                self._rope_attend(qkv, positions, slots, kc, vc, q_seq, q_ctx, attn, ws, ps, np_, True, qblocks,
                                  max_ctx, decode, qkv_part=qp, mx_out=mx_o, mx_used=used)
                if used:
                    ops.linear_mx(mx_o[0], mx_o[1], L.o_w8, L.o_ws, T, out=res, epilogue=3, residual=res, ap_out=xr,
                                  ss_out=ss_post, ss_zero=ss_in)
                else:
                    gemm(attn, L, "o", out=res, epilogue=3, residual=res, ap_out=xr, ss_out=ss_post, ss_zero=ss_in)
                gemm(xr, L, "gate_up", out=act, epilogue=1, out_packed=True, ss_in=ss_post, eps=eps)
                gemm(act, L, "down", out=res, epilogue=3, residual=res, ap_out=xr, ss_out=ss_in, ss_zero=ss_post)
            mlp = None
        elif prompt is None and self._packed_ok(T):
            # decode path: activations feeding a GEMM stay in the packed MFMA-fragment layout
            pk = ops.packed_numel
            xn = e("xn_p", (pk(T, H),))
            attn = e("attn_p", (pk(T, cfg.q_dim),))
            act = e("act_p", (pk(T, cfg.intermediate_size),))
            for li, L in self._iter_layers(_PACKED_FIELDS):
                # weights packed for the fused path (> 64 rows here) carry the norm weights in
                # their columns: normalise with a unit weight
                g_in, g_post = (self._unit_norm(), self._unit_norm()) if getattr(L, "folded", False) else \
                    (L.input_norm, L.post_norm)
                if li == 0:
                    ops.rmsnorm(h, g_in, eps, out=xn, residual=res, mode=2, packed=True)
                else:
                    ops.rmsnorm(mlp, g_in, eps, out=xn, residual=res, mode=1, packed=True)
                ops.linear(xn, L.qkv, out=qkv, wp=L.qkv_p, a_rows=T)
                kc, vc = self.cache.layer(li)
                self._rope_attend(qkv, positions, slots, kc, vc, q_seq, q_ctx, attn, ws, ps, np_, True, qblocks,
                                  max_ctx, decode)
                ops.linear(attn, L.o, out=o, wp=L.o_p, a_rows=T)
                self._ar(o)
                ops.rmsnorm(o, g_post, eps, out=xn, residual=res, mode=1, packed=True)
                if L.moe:
                    self._moe_mlp(L, xn, T, mlp, act, e, packed=True)
                    continue
                ops.linear(xn, L.gate_up, out=act, epilogue=1, wp=L.gate_up_p, a_rows=T, out_packed=True)
                ops.linear(act, L.down, out=mlp, wp=L.down_p, a_rows=T)
                self._ar(mlp)
        else:
            xn = e("xn", (T, H))
            attn = e("attn", (T, cfg.q_dim))
            act = e("act", (T, cfg.intermediate_size))
            fold_native = self._folded_native(T)
            for li, L in self._iter_layers(_DENSE_FIELDS):
                # W8A16 layers' only weights carry the norm weights folded in (prepare_w8a16).
                # bf16 layers packed for the fused path carry them in qkv_p / gate_up_p only: when
                # the native GEMM would pick those up, normalise with a unit weight; otherwise
                # keep the real norm weights and hand the GEMM the unfolded row-major weight only
                folded_bf16 = L.folded and not L.w8
                unit = (L.folded and L.w8) or (folded_bf16 and fold_native)
                g_in, g_post = (self._unit_norm(), self._unit_norm()) if unit else (L.input_norm, L.post_norm)
                qkv_p = None if (folded_bf16 and not fold_native) else L.qkv_p
                gu_p = None if (folded_bf16 and not fold_native) else L.gate_up_p
                if prompt is not None:  # deep prompt: the block input (residual stream) += prompt[li]
                    cur = h.clone() if li == 0 else ops.add(res, mlp)
                    cur.index_add_(0, prompt[0], prompt[1][li])
                    ops.rmsnorm(cur, g_in, eps, out=xn, residual=res, mode=2)
                elif li == 0:
                    ops.rmsnorm(h, g_in, eps, out=xn, residual=res, mode=2)
                else:
                    ops.rmsnorm(mlp, g_in, eps, out=xn, residual=res, mode=1)
                ops.linear(xn, L.dense("qkv"), out=qkv, wp=qkv_p)
                kc, vc = self.cache.layer(li)
                self._rope_attend(qkv, positions, slots, kc, vc, q_seq, q_ctx, attn, ws, ps, np_, False, qblocks,
                                  max_ctx, decode)
                ops.linear(attn, L.dense("o"), out=o, wp=L.o_p)
                self._ar(o)
                ops.rmsnorm(o, g_post, eps, out=xn, residual=res, mode=1)
                if L.moe:
                    self._moe_mlp(L, xn, T, mlp, act, e, packed=False)
                    continue
                ops.linear(xn, L.dense("gate_up"), out=act, epilogue=1, wp=gu_p)
                ops.linear(act, L.dense("down"), out=mlp, wp=L.down_p)
                self._ar(mlp)
        hout = res if mlp is None else ops.add(res, mlp, out=e("hout", (T, H)))
        if not self.is_last:
            return hout
        S = last_rows.numel()
        V = cfg.vocab_size
        if w.lm_head_p is not None and self._head_packed_ok(S):
            Vp = 16 * w.lm_head_p.shape[0]
            if w.lm_head_folded and mlp is None and S == T:
                # fused-norm path, every row a last row (decode): lm_head (final norm folded in)
                # reads the packed residual stream the last down GEMM left in ``xr`` and scales
                # each row by its rsqrt(mean r^2 + eps) from ``ss_in`` - no final norm launch
                logits = ops.linear(xr, None, out=e("logits", (S, Vp)), wp=w.lm_head_p, a_rows=S, ss_in=ss_in,
                                    eps=eps)
                return logits[:, :V]
            fn = ops.rmsnorm(hout, self._unit_norm() if w.lm_head_folded else w.final_norm, eps,
                             out=e("fn_p", (ops.packed_numel(S, H),)), rows=last_rows, packed=True)
            logits = ops.linear(fn, None, out=e("logits", (S, Vp)), wp=w.lm_head_p, a_rows=S)
            return logits[:, :V]
        fn = ops.rmsnorm(hout, w.final_norm, eps, out=e("fn", (S, H)), rows=last_rows)
        return ops.linear(fn, w.lm_head, out=e("logits", (S, V)))

    def warmup(self, sizes: Optional[Sequence[int]] = None) -> None:
        """Run throwaway prefill steps at start-up so the first real request does not pay the
        first-call costs of its shapes (hipBLASLt algorithm selection for the row-major GEMMs,
        first launches of the prefill kernels): a cold 64 x 128-token prefill round took 4x
        the warm one.  One single-sequence prefill per size (default: the step
        capacity, 2048 and 512 tokens); the probe session is closed afterwards."""
        cap = min(self.max_tokens, self.max_seq_len - 1)
        sizes = sorted({int(n) for n in (sizes or (cap, 2048, 512)) if 128 < int(n) <= cap}, reverse=True)
        if not sizes:
            return
        sid = "__warmup__"
        with self.exec_lock, torch.inference_mode():
            for n in sizes:
                if self.is_first:
                    x = torch.randint(0, self.cfg.vocab_size, (n,), device=self.device)
                else:
                    x = (0.1 * torch.randn(n, self.cfg.hidden_size, device=self.device)).to(self.dtype)
                try:
                    self.forward([(sid, n)], x, reset=[True])
                except Exception as e:  # noqa: BLE001 - e.g. no KV room for n tokens: warm what fits
                    logger.info(f"warmup of a {n}-token step skipped: {e}")
                finally:
                    self.sessions.close(sid)
            torch.cuda.synchronize(self.device)

    def warmup_serving(self, batch: int, prompt_len: int, decode_steps: int = 2) -> bool:
        """Warm the shapes a serving engine's FIRST steps run, so the first request pays no
        first-call costs: one ragged prefill of ``batch`` sequences x ``prompt_len`` tokens (the
        library GEMM heuristics at batch x prompt rows, the FA2 prefill plan, the last-row lm_head
        and sampler shapes), then ``decode_steps`` decode steps of the batch - the first one
        captures the decode hipGraph of that batch bucket, which the real steps then replay (same
        bucket, same attention partition).  The probe sessions are closed afterwards.  Once per
        (batch, prompt_len) per executor; returns False when skipped (already warm, no room)."""
        if self.device.type != "cuda" or not self.n_layers or batch < 1 or prompt_len < 1:
            return False
        key = (int(batch), int(prompt_len))
        done = self.__dict__.setdefault("_served_warm", set())
        if key in done:
            return False
        ab_steps = 88  # the fold A/B below: 8 windows x (1 capture / warm + 10 timed) steps
        prompt_len = int(min(prompt_len, self.max_seq_len - decode_steps - 2 - ab_steps))
        if prompt_len < 1 or batch > self.sessions.max_sessions:
            return False
        sids = [f"__warm{i}__" for i in range(batch)]
        H = self.cfg.hidden_size
        gen = torch.Generator(device=self.device).manual_seed(1)
        # no_grad, not inference_mode: the decode graph captured here keeps its static buffers,
        # which later steps (inside or outside inference mode) update in place
        with self.exec_lock, torch.no_grad():
            try:
                T = batch * prompt_len
                if self.is_first:
                    x = torch.randint(0, self.cfg.vocab_size, (T,), device=self.device, generator=gen)
                else:
                    x = (0.1 * torch.randn(T, H, device=self.device, generator=gen)).to(self.dtype)
                out = self.forward([(s, prompt_len) for s in sids], x, reset=[True] * batch)
                if self.is_last:
                    self._warm_sampler(out)
                cfg = self.cfg
                pin = ops.qkv_fold_pinned(self._bucket(batch), cfg.q_dim + 2 * cfg.kv_dim, cfg.hidden_size,
                                          bool(self._w8))
                if pin is not None and cfg.model_type != "gpt2":
                    self.qkv_fold_by_bucket[self._bucket(batch)] = pin  # capture the pinned variant below
                for _ in range(decode_steps):
                    if self.is_first:
                        x = torch.randint(0, self.cfg.vocab_size, (batch,), device=self.device, generator=gen)
                    else:
                        x = (0.1 * torch.randn(batch, H, device=self.device, generator=gen)).to(self.dtype)
                    out = self.forward([(s, 1) for s in sids], x)
                    if self.is_last:
                        self._warm_sampler(out)
                self._confirm_qkv_fold(sids, gen)
                done.add(key)
            except Exception as e:  # noqa: BLE001 - e.g. no KV room: the first request warms itself
                logger.info(f"serving warm-up ({batch} x {prompt_len}) skipped: {e}")
                return False
            finally:
                for s in sids:
                    self.sessions.close(s)
            torch.cuda.synchronize(self.device)
        return True

    def _confirm_qkv_fold(self, sids, gen, reps: int = 10) -> Optional[dict]:
        """End-to-end check of the qkv fold for this decode batch: ``ops.autotune_qkv_fold`` times
        the qkv GEMM alone (partials vs the full projection), but the fold also moves work into the
        attention kernel (its q / k / v loads sum the slabs), so the whole decode step - graph
        replays of this batch bucket - is timed both ways and the faster variant kept.  The losing variant's graph is dropped.  Returns {fold: ms} or None.

        Every timed step grows the contexts by a token, so the two variants run in ABBAABBA order
        and each keeps the MEAN of its four windows: both see the same average context (a fixed
        order with the minimum kept handed the first variant ~0.6 % of shorter attention on
        Llama-3-70B, where the fold's real gain is ~1.1 %: profiles/r5z), and short interleaved
        windows see the same clock / thermal state."""
        B = len(sids)
        cfg = self.cfg
        N = cfg.q_dim + 2 * cfg.kv_dim
        key = (ops._m_bucket(B), N, cfg.hidden_size, bool(self._w8))
        if not self.use_graphs or B > self.graph_max_batch or not (self._fuse_rope and self._fused) or \
                os.environ.get("MPAMD_QKV_FOLD", "1") == "0":
            return None
        Bb = self._bucket(B)
        pinned = ops.qkv_fold_pinned(Bb, N, cfg.hidden_size, bool(self._w8))
        if pinned is not None:  # the committed table's decision for this bucket: no timing race
            self.qkv_fold_by_bucket[Bb] = pinned
            return None
        if not ops._QKV_FOLD_CAND.get(key) or ops.autotune_mode() == "off":
            return None
        H = cfg.hidden_size

        def step():
            if self.is_first:
                x = torch.randint(0, cfg.vocab_size, (B,), device=self.device, generator=gen)
            else:
                x = (0.1 * torch.randn(B, H, device=self.device, generator=gen)).to(self.dtype)
            self.forward([(s, 1) for s in sids], x)

        t = {True: 0.0, False: 0.0}
        order = (True, False, False, True, True, False, False, True)
        for fold in order:
            self.qkv_fold_by_bucket[Bb] = fold
            step()  # capture (first time) / warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                step()
            e1.record()
            e1.synchronize()
            t[fold] += e0.elapsed_time(e1) / reps / (len(order) // 2)
        # (interleaved windows measured the 70B fold 0.2-0.8 % faster on five boxes and the 7B one
        # 0.3-1.9 % slower, profiles/r5z: the faster variant wins - with unbiased windows a near
        # tie costs nothing either way)
        keep = t[True] < t[False]
        self.qkv_fold_by_bucket[Bb] = keep
        ops.pin_qkv_fold(Bb, N, cfg.hidden_size, bool(self._w8), keep)  # (ops.save_kernel_table keeps it)
        self.__dict__.setdefault("qkv_fold_ab_ms", {})[Bb] = (round(t[True], 4), round(t[False], 4))
        for k in [k for k in self._graphs if k[0] == Bb and k[3] != keep]:
            del self._graphs[k]
        logger.info(f"qkv fold at batch {B}: {t[True]:.3f} ms/step folded vs {t[False]:.3f} unfolded -> "
                    f"{'fold' if keep else 'reduce launch'}")
        return t

    def _warm_sampler(self, logits: torch.Tensor) -> None:
        """The sampling kernel at this row count, on scratch parameters (no session state)."""
        n, dev = logits.shape[0], self.device
        from .sampler import RECENT

        ops.sample(logits, torch.ones(n, device=dev), torch.full((n,), 0.92, device=dev),
                   torch.full((n,), 50, dtype=torch.int32, device=dev), torch.full((n,), 1.5, device=dev),
                   torch.zeros(n, RECENT, dtype=torch.int32, device=dev), torch.zeros(n, dtype=torch.int32, device=dev),
                   torch.arange(n, dtype=torch.int64, device=dev),
                   workspace=torch.empty(max(n, 64) * logits.shape[1], dtype=torch.float32, device=dev),
                   update_history=True)

    def _folded_native(self, T: int) -> bool:
        """Would ``ops.linear`` run BOTH norm-consuming projections (qkv, gate/up) of a T-row
        row-major step on the native GEMM (i.e. over the norm-folded packed weights)?  The
        row-major branch must then normalise with a unit weight, else with the real one and
        the unfolded weights (one decision per step, so the two never mix)."""
        if self.device.type != "cuda" or ops.gemm_policy() == "hipblaslt":
            return False
        cfg = self.cfg
        H, F = cfg.hidden_size, cfg.intermediate_size
        return ops.native_gemm_ok(T, cfg.q_dim + 2 * cfg.kv_dim, H, 0) and \
            ops.native_gemm_ok(T, 2 * F, H, 1)

    def _unit_norm(self) -> torch.Tensor:
        u = getattr(self, "_ones", None)
        if u is None:
            u = self._ones = torch.ones(self.cfg.hidden_size, dtype=self.dtype, device=self.device)
        return u

    def _moe_mlp(self, L, xn, T, mlp, act, e, packed: bool) -> None:
        """Mixtral sparse-MoE MLP into ``mlp`` (ops/moe.py has the routing math and the
        decode-vs-prefill strategy).  Decode steps run every expert on the whole batch with a
        dense combine matrix: no host sync, so the step stays graph-capturable."""
        cfg = self.cfg
        E, k, H = cfg.num_local_experts, cfg.num_experts_per_tok, cfg.hidden_size
        if packed:
            logits = ops.linear(xn, None, out=e("moe_logits", (T, 16 * L.router_p.shape[0])), wp=L.router_p,
                                a_rows=T)[:, :E]
        else:
            logits = ops.linear(xn, L.router)
        w, idx = moe.route(logits, k)
        acc = e("moe_acc", (T, H), torch.float32)
        acc.zero_()
        gp = (lambda j: L.gate_up_p[j]) if L.gate_up_p is not None else (lambda j: None)  # noqa: E731
        dp = (lambda j: L.down_p[j]) if L.down_p is not None else (lambda j: None)  # noqa: E731
        capturing = self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()
        if packed or T <= 64 or capturing:
            wd = moe.dense_weights(w, idx, E, out=e("moe_w", (T, E), torch.float32))
            # small decode batches leave experts unrouted: their GEMMs are skipped on the device
            # (gate = routed-token count) so a 1-session step streams ~k/E of the expert bytes.
            # y persists per T and starts zeroed: a skipped GEMM leaves finite values * weight 0.
            gated = packed and T * k <= 2 * E
            cnt = (wd > 0).sum(0, dtype=torch.int32) if gated else None
            y = self._moe_y.get(T)
            if y is None:
                y = self._moe_y[T] = torch.zeros(T, H, dtype=self.dtype, device=self.device)
            for j in range(E):
                if packed:
                    g = cnt[j:j + 1] if gated else None
                    ops.linear(xn, L.gate_up[j], out=act, epilogue=1, wp=gp(j), a_rows=T, out_packed=True, gate=g)
                    ops.linear(act, L.down[j], out=y, wp=dp(j), a_rows=T, gate=g)
                else:
                    ops.linear(xn, L.gate_up[j], out=act, epilogue=1, wp=gp(j))
                    ops.linear(act, L.down[j], out=y, wp=dp(j))
                acc.addcmul_(y, wd[:, j:j + 1])
        else:
            # prefill: group the T*k (token, expert) pairs by expert (one host sync per layer)
            flat = idx.reshape(-1)
            order = torch.argsort(flat, stable=True)
            counts = torch.bincount(flat, minlength=E).tolist()
            tok = order // k
            wsel = w.reshape(-1)[order]
            off = 0
            for j, c in enumerate(counts):
                if c == 0:
                    continue
                rows = tok[off:off + c]
                xe = xn.index_select(0, rows)
                a = ops.linear(xe, L.gate_up[j], epilogue=1, wp=gp(j))
                ye = ops.linear(a, L.down[j], wp=dp(j))
                acc.index_add_(0, rows, ye.float() * wsel[off:off + c].unsqueeze(1))
                off += c
        mlp.copy_(acc)
        self._ar(mlp)

    def _ar(self, t: torch.Tensor) -> None:
        """Tensor parallelism: sum the row-parallel partial results over the TP group."""
        if self._tp is not None:
            self._tp.all_reduce(t)

    def _iter_layers(self, fields):
        """``(index, layer)`` over this stage's blocks; with CPU offload the streamed layers come
        from the pinned-host ring (runtime/offload.py) and the resident tail follows."""
        if self._streamer is None:
            yield from enumerate(self.w.layers)
            return
        yield from self._streamer.layers(fields)
        for j in range(self._n_stream, self.n_layers):
            yield j, self.w.layers[j]

    def _setup_offload(self, keep_layers_on_gpu: int) -> None:
        from .offload import LayerStreamer, pin_layer

        w = self.w
        if w.fp8:
            raise ValueError("CPU offload is not supported with fp8 weights")

        keep = max(0, min(int(keep_layers_on_gpu), self.n_layers))
        n_stream = self.n_layers - keep
        host = [pin_layer(L) for L in w.layers[:n_stream]]
        tail = [dataclasses.replace(L, **{f.name: getattr(L, f.name).to(self.device) for f in dataclasses.fields(L)
                                          if isinstance(getattr(L, f.name), torch.Tensor)})
                for L in w.layers[n_stream:]]
        w.layers = host + tail
        for name in ("embed", "pos_embed", "final_norm", "final_norm_b", "lm_head", "lm_head_p"):
            t = getattr(w, name)
            if t is not None:
                setattr(w, name, t.to(self.device))
        self._n_stream = n_stream
        self._streamer = LayerStreamer(host, self.device) if host else None
        self.use_graphs = False  # the slot ring is re-filled every step; graphs would pin one layer set
        logger.info(f"CPU offload: {n_stream} layers streamed from pinned host memory, {keep} resident")

    def _fused_wide_ok(self, M: int) -> bool:
        """Fused-norm decode path at 65..256 rows (bf16): the wide kernels cover every
        projection with its fused epilogue - qkv and gate/up consume the row statistics
        (balanced ring or split-K ring + reduce), o and down produce them (split-K ring, the
        reduce launch applies the residual / packed copy / statistics epilogue)."""
        if not 64 < M <= ops.wide_rows() or self.device.type != "cuda" or not self._packed_ok(M):
            return False
        cfg = self.cfg
        H, F = cfg.hidden_size, cfg.intermediate_size
        return ops.wide_gemm_ok(M, H, cfg.q_dim, 3) and ops.wide_gemm_ok(M, H, F, 3)

    def _head_packed_ok(self, M: int) -> bool:
        return self.device.type == "cuda" and ops.gemm_policy() != "hipblaslt" and 0 < M <= 64 and \
            self.cfg.hidden_size % 128 == 0

    def _fp8_ok(self, M: int) -> bool:
        """fp8 W8A8 decode path: GPU, fp8 weights, fp8 GEMM shape constraints."""
        if self.device.type != "cuda" or not 0 < M <= 64 or not self.w.fp8 or self._w8:
            return False
        cfg = self.cfg
        return all(d % 256 == 0 for d in (cfg.hidden_size, cfg.q_dim, cfg.intermediate_size)) and \
            (cfg.q_dim + 2 * cfg.kv_dim) % 32 == 0

    def _packed_ok(self, M: int) -> bool:
        """Packed-activation decode path: GPU, native GEMM allowed, all projections packed; 65..256
        rows when the balanced ring kernel covers every projection of the layer (dense Llama)."""
        if self.device.type != "cuda" or ops.gemm_policy() == "hipblaslt" or not 0 < M <= ops.wide_rows():
            return False
        if getattr(self, "_packed_ready", None) is None:
            cfg = self.cfg
            dims_ok = all(d % 128 == 0 for d in (cfg.hidden_size, cfg.q_dim, cfg.intermediate_size))
            self._packed_ready = dims_ok and all(getattr(L, "qkv_p", None) is not None for L in self.w.layers)
        if not self._packed_ready:
            return False
        if M > 64:
            cfg = self.cfg
            H, F = cfg.hidden_size, cfg.intermediate_size
            return not cfg.is_moe and self._tp is None and all(
                ops.wide_gemm_ok(M, N, K, epi, epi == 1) for N, K, epi in
                ((cfg.q_dim + 2 * cfg.kv_dim, H, 0), (H, cfg.q_dim, 0), (2 * F, H, 1), (H, F, 0)))
        return True

    # ------------------------------------------------------------------ gpt2 (plumbing family)
    def _forward_gpt2(self, plan: Plan, x, prompt=None):
        cfg, w = self.cfg, self.w
        F = torch.nn.functional
        T, H = plan.T, cfg.hidden_size
        table = self.sessions.table_dev
        if self.is_first:
            h = w.embed[x.long()] + w.pos_embed[plan.positions]
        else:
            h = x
        for li, L in self._iter_layers(_GPT2_FIELDS):
            if prompt is not None:
                h = h.index_add(0, prompt[0], prompt[1][li])
            a = F.layer_norm(h, (H,), L.ln1_w, L.ln1_b, cfg.layer_norm_eps)
            qkv = F.linear(a, L.attn_w, L.attn_b)
            q, k, v = qkv.split(H, dim=1)
            kc, vc = self.cache.layer(li)
            ops.kv_write(k.contiguous(), v.contiguous(), kc, vc, plan.slots)
            att = ops.paged_attention(q.contiguous(), kc, vc, table, plan.q_seq, plan.q_ctx, self.nh, self.nkv,
                                      self.scale, max_ctx=plan.max_ctx)
            h = h + F.linear(att, L.proj_w, L.proj_b)
            m = F.layer_norm(h, (H,), L.ln2_w, L.ln2_b, cfg.layer_norm_eps)
            m = F.gelu(F.linear(m, L.fc_w, L.fc_b), approximate="tanh")
            h = h + F.linear(m, L.fc2_w, L.fc2_b)
        if not self.is_last:
            return h
        hl = h.index_select(0, plan.last_rows.long())
        hl = F.layer_norm(hl, (H,), w.final_norm, w.final_norm_b, cfg.layer_norm_eps)
        return F.linear(hl, w.lm_head)

    # ------------------------------------------------------------------ hipGraph decode
    def _bucket(self, b: int) -> int:
        for cand in (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 192, 256):
            if b <= cand:
                return min(cand, self.graph_max_batch)
        return b

    def _ctx_bucket(self, c: int) -> int:
        c = max(c, 256)
        return 1 << (c - 1).bit_length()

    def _graph_key(self, T: int, max_ctx: int, hooked: bool, slot: int = 0, tag: int = 0) -> tuple:
        """(batch bucket, attention part size, parts, qkv fold, hooked, owner tag, input slot).  Slot 0
        (tag 0) is the graph every caller replays; slots 1 / 2 are an owner's two receive graphs
        (``graph_input``)."""
        B = self._bucket(T)
        ctxb = min(self._ctx_bucket(max_ctx), self._ctx_bucket(self.max_seq_len))
        part = ops.attention_partition(B, self.nkv, ctxb, min_part=self._attn_min_part)
        return (B, part[0], part[1], self._qkv_fold(B), bool(hooked), int(tag), int(slot))

    def _graph(self, key: tuple) -> "_DecodeGraph":
        g = self._graphs.get(key)
        if g is None:
            if self._graph_pool is None:
                self._graph_pool = torch.cuda.graph_pool_handle()
            g = _DecodeGraph(self, key[0], (key[1], key[2]), self._graph_pool, hook=self.graph_hook if key[4] else None)
            self._graphs[key] = g
        return g

    def _run_graph(self, plan: Plan, x: torch.Tensor, hooked: bool = False, owner=None) -> torch.Tensor:
        key = self._graph_key(plan.T, plan.max_ctx, hooked)
        read = None  # a receive graph whose static input this replay reads without being that graph
        tag = self._tag_of(owner)
        pin = self._recv_pin.pop(tag, None) if tag is not None else None
        if pin is not None:
            pkey, pg = pin
            if pkey[:5] == key[:5] and self._graphs.get(pkey) is pg:
                key = pkey  # the receive graph whose static input the hop landed in
            else:  # (step shape changed, or the graph was dropped meanwhile): copied from its input
                read = pg
        g = self._graph(key)
        out = g.replay(plan, x)
        g.mark_replayed()
        if read is not None:  # the next receive into that buffer must wait for this replay's copy
            read.done_ev = g.done_ev
        return out

    def graph_input(self, T: int, max_ctx: int, owner=None):
        """Receive target of a stage hop (``PipelineServingEngine``): the static input of the decode
        graph the owner's NEXT step of ``T`` rows will replay, and the event after which that buffer
        is free (the end of its last replay), or None when that step runs eagerly.  The hidden
        states then land where the graph reads them: no receive slab, no copy.  Two receive graphs
        per (owner, bucket) alternate, so the hop of step k lands in one while step k - 1 still
        replays the other (a single buffer would serialise every receive behind the previous step's
        compute); other callers of the executor - other owners included - never replay them."""
        if self.is_first or not (self.use_graphs and T <= self.graph_max_batch) or owner is None:
            return None
        with self.exec_lock:
            tag = self._tag_of(owner)
            if tag is None:
                tag = self._next_tag
                self._next_tag += 1
                try:
                    self._owner_tags[owner] = tag
                except TypeError:  # an owner without weak references: kept alive until release_owner
                    self._owner_strong[id(owner)] = (owner, tag)
            hooked = self.graph_hook is not None and owner is self._hook_owner
            base = self._graph_key(T, max_ctx, hooked)
            sk = (tag,) + base[:5]
            slot = 3 - self._recv_slot.get(sk, 2)  # 1, 2, 1, ...
            self._recv_slot[sk] = slot
            key = base[:5] + (tag, slot)
            g = self._graph(key)
            self._recv_pin[tag] = (key, g)
            return g.x, g.done_ev

    def _tag_of(self, owner) -> Optional[int]:
        if owner is None:
            return None
        try:
            return self._owner_tags.get(owner)
        except TypeError:
            got = self._owner_strong.get(id(owner))
            return got[1] if got is not None and got[0] is owner else None

    def release_owner(self, owner) -> None:
        """Drop ``owner``'s receive graphs and pins (its engine stopped or failed)."""
        with self.exec_lock:
            tag = self._tag_of(owner)
            if tag is None:
                return
            try:
                self._owner_tags.pop(owner, None)
            except TypeError:
                self._owner_strong.pop(id(owner), None)
            self._recv_pin.pop(tag, None)
            for k in [k for k in self._recv_slot if k[0] == tag]:
                del self._recv_slot[k]
            for k in [k for k in self._graphs if k[5] == tag]:
                del self._graphs[k]

    def graph_rows(self, T: int, is_decode: bool) -> Optional[int]:
        """Rows of the static output a step of ``T`` tokens would replay into (its batch bucket),
        or None when the step runs eagerly (same rule as ``run``, no deep prompts)."""
        if self.use_graphs and is_decode and T <= self.graph_max_batch:
            return self._bucket(T)
        return None

    def graph_hook_free(self, owner=None) -> bool:
        """True when no other owner's graph hook is installed (``owner`` may hold it already)."""
        return self.graph_hook is None or self._hook_owner is owner

    def set_graph_hook(self, fn, owner=None) -> None:
        """Record ``fn(out)`` at the end of the decode graphs captured for ``owner`` (the engine
        whose stage hop it is).  Steps run with ``forward(..., hook_owner=owner)`` replay those
        graphs; every other caller (a second engine on a shared executor, TCP requests, the
        throughput probe) gets hook-free graphs of its own, so a recorded send can never be
        replayed on someone else's behalf.  One owner at a time: a different owner raises."""
        with self.exec_lock:
            if fn is not None and not self.graph_hook_free(owner):
                raise RuntimeError("this executor already records another engine's graph hop")
            self._drop_hooked()
            self.graph_hook = fn
            self._hook_owner = owner if fn is not None else None

    def clear_graph_hook(self, owner=None) -> None:
        """Remove ``owner``'s hook and the graphs that recorded it (no-op for a non-owner)."""
        with self.exec_lock:
            if self.graph_hook is not None and self._hook_owner is owner:
                self._drop_hooked()
                self.graph_hook = None
                self._hook_owner = None

    def _drop_hooked(self) -> None:
        for k in [k for k in self._graphs if k[4]]:
            del self._graphs[k]

    def clear_graphs(self):
        self._graphs.clear()


class _DecodeGraph:
    """A captured decode step for a fixed (batch bucket, attention partition).

    Its metadata lives in ONE device blob (positions, slots | q_seq, q_ctx, last_rows) that a
    replay refills with a single host-to-device copy from a double-buffered pinned staging
    blob, padded for the bucket (padding rows: slot -1, context 0): round 1 issued six small
    copies / fills per step (profiles/r2_decode_step_*.txt)."""

    def __init__(self, ex: StageExecutor, B: int, part: Tuple[int, int], pool, hook=None):
        self.ex, self.B, self.part = ex, B, part
        dev, H, dt = ex.device, ex.cfg.hidden_size, ex.dtype
        if ex.is_first:
            self.x = torch.zeros(B, dtype=torch.long, device=dev)
        else:
            self.x = torch.zeros(B, H, dtype=dt, device=dev)
        nbytes = 16 * B + 12 * B  # int64 [2, B] + int32 [3 B]
        self.blob = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        self.meta64 = self.blob[: 16 * B].view(torch.int64).view(2, B)
        self.meta32 = self.blob[16 * B:].view(torch.int32)
        self._stage = [torch.zeros(nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        self._stage_ev = [None, None]
        self._k = 0
        host = self._stage[0].numpy()
        h64 = host[: 16 * B].view(np.int64).reshape(2, B)
        h32 = host[16 * B:].view(np.int32)
        h64[0] = 0
        h64[1] = -1
        h32[:] = 0
        h32[2 * B:] = np.arange(B, dtype=np.int32)
        self.blob.copy_(self._stage[0])
        self._stage[1].copy_(self._stage[0])
        if ex.gqa_decode_mfma:
            ex.decode_qblocks(B)  # allocated outside the capture
        self.bufs: dict = {}
        self.done_ev = None  # end of the last replay on the compute stream (graph_input)
        args = (self.x, self.meta64[0], self.meta64[1], self.meta32[:B], self.meta32[B:2 * B], self.meta32[2 * B:], B,
                0, part)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # warm up (allocator, hipBLASLt heuristics) outside capture
                ex._forward_llama(*args, decode=True)
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        # thread-local capture: another thread's stream work (a channel receive posted outside the
        # executor lock) neither breaks this capture nor fails because of it
        with torch.cuda.graph(self.graph, pool=pool, capture_error_mode="thread_local"):
            self.out = ex._forward_llama(*args, decode=True)
            if hook is not None:  # recorded only: the warm-up runs above never call it
                hook(self.out)
        self.mark_replayed()  # the warm-up runs read ``x``: a receive into it waits for them

    def replay(self, plan: Plan, x: torch.Tensor) -> torch.Tensor:
        b, B = plan.T, self.B
        self._k ^= 1
        k = self._k
        if self._stage_ev[k] is not None:
            self._stage_ev[k].synchronize()  # the copy issued two replays ago
        host = self._stage[k].numpy()
        h64 = host[: 16 * B].view(np.int64).reshape(2, B)
        h32 = host[16 * B:].view(np.int32)
        h64[:, :b] = plan.h64
        h64[0, b:] = 0
        h64[1, b:] = -1
        h32[:b] = plan.h32[:b]
        h32[b:B] = 0
        h32[B:B + b] = plan.h32[b:2 * b]
        h32[B + b:2 * B] = 0
        self.blob.copy_(self._stage[k], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._stage_ev[k] = ev
        if self.ex.is_first:
            self.x[:b].copy_(x.view(-1))
        elif x.data_ptr() != self.x.data_ptr():  # (a hop received into the static input: no copy)
            self.x[:b].copy_(x)
        self.graph.replay()
        return self.out[:b]

    def mark_replayed(self) -> None:
        ev = torch.cuda.Event()
        ev.record()
        self.done_ev = ev
