"""Tensor parallelism inside one pipeline stage (Megatron-style, RCCL all-reduce over xGMI).

The reference carries TP only as dead code (upstream Petals wraps blocks in the external
``tensor_parallel`` library: petals/server/backend.py:12-13,43,67-73,
petals/server/server.py:182-187,282-293).  Here a stage's blocks can be
sharded over ``tp`` ranks of one node, one process per GPU:

* column-parallel: ``qkv`` (rank r keeps q heads [r*nh/tp, (r+1)*nh/tp) and the matching
  k / v heads), ``gate_up`` (rows of the interleaved gate/up pair for an F/tp slice, so the
  fused SwiGLU epilogue is unchanged); every MoE expert is sharded the same way;
* row-parallel: ``o`` and ``down`` keep the matching input-column slice; their [T, H]
  partial sums are all-reduced (one RCCL all-reduce after attention and one after the MLP
  per block);
* norms, embeddings, router and ``lm_head`` are replicated; the KV cache holds only the
  rank's kv heads, so each GPU stores 1/tp of the session KV.

The executor runs unchanged on a *shard config* (nh/tp, nkv/tp, F/tp heads and widths):
attention, RoPE and the paged KV see fewer heads, the GEMMs see narrower weights.  On
xGMI a decode step's all-reduces carry 2 * n_layers * T * H * 2 bytes (64 sessions, 7B:
32 KiB per all-reduce) - latency-, not bandwidth-bound - which is why pipeline
replicas stay the default for throughput and TP is for fitting / per-token latency.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..models.config import ModelConfig
from ..models.weights import LlamaLayer, StageWeights, interleave_gate_up, split_gate_up


def check_tp(cfg: ModelConfig, tp: int) -> None:
    if cfg.model_type == "gpt2":
        raise ValueError("tensor parallelism supports the LLaMA-family (llama/mistral/mixtral) blocks only")
    for name, v in (("num_attention_heads", cfg.num_attention_heads), ("num_key_value_heads", cfg.num_key_value_heads)):
        if v % tp:
            raise ValueError(f"{name}={v} is not divisible by tp={tp}")
    if cfg.intermediate_size % (16 * tp):
        raise ValueError(f"intermediate_size={cfg.intermediate_size} must be a multiple of 16*tp={16 * tp}")


def shard_config(cfg: ModelConfig, tp: int) -> ModelConfig:
    """Per-rank view of ``cfg``: 1/tp of the attention heads and of the MLP width."""
    check_tp(cfg, tp)
    if tp == 1:
        return cfg
    return dataclasses.replace(cfg, num_attention_heads=cfg.num_attention_heads // tp,
                               num_key_value_heads=cfg.num_key_value_heads // tp,
                               intermediate_size=cfg.intermediate_size // tp)


def _shard_gate_up(gu: torch.Tensor, r: int, tp: int) -> torch.Tensor:
    g, u = split_gate_up(gu)
    f = g.shape[0] // tp
    return interleave_gate_up(g[r * f:(r + 1) * f].contiguous(), u[r * f:(r + 1) * f].contiguous()).contiguous()


def _shard_layer(L: LlamaLayer, cfg: ModelConfig, r: int, tp: int) -> LlamaLayer:
    if L.fp8 and L.qkv is None:
        raise ValueError("shard bf16 weights before fp8 quantization")
    D, nh, nkv = cfg.head_dim, cfg.num_attention_heads, cfg.num_key_value_heads
    qh, kh = nh // tp * D, nkv // tp * D
    q = L.qkv[: nh * D][r * qh:(r + 1) * qh]
    k = L.qkv[nh * D: (nh + nkv) * D][r * kh:(r + 1) * kh]
    v = L.qkv[(nh + nkv) * D:][r * kh:(r + 1) * kh]
    qkv = torch.cat([q, k, v], 0).contiguous()
    o = L.o[:, r * qh:(r + 1) * qh].contiguous()
    f = cfg.intermediate_size // tp
    if L.moe:
        gu = torch.stack([_shard_gate_up(L.gate_up[e], r, tp) for e in range(L.gate_up.shape[0])])
        dn = L.down[:, :, r * f:(r + 1) * f].contiguous()
    else:
        gu = _shard_gate_up(L.gate_up, r, tp)
        dn = L.down[:, r * f:(r + 1) * f].contiguous()
    return LlamaLayer(L.input_norm, qkv, o, L.post_norm, gu, dn, router=L.router)


def shard_stage_weights(sw: StageWeights, rank: int, tp: int) -> StageWeights:
    """Rank ``rank``'s shard of a stage (replicated embed / norms / head).  ``sw.cfg`` is the
    full config; the result carries the shard config."""
    if tp == 1:
        return sw
    scfg = shard_config(sw.cfg, tp)
    layers = [_shard_layer(L, sw.cfg, rank, tp) for L in sw.layers]
    return dataclasses.replace(sw, cfg=scfg, layers=layers, lm_head_p=None)


class TPGroup:
    """The all-reduce a sharded stage issues after its row-parallel GEMMs.

    With ``comm`` (a direct ``parallel.rccl.RcclComm`` over the group's GPUs) the all-reduce is
    enqueued on the current stream, so the executor captures it inside its decode hipGraphs
    (``capturable``); otherwise it is torch's all-reduce on ``group`` (gloo on CPU, or RCCL
    through ProcessGroupNCCL, which a graph cannot replay).  ``force``: treat a one-rank group
    as a TP group (issue the collectives anyway) - the 1-GPU test of the captured RCCL path."""

    def __init__(self, group: Optional["dist.ProcessGroup"] = None, comm=None, force: bool = False):
        self.group = group
        self.comm = comm
        if comm is not None:
            self.size, self.rank = comm.world, comm.rank
        else:
            self.size = dist.get_world_size(group) if dist.is_initialized() else 1
            self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.force = bool(force)

    @property
    def active(self) -> bool:
        return self.size > 1 or self.force

    @property
    def capturable(self) -> bool:
        return self.comm is not None

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.comm is not None and t.is_cuda:
            self.comm.all_reduce(t)
        elif self.size > 1:
            dist.all_reduce(t, group=self.group)
        return t

    def close(self) -> None:
        if self.comm is not None:
            self.comm.close()


def make_tp_groups(world: int, stages: int, tp: int, device=None) -> Optional[TPGroup]:
    """TP groups for a (replica x tp-lane x stage) rank layout: rank = lane * stages + stage,
    lane = replica * tp + t.  Each lane is a full pipeline (its own send/recv chain, fed the
    identical hidden states); the ranks holding the same stage in the tp lanes of one replica
    form a TP group.  Every rank must call this (groups are created in the same order).

    On GPU (``device`` a cuda device) each group also gets a direct RCCL communicator
    (``MPAMD_TP_RCCL=0``: torch's all-reduce only), so TP decode steps run as hipGraphs."""
    if tp <= 1 or not dist.is_initialized():
        return None
    lanes = world // stages
    if world % stages or lanes % tp:
        raise ValueError(f"world {world} does not factor into stages={stages} x tp={tp} x replicas")
    rank, mine, mine_ranks = dist.get_rank(), None, None
    for lane0 in range(0, lanes, tp):
        for st in range(stages):
            ranks = [(lane0 + j) * stages + st for j in range(tp)]
            g = dist.new_group(ranks)
            if rank in ranks:
                mine, mine_ranks = g, ranks
    comm = None
    # the direct RCCL communicator (graph-capturable all-reduces) stays opt-in (MPAMD_TP_RCCL=1) until a
    # tp2 run on two GPUs has matched the eager TP tokens; if its init fails (e.g. several TP ranks on
    # one GPU) the group keeps torch's ProcessGroupNCCL and eager steps
    if device is not None and torch.device(device).type == "cuda" and os.environ.get("MPAMD_TP_RCCL", "0") == "1":
        from . import rccl
        from torch.distributed import distributed_c10d as c10d

        try:
            store = c10d._get_default_store()
            comm = rccl.RcclComm(store, "tp/" + "_".join(map(str, mine_ranks)), mine_ranks.index(rank), tp, device)
        except Exception as e:  # noqa: BLE001
            import logging

            logging.getLogger(__name__).warning(f"TP RCCL communicator unavailable ({e}): eager ProcessGroupNCCL")
            comm = None
    return TPGroup(mine, comm=comm)
