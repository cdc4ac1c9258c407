"""Stage construction API (``load_stage_model`` / ``Stage0`` / ``StageSegment`` / ``StageLast``).

Reference: src/llama_partition.py:76-550.  There, ``load_stage_model`` loads the full HF
model on CPU and prunes it to the role's layers; ``Stage0`` / ``StageSegment`` /
``StageLast`` are nn.Modules whose ``forward(x, position_ids, attention_mask,
past_key_values, use_cache)`` returns ``(out, present)`` with a tuple-of-(k, v) cache that
the caller threads through.

Here a stage is a ``StageExecutor`` (resident weights, paged KV cache, HIP kernels), so
the KV cache lives server-side in pages and the "past" a caller threads through is a
``SessionHandle``.  The wrappers keep the reference call shape so code written against
it keeps working:

    full = load_stage_model("llama2-7b", dev, role="stage0", end=8)
    s0 = Stage0(full, 8)
    hidden, past = s0(input_ids, position_ids, None, None, use_cache=True)   # prefill
    hidden, past = s0(next_ids, pos, None, past, use_cache=True)             # decode

``role`` is one of stage0 / segment / last (plus "full" = every block + embeddings + head).
``use_cpu_offload`` keeps weights in host memory until the first forward (opt-in; the
reference streams every layer over PCIe on every token by default).
"""
from __future__ import annotations

import dataclasses
import logging
import uuid
from typing import Optional

import torch

from .models.config import ModelConfig, resolve_model
from .models.weights import StageWeights, build_stage_weights
from .runtime.executor import StageExecutor

logger = logging.getLogger(__name__)

_DTYPES = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32,
           torch.float16: torch.float16, torch.bfloat16: torch.bfloat16, torch.float32: torch.float32}


@dataclasses.dataclass
class SessionHandle:
    """Opaque "past_key_values": the session whose KV pages hold this sequence's cache."""
    session_id: str
    length: int


@dataclasses.dataclass
class LoadedStage:
    cfg: ModelConfig
    weights: StageWeights
    role: str
    start: int
    end: int
    device: torch.device
    dtype: torch.dtype
    model_name: str
    executor_kwargs: dict
    use_cpu_offload: bool = False

    @property
    def config(self):
        return self.cfg


def resolve_dtype(dtype, device) -> torch.dtype:
    dt = _DTYPES.get(dtype, dtype)
    if torch.device(device).type == "cuda" and dt == torch.float16:
        logger.info("fp16 requested on MI355X: the HIP kernels are bf16 (same width, fp32 range); using bf16")
        dt = torch.bfloat16
    elif torch.device(device).type == "cpu" and dt == torch.float16:
        dt = torch.float32  # CPU path: fp16 GEMMs are slow and lossy on host (reference quirk)
    return dt


def load_stage_model(model_name: str, device, role: str, *, start: int = 0, end: Optional[int] = None,
                     dtype=torch.bfloat16, use_cpu_offload: bool = False, seed: int = 0,
                     **executor_kwargs) -> LoadedStage:
    """Load ONLY the role's blocks (+ embeddings for stage0, norm/head for last)."""
    cfg = resolve_model(model_name)
    L = cfg.num_hidden_layers
    if role == "stage0":
        s, e = 0, end
    elif role == "segment":
        s, e = start, end
    elif role == "last":
        s, e = start, L if end is None else end
    elif role == "full":
        s, e = 0, L
    else:
        raise ValueError(f"Unknown role: {role}")
    if e is None or s is None:
        raise ValueError(f"role={role} needs start/end")
    if not (0 <= s < e <= L):
        raise ValueError(f"Pruned model has 0 layers for role={role} (start={start}, end={end}). Check --splits.")
    device = torch.device(device)
    dt = resolve_dtype(dtype, device)
    load_dev = torch.device("cpu") if use_cpu_offload else device
    w = build_stage_weights(cfg, model_name, s, e, has_embed=role in ("stage0", "full"),
                            has_head=role in ("last", "full"), device=load_dev, dtype=dt, seed=seed)
    logger.info(f"load_stage_model: role={role}, layers={e - s}, start={s}, end={e}")
    return LoadedStage(cfg, w, role, s, e, device, dt, model_name, executor_kwargs, bool(use_cpu_offload))


def _to_device(w: StageWeights, device) -> StageWeights:
    for lay in w.layers:
        for f in dataclasses.fields(lay):
            t = getattr(lay, f.name)
            if isinstance(t, torch.Tensor):
                setattr(lay, f.name, t.to(device))
    for name in ("embed", "pos_embed", "final_norm", "final_norm_b", "lm_head", "lm_head_p"):
        t = getattr(w, name)
        if t is not None:
            setattr(w, name, t.to(device))
    return w


class _StageModule(torch.nn.Module):
    """Shared body of Stage0 / StageSegment / StageLast.

    The span arguments of the reference constructors are checked against the loaded span
    (a mismatch raises instead of silently serving other blocks).  ``gpu_device`` places the
    executor (default: the device ``load_stage_model`` was given).  ``keep_layers_on_gpu``
    applies to a stage loaded with ``use_cpu_offload``: the first ``n - keep`` blocks stream
    from pinned host memory each forward, the last ``keep`` stay resident (reference
    src/llama_partition.py:169-180, :290-293); without offload every block is resident."""
    role = "segment"

    def __init__(self, full: LoadedStage, *, start: Optional[int] = None, end: Optional[int] = None,
                 gpu_device=None, keep_layers_on_gpu: int = 0, **kw):
        super().__init__()
        if start is not None and int(start) != full.start:
            raise ValueError(f"{type(self).__name__}: start={start} but the loaded span starts at {full.start}")
        if end is not None and int(end) != full.end:
            raise ValueError(f"{type(self).__name__}: end={end} but the loaded span ends at {full.end}")
        n = full.end - full.start
        if not 0 <= int(keep_layers_on_gpu) <= n:
            raise ValueError(f"keep_layers_on_gpu={keep_layers_on_gpu} outside [0, {n}] for a {n}-block span")
        self.full = full
        self.config = full.cfg
        device = torch.device(gpu_device) if gpu_device is not None else full.device
        offload = full.use_cpu_offload and device.type == "cuda"
        w = full.weights
        if not offload and next(iter(w.tensors())).device != device:
            w = _to_device(w, device)
        ekw = dict(full.executor_kwargs)
        ekw.update(kw)
        if offload:
            ekw.update(offload=True, keep_layers_on_gpu=int(keep_layers_on_gpu))
        self.executor = StageExecutor(full.cfg, w, device, dtype=full.dtype, **ekw)

    @property
    def device(self):
        return self.executor.device

    def forward(self, x, position_ids=None, attention_mask=None, past_key_values=None, use_cache=True):
        """x: ids [1, T] (stage0) or hidden [1, T, H]; returns (out, SessionHandle)."""
        if past_key_values is None:
            past = SessionHandle(uuid.uuid4().hex, 0)
            reset = True
        else:
            past = past_key_values
            reset = False
        T = x.shape[-1] if self.executor.is_first else x.shape[-2]
        start = int(position_ids.reshape(-1)[0]) if position_ids is not None else past.length
        flat = x.reshape(-1) if self.executor.is_first else x.reshape(-1, x.shape[-1])
        out = self.executor.forward([(past.session_id, T)], flat, reset=[reset], starts=[start])
        past = SessionHandle(past.session_id, start + T)
        if self.executor.is_last:
            return out.unsqueeze(1), past  # [1, 1, V]: logits of the last position
        return out.unsqueeze(0), past

    def release(self, past: Optional[SessionHandle]):
        if past is not None:
            self.executor.sessions.close(past.session_id)


class Stage0(_StageModule):
    role = "stage0"

    def __init__(self, full: LoadedStage, end: Optional[int] = None, **kw):
        super().__init__(full, start=0, end=end, **kw)


class StageSegment(_StageModule):
    role = "segment"

    def __init__(self, full: LoadedStage, start: Optional[int] = None, end: Optional[int] = None, gpu_device=None,
                 keep_layers_on_gpu: int = 0, **kw):
        super().__init__(full, start=start, end=end, gpu_device=gpu_device, keep_layers_on_gpu=keep_layers_on_gpu,
                         **kw)


class StageLast(_StageModule):
    role = "last"

    def __init__(self, full: LoadedStage, start: Optional[int] = None, gpu_device=None, keep_layers_on_gpu: int = 0,
                 **kw):
        super().__init__(full, start=start, gpu_device=gpu_device, keep_layers_on_gpu=keep_layers_on_gpu, **kw)
