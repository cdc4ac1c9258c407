"""Block sizing helpers (upstream Petals server).

Reference: petals/server/block_utils.py:12-65 (``resolve_block_dtype``, ``get_block_size``
for memory/disk with quantization-aware bytes per parameter) and petals/server/server.py
(auto ``num_blocks`` = floor((GPU memory - autograd reserve) / (block bytes + KV-cache bytes
per block)), ``attn_cache_tokens`` default 16384 for GQA models, 4096 otherwise).

MI355X specifics: weights and KV are both resident in HBM (288 GB per GPU), there is no
autograd reserve in an inference-only server, and the quantized weight format is OCP fp8
(e4m3, 1 byte per parameter + per-channel scales) rather than bitsandbytes INT8/NF4.
"""
from __future__ import annotations

from typing import Optional

import torch

from .models.config import ModelConfig

# bytes per parameter of the stored weight format
_QUANT_BYTES = {None: None, "none": None, "fp8": 1.0, "int8": 1.0, "nf4": 4.25 / 8}
_DTYPE_BYTES = {torch.float32: 4, torch.float16: 2, torch.bfloat16: 2}


def resolve_block_dtype(cfg: ModelConfig, dtype) -> torch.dtype:
    """``"auto"`` -> the checkpoint's dtype when it is a 16/32-bit float, else bf16."""
    if dtype in (None, "auto"):
        td = getattr(cfg, "torch_dtype", None)
        if isinstance(td, str):
            td = getattr(torch, td, None)
        return td if td in _DTYPE_BYTES else torch.bfloat16
    if isinstance(dtype, str):
        return {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}.get(dtype, getattr(torch, dtype))
    return dtype


def get_block_size(cfg: ModelConfig, location: str = "memory", dtype=torch.bfloat16,
                   quant_type: Optional[str] = None) -> int:
    """Bytes of one decoder block's parameters (``location`` = "memory" or "disk").

    On disk the checkpoint dtype counts; in memory the quantized format does (fp8: 1 B per
    parameter for the projection matrices, norms stay 16-bit).
    """
    if location not in ("memory", "disk"):
        raise ValueError(f"location must be 'memory' or 'disk', got {location!r}")
    elt = _DTYPE_BYTES[resolve_block_dtype(cfg, dtype)]
    if location == "disk" or _QUANT_BYTES.get(quant_type) is None:
        return cfg.layer_param_bytes(elt)
    q = _QUANT_BYTES[quant_type]
    H = cfg.hidden_size
    norms = 2 * H * elt
    matrices = cfg.layer_param_bytes(1.0) - 2 * H  # parameter count of the projection matrices
    scales = (cfg.q_dim + 2 * cfg.kv_dim + H + 2 * cfg.intermediate_size + H) * 4  # per-channel fp32
    return int(matrices * q + norms + scales)


def default_attn_cache_tokens(cfg: ModelConfig) -> int:
    """Upstream default KV budget per block: 16384 tokens for GQA models, 4096 otherwise."""
    return 16384 if cfg.num_key_value_heads < cfg.num_attention_heads else 4096


def kv_cache_bytes_per_block(cfg: ModelConfig, tokens: Optional[int] = None, dtype=torch.bfloat16) -> int:
    tokens = default_attn_cache_tokens(cfg) if tokens is None else int(tokens)
    return tokens * cfg.kv_bytes_per_token_per_layer(_DTYPE_BYTES[resolve_block_dtype(cfg, dtype)])


def auto_num_blocks(cfg: ModelConfig, free_bytes: Optional[int] = None, dtype=torch.bfloat16,
                    quant_type: Optional[str] = None, attn_cache_tokens: Optional[int] = None,
                    reserve_bytes: int = 2 << 30, device=None, total_blocks: Optional[int] = None) -> int:
    """How many blocks this GPU can serve: floor((free - reserve) / (block + KV per block)).

    ``free_bytes`` defaults to the device's free memory (``torch.cuda.mem_get_info``); on a
    CPU host the caller must pass it.  The result is clamped to [1, total_blocks].
    """
    if free_bytes is None:
        if device is None or torch.device(device).type != "cuda":
            raise ValueError("free_bytes is required off-GPU")
        free_bytes = torch.cuda.mem_get_info(torch.device(device))[0]
    per_block = get_block_size(cfg, "memory", dtype, quant_type) + kv_cache_bytes_per_block(cfg, attn_cache_tokens,
                                                                                           dtype)
    n = int((int(free_bytes) - int(reserve_bytes)) // per_block)
    total = cfg.num_hidden_layers if total_blocks is None else int(total_blocks)
    return max(1, min(n, total))
