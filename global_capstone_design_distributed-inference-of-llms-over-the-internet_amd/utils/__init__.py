"""Small helpers kept for API parity with the reference's ``src/utils.py``.

Reference: ``default_position_ids`` (src/utils.py:5-37), ``normalize_cache``
(:40-48), ``extract_kv_tuple`` (:51-64).  With server-side paged KV the "cache" a caller
holds is a ``SessionHandle``; legacy tuple caches are still understood for length queries.
"""
from __future__ import annotations

import logging
import os
from typing import Any, Optional

import torch


def past_length(past: Any) -> int:
    if past is None:
        return 0
    if hasattr(past, "length"):
        return int(past.length)
    if hasattr(past, "get_seq_length"):
        try:
            return int(past.get_seq_length())
        except Exception:
            return 0
    if isinstance(past, (list, tuple)) and past:
        first = past[0]
        if isinstance(first, (list, tuple)) and first and first[0] is not None:
            return int(first[0].shape[-2])
    return 0


def default_position_ids(layer_past: Any, seq_len: int, device=None) -> torch.Tensor:
    start = past_length(layer_past)
    return torch.arange(start, start + seq_len, device=device, dtype=torch.long).unsqueeze(0)


def normalize_cache(past: Any) -> Any:
    """HF Cache objects -> legacy tuples; session handles pass through unchanged."""
    if past is not None and hasattr(past, "to_legacy_cache"):
        try:
            return past.to_legacy_cache()
        except Exception:
            return past
    return past


def extract_kv_tuple(past: Any, layer: int = 0):
    past = normalize_cache(past)
    if isinstance(past, (list, tuple)) and len(past) > layer:
        return past[layer]
    return None


def setup_logging(level: Optional[str] = None) -> None:
    lvl = getattr(logging, (level or os.environ.get("MPAMD_LOG", "INFO")).upper(), logging.INFO)
    logging.basicConfig(level=lvl, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
