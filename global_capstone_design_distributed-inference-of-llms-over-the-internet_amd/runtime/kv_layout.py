"""KV-cache export/import between the paged HBM cache and the dense layouts other servers use.

Reference:
* ``WrappedLlamaBlock._reorder_cache_from_bloom_to_llama`` / ``_from_llama_to_bloom``
  (petals/llama/block.py:306-326): the upstream Petals wire/cache layout is the BLOOM one,
  keys ``[B*kvh, hd, T]`` and values ``[B*kvh, T, hd]``, while LLaMA code wants ``[B, kvh, T, hd]``;
* the reference stage handler returns / replays legacy per-layer ``(k, v)`` tuples
  (src/rpc_handler.py:176-230,266, src/llama_partition.py:52-73).

Our cache is paged (``k[l] : [num_pages, kvh, page, hd]``, runtime/kv_cache.py), so these helpers
gather a session's pages into the dense LLaMA layout (one index_select per layer, on the device)
and scatter a dense cache back into freshly reserved pages. That makes a session portable
between servers (migration, debugging against HF ``past_key_values``) without the per-token
``torch.cat`` the reference pays.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

KV = Tuple[torch.Tensor, torch.Tensor]


def llama_to_bloom(k: torch.Tensor, v: torch.Tensor) -> KV:
    """``[B, kvh, T, hd]`` x2 -> keys ``[B*kvh, hd, T]``, values ``[B*kvh, T, hd]``."""
    b, h, t, d = k.shape
    return k.reshape(b * h, t, d).permute(0, 2, 1), v.reshape(b * h, t, d)


def bloom_to_llama(k: torch.Tensor, v: torch.Tensor, batch_size: int) -> KV:
    """Inverse of :func:`llama_to_bloom`."""
    bh, d, t = k.shape
    h = bh // batch_size
    return k.permute(0, 2, 1).reshape(batch_size, h, t, d), v.reshape(batch_size, h, t, d)


def _layer_ids(cache, layers: Optional[Sequence[int]]) -> List[int]:
    return list(range(cache.num_layers)) if layers is None else list(layers)


def export_session_kv(cache, session, layers: Optional[Sequence[int]] = None,
                      length: Optional[int] = None) -> List[KV]:
    """Dense per-layer ``(k, v)`` of one session, LLaMA layout ``[1, kvh, T, hd]``."""
    t = session.length if length is None else int(length)
    if t > session.length:
        raise ValueError(f"session holds {session.length} tokens, asked for {t}")
    ps = cache.page_size
    npg = -(-t // ps)
    idx = torch.tensor(session.pages[:npg], dtype=torch.long, device=cache.device)
    out = []
    for l in _layer_ids(cache, layers):
        kk = cache.k[l].index_select(0, idx)  # [P, kvh, ps, hd]
        vv = cache.v[l].index_select(0, idx)
        kk = kk.permute(1, 0, 2, 3).reshape(cache.nkv, npg * ps, cache.head_dim)[:, :t]
        vv = vv.permute(1, 0, 2, 3).reshape(cache.nkv, npg * ps, cache.head_dim)[:, :t]
        out.append((kk.unsqueeze(0).contiguous(), vv.unsqueeze(0).contiguous()))
    return out


def import_session_kv(sessions, sid: str, kv: Sequence[KV], max_length: Optional[int] = None):
    """Create (or reset) session ``sid`` and fill its pages from dense LLaMA-layout ``kv``.

    ``kv`` has one ``(k, v)`` per cache layer, each ``[1, kvh, T, hd]``. Returns the session.
    """
    cache = sessions.cache
    if len(kv) != cache.num_layers:
        raise ValueError(f"expected {cache.num_layers} layers, got {len(kv)}")
    t = kv[0][0].shape[2]
    s = sessions.get(sid)
    if s is None:
        s = sessions.open(sid, max_length)
    else:
        sessions.reset(sid)
    sessions.reserve(s, t)
    ps = cache.page_size
    npg = -(-t // ps)
    idx = torch.tensor(s.pages[:npg], dtype=torch.long, device=cache.device)
    for l, (k, v) in enumerate(kv):
        if k.shape != (1, cache.nkv, t, cache.head_dim) or v.shape != k.shape:
            raise ValueError(f"layer {l}: bad kv shape {tuple(k.shape)}")
        for src, dst in ((k, cache.k[l]), (v, cache.v[l])):
            pad = torch.zeros(cache.nkv, npg * ps, cache.head_dim, dtype=dst.dtype, device=dst.device)
            pad[:, :t] = src[0].to(device=dst.device, dtype=dst.dtype)
            dst.index_copy_(0, idx, pad.view(cache.nkv, npg, ps, cache.head_dim).permute(1, 0, 2, 3))
    s.length = t
    sessions.sync_table()
    return s
