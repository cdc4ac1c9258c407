"""Paged KV cache resident in HBM, plus a page allocator with a byte budget.

Reference behaviour being replaced:
* ``src/rpc_handler.py:70,266`` keeps a per-session tuple of per-layer (k, v) tensors that
  grows by ``torch.cat`` every token (petals/llama/block.py:123-128) and is never evicted;
* the vendored Petals server sizes a cache budget (``attn_cache_tokens``,
  petals/server/server.py:204-209) and allocates handles through ``MemoryCache``
  (petals/server/memory_cache.py:26-225) with ``AllocationFailed`` on exhaustion.

Here every stage owns ONE pair of preallocated tensors per layer,
``k[l], v[l] : [num_pages, nkv, page_size, head_dim]`` (bf16), sized from the HBM left
after the weights (288 GB per MI355X), and sessions own lists of page ids.  Tokens are
written in place by the fused RoPE kernel; nothing is ever copied or concatenated.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch

from .. import native


class AllocationFailed(RuntimeError):
    """Raised when the page pool cannot satisfy a request (Petals' AllocationFailed)."""


class PageAllocator:
    """LIFO free list of page ids (C++ implementation when the native runtime is built)."""

    def __init__(self, num_pages: int):
        self.num_pages = int(num_pages)
        self._impl = native.make_page_allocator(self.num_pages)

    @property
    def free_pages(self) -> int:
        return self._impl.free_count()

    def alloc(self, n: int) -> List[int]:
        if n <= 0:
            return []
        got = self._impl.alloc(int(n))
        if got is None:
            raise AllocationFailed(f"KV cache exhausted: requested {n} pages, {self.free_pages} free")
        return list(got)

    def free(self, pages: List[int]) -> None:
        if pages:
            self._impl.free(list(pages))


class PagedKVCache:
    def __init__(self, num_layers: int, num_pages: int, num_kv_heads: int, head_dim: int, page_size: int = 64,
                 dtype=torch.bfloat16, device="cpu"):
        assert page_size & (page_size - 1) == 0, "page_size must be a power of two"
        self.num_layers = num_layers
        self.num_pages = num_pages
        self.nkv = num_kv_heads
        self.head_dim = head_dim
        self.page_size = page_size
        self.dtype = dtype
        self.device = torch.device(device)
        shape = (max(num_layers, 1), num_pages, num_kv_heads, page_size, head_dim)
        self.k = torch.zeros(shape, dtype=dtype, device=self.device)
        self.v = torch.zeros(shape, dtype=dtype, device=self.device)
        self.allocator = PageAllocator(num_pages)

    def layer(self, i: int):
        return self.k[i], self.v[i]

    def copy_pages(self, src: List[int], dst: List[int]) -> None:
        """Copy whole pages (every layer, K and V) src[i] -> dst[i] on the device."""
        si = torch.tensor(src, dtype=torch.long, device=self.device)
        di = torch.tensor(dst, dtype=torch.long, device=self.device)
        self.k.index_copy_(1, di, self.k.index_select(1, si))
        self.v.index_copy_(1, di, self.v.index_select(1, si))

    @property
    def bytes_per_page(self) -> int:
        return 2 * self.num_layers * self.nkv * self.page_size * self.head_dim * torch.tensor([], dtype=self.dtype).element_size()

    @property
    def nbytes(self) -> int:
        return self.bytes_per_page * self.num_pages

    @staticmethod
    def pages_for_bytes(budget_bytes: int, num_layers: int, nkv: int, head_dim: int, page_size: int,
                        elt_bytes: int = 2) -> int:
        per_page = 2 * max(num_layers, 1) * nkv * page_size * head_dim * elt_bytes
        return max(1, int(budget_bytes // per_page))

    @staticmethod
    def auto_budget_bytes(device, weights_bytes_reserved: int = 0, fraction: float = 0.9,
                          cap_bytes: Optional[int] = None) -> int:
        """Free HBM x fraction (after weights are resident); capped by ``cap_bytes``."""
        device = torch.device(device)
        if device.type == "cuda":
            free, _total = torch.cuda.mem_get_info(device)
            budget = int(free * fraction) - weights_bytes_reserved
        else:
            budget = 1 << 30
        if cap_bytes is not None:
            budget = min(budget, cap_bytes)
        return max(budget, 0)


def pages_needed(num_tokens: int, page_size: int) -> int:
    return int(math.ceil(num_tokens / page_size)) if num_tokens > 0 else 0
