"""``make_inference_graphed_callable``: the upstream Petals helper that turns a callable into a
hipGraph-replayed one (reference petals/llama/cuda_graphs.py:5-76), kept as public API.

The stage executor does not use it - it captures the WHOLE decode step per batch bucket
(``runtime/executor.py`` ``_DecodeGraph``) - but code written against the upstream surface (a
graphed RMSNorm / RoPE callable, as petals/llama/block.py:118-121, 210-213 build them) runs
unchanged.  Semantics:

* ``sample_args``: tensors (or other values, passed through) shaping the static input surface;
  the callable runs a few warm-up iterations on a side stream, then is captured once;
* a call copies each tensor argument into its static input unless it already IS that buffer
  (same data pointer), replays, and returns the static outputs detached - later calls overwrite
  them, as upstream;
* off the GPU (or with graphs disabled) the callable itself is returned.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch


def make_inference_graphed_callable(fn: Callable, sample_args: Sequence, warmup_iters: int = 3,
                                    pool=None) -> Callable:
    tensors = [a for a in sample_args if isinstance(a, torch.Tensor)]
    if not tensors or not tensors[0].is_cuda:
        return fn
    static = [a.clone() if isinstance(a, torch.Tensor) else a for a in sample_args]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.no_grad():
        for _ in range(warmup_iters):
            fn(*static)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(graph, pool=pool, capture_error_mode="thread_local"):
        out = fn(*static)
    single = isinstance(out, torch.Tensor)
    outs = (out,) if single else tuple(out)

    def graphed(*args):
        if len(args) != len(static):
            raise TypeError(f"graphed callable takes {len(static)} arguments, got {len(args)}")
        for dst, src in zip(static, args):
            if isinstance(dst, torch.Tensor):
                if src.shape != dst.shape or src.dtype != dst.dtype:
                    raise ValueError(f"argument {tuple(src.shape)} {src.dtype} does not match the captured "
                                     f"{tuple(dst.shape)} {dst.dtype}")
                if src.data_ptr() != dst.data_ptr():
                    dst.copy_(src)
        graph.replay()
        res = tuple(o.detach() for o in outs)
        return res[0] if single else res

    graphed.graph = graph
    graphed.static_inputs = static
    return graphed
