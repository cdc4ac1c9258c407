"""Single-callable HIP-graph capture for inference (no backward graph).

Reference: ``make_inference_graphed_callable`` (petals/llama/cuda_graphs.py:5-76), used by the
reference decoder layer to graph its decode-time RMSNorm / RoPE pieces
(petals/llama/block.py:118-121,210-213,232-235).

The stage executor does not need this helper for its own hot path -- it captures the WHOLE
stage decode step (every layer, attention over the paged cache, sampling) per (batch bucket,
context bucket) in ``runtime/executor.py`` -- but it is part of the public surface for users
who want to graph an arbitrary tensor function (e.g. a custom head or a draft model).

Semantics kept from the reference:
* sample args are a (possibly nested) pytree of tensors; the flattened leaves become the static
  input surface;
* ``num_warmup_iters`` eager runs on a side stream before capture (lazy init stays out of the
  graph);
* on replay an argument whose storage differs from the captured one is copied into the
  static surface; the returned tensors are the static outputs, detached and re-nested.
"""
from __future__ import annotations

from typing import Callable

import torch
from torch.utils._pytree import tree_flatten, tree_unflatten


def make_inference_graphed_callable(fn: Callable, sample_args, num_warmup_iters: int = 3,
                                    pool=None) -> Callable:
    if isinstance(fn, torch.nn.Module):
        raise TypeError("pass a function (e.g. module.forward wrapped in a lambda), not an nn.Module")
    if torch.is_autocast_enabled() and torch.is_autocast_cache_enabled():
        raise RuntimeError("autocast weight caching is incompatible with graph capture; use cache_enabled=False")
    if not isinstance(sample_args, tuple):
        sample_args = (sample_args,)
    leaves, in_spec = tree_flatten(sample_args)
    if not all(isinstance(t, torch.Tensor) for t in leaves):
        raise TypeError("sample_args may contain only tensors")
    if not all(t.is_cuda for t in leaves):
        raise ValueError("graph capture needs device tensors")
    static_in = tuple(leaves)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side), torch.no_grad():
        for _ in range(num_warmup_iters):
            fn(*sample_args)
    torch.cuda.current_stream().wait_stream(side)

    graph = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(graph, pool=pool):
        out = fn(*sample_args)
    out_leaves, out_spec = tree_flatten(out)
    static_out = tuple(out_leaves)

    def graphed(*args):
        new, spec = tree_flatten(args)
        if spec != in_spec:
            raise ValueError("argument structure differs from the captured sample_args")
        for dst, src in zip(static_in, new):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
        graph.replay()
        return tree_unflatten([o.detach() for o in static_out], out_spec)

    graphed.graph = graph
    graphed.static_inputs = static_in
    graphed.static_outputs = static_out
    return graphed
