"""Opt-in CPU offload: layer weights live in pinned host memory and stream into HBM per step.

Reference: ``--use_cpu_offload`` / ``--keep_layers_on_gpu`` (StageSegment / StageLast,
src/llama_partition.py:140-297,300-474). Every forward, the reference:
* moves layer i to the GPU and layer i-1 back to the CPU, synchronously, on the compute stream;
* moves that layer's KV cache as well;
* and does all this even when offload is off.

Here offload is opt-in and stays off the compute stream's critical path:

* Only layer WEIGHTS stream. The paged KV cache stays resident in HBM.
* Host copies are pinned, so H2D runs as async DMA. Nothing is copied back: weights are
  read-only.
* ``n_slots`` device slots (default 2) form a ring. Layer i+n_slots is copied on a dedicated
  copy stream while layer i computes:
  * the copy of layer j waits on an event recorded when the layer that used its slot finished;
  * compute of layer j waits on the copy's event.
* Only the tensors the current path reads are streamed:
  * decode: packed projections (``*_p``) + norms;
  * prefill: row-major projections + norms.
* The last ``keep_layers_on_gpu`` layers are resident and never streamed (reference flag,
  same meaning).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Iterator, List, Sequence, Tuple

import torch


def _tensor_fields(layer) -> List[str]:
    return [f.name for f in dataclasses.fields(layer) if isinstance(getattr(layer, f.name), torch.Tensor)]


def pin_layer(layer):
    """Copy of ``layer`` with every tensor in pinned host memory."""
    kw = {}
    for name in _tensor_fields(layer):
        t = getattr(layer, name).detach()
        kw[name] = t.to("cpu").pin_memory() if torch.cuda.is_available() else t.to("cpu")
    return dataclasses.replace(layer, **kw)


class LayerStreamer:
    def __init__(self, host_layers: Sequence, device, n_slots: int = 2):
        self.host = list(host_layers)
        self.device = torch.device(device)
        self.n_slots = max(1, min(int(n_slots), max(len(self.host), 1)))
        self.stream = torch.cuda.Stream(self.device)
        self._slots: Dict[Tuple[str, ...], List] = {}
        self.bytes_streamed = 0

    def _slot(self, k: int, fields: Tuple[str, ...]):
        ring = self._slots.get(fields)
        if ring is None:
            ring = []
            proto = self.host[0]
            for _ in range(self.n_slots):
                kw = {name: None for name in _tensor_fields(proto)}
                for name in fields:
                    t = getattr(proto, name)
                    kw[name] = torch.empty(t.shape, dtype=t.dtype, device=self.device)
                ring.append(dataclasses.replace(proto, **kw))
            self._slots[fields] = ring
        return ring[k]

    def layers(self, fields: Sequence[str]) -> Iterator[Tuple[int, object]]:
        """Yield ``(index, device layer)``. The caller enqueues that layer's kernels on the current
        stream before advancing the iterator."""
        fields = tuple(f for f in fields if getattr(self.host[0], f, None) is not None) if self.host else ()
        n, S = len(self.host), self.n_slots
        compute = torch.cuda.current_stream(self.device)
        ready: List = [None] * n
        free: List = [None] * S

        def issue(j: int):
            slot = self._slot(j % S, fields)
            with torch.cuda.stream(self.stream):
                if free[j % S] is not None:
                    self.stream.wait_event(free[j % S])
                src = self.host[j]
                for name in fields:
                    s = getattr(src, name)
                    getattr(slot, name).copy_(s, non_blocking=True)
                    self.bytes_streamed += s.numel() * s.element_size()
                ev = torch.cuda.Event()
                ev.record(self.stream)
                ready[j] = ev

        # the previous step's kernels may still read the slots: the first copies wait for them
        start = torch.cuda.Event()
        start.record(compute)
        for k in range(S):
            free[k] = start
        for j in range(min(S, n)):
            issue(j)
        for i in range(n):
            compute.wait_event(ready[i])
            yield i, self._slot(i % S, fields)
            done = torch.cuda.Event()
            done.record(compute)
            free[i % S] = done
            if i + S < n:
                issue(i + S)
