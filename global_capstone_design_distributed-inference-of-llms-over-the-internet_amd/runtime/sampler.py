"""Batched server-side sampling (the last stage samples; only token ids leave it).

Reference: ``StageConnectionHandler._sample_token`` samples one row per request in
Python (reference src/rpc_handler.py:327-403) with defaults temperature 0.8 / top_p 0.9 /
top_k 0 in the handler (:71-73) and repetition penalty 1.5 (:164); the CLI sends
temperature 1.0 / top_p 0.92 / top_k 50 (src/main.py:806-809).  Here all rows of a step are
sampled by one HIP kernel launch with per-row parameters (``ops.sample``).
"""
from __future__ import annotations

import dataclasses
import hashlib
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import ops

RECENT = 50  # reference: generated_tokens[-50:] (src/rpc_handler.py:348; src/rpc_transport.py:797)


@dataclasses.dataclass
class SamplingParams:
    temperature: float = 0.8
    top_p: float = 0.9
    top_k: int = 0
    repetition_penalty: float = 1.5

    @classmethod
    def from_metadata(cls, md: dict) -> "SamplingParams":
        return cls(float(md.get("temperature", 0.8)), float(md.get("top_p", 0.9)), int(md.get("top_k", 0)),
                   float(md.get("repetition_penalty", 1.5)))


def session_seed(session_id: str, step: int, base_seed: int = 0) -> int:
    h = hashlib.blake2b(f"{base_seed}:{session_id}:{step}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") & 0x7FFFFFFFFFFFFFFF


class BatchSampler:
    def __init__(self, device, max_rows: int = 256):
        self.device = torch.device(device)
        self.max_rows = max_rows
        pin = self.device.type == "cuda"
        self._f = torch.empty(3, max_rows, dtype=torch.float32, pin_memory=pin)
        self._i = torch.empty(2 + RECENT, max_rows, dtype=torch.int32, pin_memory=pin)
        self._s = torch.empty(max_rows, dtype=torch.int64, pin_memory=pin)
        self._ws: Optional[torch.Tensor] = None

    def __call__(self, logits: torch.Tensor, params: Sequence[SamplingParams], histories: Sequence[Sequence[int]],
                 seeds: Sequence[int]) -> torch.Tensor:
        R, V = logits.shape
        assert R == len(params) == len(histories) == len(seeds)
        if R == 0:
            return torch.empty(0, dtype=torch.long, device=logits.device)
        if all(p.temperature <= 0 for p in params):
            return ops.argmax(logits)
        if R > self.max_rows:
            return torch.cat([self(logits[i:i + self.max_rows], params[i:i + self.max_rows],
                                   histories[i:i + self.max_rows], seeds[i:i + self.max_rows])
                              for i in range(0, R, self.max_rows)])
        f = self._f[:, :R].numpy()
        ii = self._i[:, :R].numpy()
        f[0] = [p.temperature for p in params]
        f[1] = [p.top_p for p in params]
        f[2] = [p.repetition_penalty for p in params]
        ii[0] = [p.top_k for p in params]
        rec = np.zeros((R, RECENT), dtype=np.int32)
        lens = np.zeros(R, dtype=np.int32)
        for r, h in enumerate(histories):
            h = list(h)[-RECENT:]
            lens[r] = len(h)
            if h:
                rec[r, : len(h)] = h
        ii[1] = lens
        self._s[:R].numpy()[:] = [int(s) & 0x7FFFFFFFFFFFFFFF for s in seeds]
        dev = logits.device
        fd = self._f[:, :R].to(dev, non_blocking=True)
        idv = self._i[:2, :R].to(dev, non_blocking=True)
        recent = torch.from_numpy(rec).to(dev, non_blocking=False)
        seeds_d = self._s[:R].to(dev, non_blocking=True)
        if dev.type == "cuda":
            if self._ws is None or self._ws.numel() < R * V:
                self._ws = torch.empty(self.max_rows * V, dtype=torch.float32, device=dev)
            ws = self._ws
        else:
            ws = None
        out = ops.sample(logits, fd[0].contiguous(), fd[1].contiguous(), idv[0].contiguous(), fd[2].contiguous(),
                         recent, idv[1].contiguous(), seeds_d, workspace=ws)
        if dev.type == "cuda":
            torch.cuda.current_stream().synchronize()  # pinned staging is reused by the next call
        return out
