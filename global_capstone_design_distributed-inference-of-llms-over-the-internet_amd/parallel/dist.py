"""torch.distributed bootstrap: one process per GPU, RCCL (backend "nccl") on MI355X, gloo on CPU."""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def init_distributed(device_type: Optional[str] = None, timeout_s: float = 600.0):
    """Initialise the default process group from torchrun-style env vars.

    Returns (rank, world, local_rank, device).  With WORLD_SIZE == 1 no group is created.
    """
    rank, world, local = env_rank_world()
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    # rehearsal of a multi-GPU layout on fewer GPUs (MPAMD_DIST_BACKEND=gloo, with
    # MPAMD_CHANNEL_DATA=gloo): ranks wrap around the visible devices; RCCL itself refuses two
    # ranks on one GPU, so such a run exercises everything but the RCCL transport
    backend_override = os.environ.get("MPAMD_DIST_BACKEND")
    if device_type == "cuda":
        idx = local % max(1, torch.cuda.device_count()) if backend_override == "gloo" else local
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        backend = backend_override or ("nccl" if device_type == "cuda" else "gloo")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if device_type == "cuda" and backend == "nccl":
            kw["device_id"] = device  # eager communicator init on this GPU
        dist.init_process_group(**kw)
    return rank, world, local, device


def barrier(device=None):
    if dist.is_initialized():
        if device is not None and torch.device(device).type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.device(device).index])
        else:
            dist.barrier()


def all_max(value: float, device) -> float:
    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_floats(values, device):
    if not dist.is_initialized():
        return [list(values)]
    t = torch.tensor(list(values), dtype=torch.float64, device=device if dist.get_backend() == "nccl" else "cpu")
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()
