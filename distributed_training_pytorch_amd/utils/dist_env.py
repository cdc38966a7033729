"""Process-group helpers shared by bench.py, the demos and the tests."""
from __future__ import annotations

import datetime
import os
import socket

import torch
import torch.distributed as dist


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def init_from_env(backend: str | None = None, timeout_s: int = 3600, single_rank_pg: bool = False):
    """Initialise torch.distributed from torchrun-style env vars.

    Returns (rank, world, local_rank).  With WORLD_SIZE unset and
    single_rank_pg=True a 1-rank group on 127.0.0.1 is created (so code paths
    that need a process group run unchanged on one GPU).
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if world > 1 or single_rank_pg:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if not dist.is_initialized():
            kw = {}
            if backend == "nccl" and torch.cuda.is_available():
                torch.cuda.set_device(local_rank)
                kw["device_id"] = torch.device("cuda", local_rank)
            dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world, local_rank


def barrier():
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def _scalar_device(device):
    # gloo reduces host tensors; RCCL device tensors
    return device if dist.get_backend() == "nccl" else torch.device("cpu")


def allreduce_max(x: float, device) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_scalar_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(x: float, device) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_scalar_device(device))
    dist.all_reduce(t)
    return float(t.item())
