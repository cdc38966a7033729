"""Collective helpers that work for every (backend, device) pair the harness uses.

* ``nccl`` (RCCL on ROCm) with GPU tensors: the collective runs on the device.
* ``gloo`` with GPU tensors (CPU-side control groups, one-GPU multi-process
  tests): staged through host memory.
* ``gloo`` with CPU tensors: direct.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _backend(group) -> str:
    return dist.get_backend(group)


def _comm_tensor(t: torch.Tensor, group) -> torch.Tensor:
    """The tensor the backend can run the collective on (a staged copy if needed)."""
    b = _backend(group)
    if t.is_cuda and b == "gloo":
        return t.detach().cpu()
    if not t.is_cuda and b == "nccl":
        return t.detach().to(torch.device("cuda", torch.cuda.current_device()))
    return t


def all_reduce_(t: torch.Tensor, group=None, op=dist.ReduceOp.SUM) -> torch.Tensor:
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return t
    c = _comm_tensor(t, group)
    dist.all_reduce(c, op=op, group=group)
    if c is not t:
        t.copy_(c)
    return t


def broadcast_(t: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return t
    c = _comm_tensor(t, group)
    dist.broadcast(c, src=src, group=group)
    if c is not t:
        t.copy_(c)
    return t


def barrier(group=None):
    if not dist.is_initialized():
        return
    if _backend(group) == "nccl" and torch.cuda.is_available():
        dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier(group=group)


def all_reduce_scalar(x: float, op=dist.ReduceOp.SUM, group=None) -> float:
    """Reduce one host float over the group (f64; a no-op without a process group)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    return float(all_reduce_(t, group, op=op).item())


def all_gather_scalar(x: float, group=None) -> list[float]:
    """Every rank's host float, in rank order (one SUM all-reduce of a one-hot f64 vector)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [float(x)]
    t = torch.zeros(dist.get_world_size(group), dtype=torch.float64)
    t[dist.get_rank(group)] = float(x)
    return [float(v) for v in all_reduce_(t, group).tolist()]
