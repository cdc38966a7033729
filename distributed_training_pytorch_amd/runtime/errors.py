"""Failure reporting, fault injection and debug checks.

* :func:`record` -- the equivalent of ``torch.distributed.elastic...errors.record``
  (``demo.py:14,156``): on an uncaught exception the worker writes the JSON error
  file torchrun's agent reads (``TORCHELASTIC_ERROR_FILE``) so the root-cause rank
  is reported, then re-raises.
* :class:`FaultInjector` -- ``--fail_at_iter N --fail_rank R`` kills one rank on the
  first attempt only (``TORCHELASTIC_RESTART_COUNT == 0``), so
  ``torchrun --max_restarts`` + checkpoint/resume can be exercised.
* :func:`check_replicas` -- the data-parallel "race detector": all ranks must hold
  bitwise identical parameters (a hash all-reduce).
"""
from __future__ import annotations

import functools
import json
import os
import socket
import sys
import time
import traceback

import torch
import torch.distributed as dist


def _error_payload(exc: BaseException) -> dict:
    return {
        "message": {
            "message": f"{type(exc).__name__}: {exc}",
            "extraInfo": {
                "py_callstack": "".join(traceback.format_exception(type(exc), exc, exc.__traceback__)),
                "timestamp": str(int(time.time())),
            },
        },
        "hostname": socket.gethostname(),
        "rank": os.environ.get("RANK"),
    }


def write_error_file(exc: BaseException, path: str | None = None) -> str | None:
    path = path or os.environ.get("TORCHELASTIC_ERROR_FILE")
    if not path:
        return None
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(_error_payload(exc), f)
    return path


def record(fn):
    """Decorator: write the torchelastic error file for any uncaught exception."""

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        try:
            return fn(*args, **kwargs)
        except SystemExit:
            raise
        except BaseException as e:
            write_error_file(e)
            print(f"[rank {os.environ.get('RANK', '?')}] failed: {type(e).__name__}: {e}", file=sys.stderr,
                  flush=True)
            raise

    return wrapper


class InjectedFault(RuntimeError):
    pass


class FaultInjector:
    def __init__(self, fail_at_iter: int | None, fail_rank: int = 0, rank: int = 0):
        self.fail_at_iter = fail_at_iter
        self.fail_rank = fail_rank
        self.rank = rank
        self.restart = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))

    def armed(self) -> bool:
        return self.fail_at_iter is not None and self.fail_at_iter >= 0 and self.restart == 0 \
            and self.rank == self.fail_rank

    def check(self, iteration: int) -> None:
        if self.armed() and iteration >= self.fail_at_iter:
            raise InjectedFault(f"injected fault on rank {self.rank} at iteration {iteration}")


def param_digest(t: torch.Tensor) -> float:
    """Order-sensitive float64 digest of a parameter buffer."""
    x = t.detach().double().reshape(-1)
    w = torch.arange(1, x.numel() + 1, dtype=torch.float64, device=x.device)
    return float((x * w).sum().item())


def check_replicas(t: torch.Tensor, group=None) -> None:
    """Raise if data-parallel replicas diverged (exact: every rank must hold the same bits)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    from ..parallel import comm_util

    d = torch.tensor([param_digest(t)], dtype=torch.float64)
    lo, hi = d.clone(), d.clone()
    comm_util.all_reduce_(lo, group, dist.ReduceOp.MIN)
    comm_util.all_reduce_(hi, group, dist.ReduceOp.MAX)
    if lo.item() != hi.item():
        raise RuntimeError(f"data-parallel replicas diverged (param digest min {lo.item()!r} != max {hi.item()!r})")
