"""Tracing helpers: roctx ranges and device-synchronised phase timers.

The reference has no tracing at all (only the rank-0 tqdm bar,
``demo.py:91-92``).  Here:

* ``trace_range(name)`` pushes/pops a roctx range (``torch.cuda.nvtx`` is backed
  by roctx on ROCm builds) when ``DTP_TRACE=1``; ``rocprofv3 --marker-trace``
  then shows data / forward / backward / all-reduce / optimizer phases next to
  the kernels.  It is a no-op otherwise (no cost on timed runs).
* ``PhaseTimer`` accumulates host wall time per phase, optionally synchronising
  the device at phase boundaries (``DTP_TRACE_SYNC=1``) so the numbers are GPU
  time, and reports them as a dict (logged by the runner at the end of a run).
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict

import torch

_ENABLED = os.environ.get("DTP_TRACE", "0") == "1"
_SYNC = os.environ.get("DTP_TRACE_SYNC", "0") == "1"


def enabled() -> bool:
    return _ENABLED


def set_enabled(on: bool, sync: bool | None = None) -> None:
    global _ENABLED, _SYNC
    _ENABLED = bool(on)
    if sync is not None:
        _SYNC = bool(sync)


def _push(name: str) -> None:
    try:
        torch.cuda.nvtx.range_push(name)
    except Exception:  # pragma: no cover - builds without roctx/nvtx
        pass


def _pop() -> None:
    try:
        torch.cuda.nvtx.range_pop()
    except Exception:  # pragma: no cover
        pass


@contextlib.contextmanager
def trace_range(name: str):
    if not _ENABLED:
        yield
        return
    _push(name)
    try:
        yield
    finally:
        _pop()


class PhaseTimer:
    """``with timer.phase("fwd"): ...`` -> ``timer.summary()`` = {phase: seconds}."""

    def __init__(self, device: torch.device | None = None):
        self.device = device
        self.total: dict[str, float] = defaultdict(float)
        self.count: dict[str, int] = defaultdict(int)

    def _sync(self):
        if _SYNC and self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not _ENABLED:
            yield
            return
        self._sync()
        t = time.perf_counter()
        _push(name)
        try:
            yield
        finally:
            self._sync()
            _pop()
            self.total[name] += time.perf_counter() - t
            self.count[name] += 1

    def summary(self) -> dict:
        return {k: {"s": round(v, 6), "calls": self.count[k]} for k, v in self.total.items()}
