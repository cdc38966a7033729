"""CapturedStep: one whole training iteration replayed as a hipGraph.

MI355X-first replacement for a tracing compiler on launch-bound loops: the
iteration of an ``nn.Module`` engine (batch gather, forward kernels, loss,
autograd backward with its in-place gradient kernels and bucketed all-reduce,
the flat optimizer, the device loss ring) is captured ONCE with
``torch.cuda.graph`` (a hipGraph on ROCm) and then replayed: one host call per
iteration instead of ~25 kernel launches and the Python/autograd work between
them.  The reference runs that iteration eagerly (``demo.py:99-111``).

Rules the body must follow (the module engine's does):
* every tensor it reads or writes lives across replays (static inputs are
  refreshed by the caller before ``run``, e.g. the batch indices);
* device-side state only (step counters, loss-ring slot): no host syncs or
  host-side branching on device values;
* one graph per static shape: ``key`` selects it (the batch size, which shrinks on
  an epoch's last partial batch).

The first ``warmup`` iterations of each key run eagerly on a side stream (they
are real training iterations; they also settle allocator and library state), the
next one is captured and replayed, and every later one is a replay.  If capture
fails (e.g. a collective backend that cannot be captured), the key falls back to
eager for the rest of the run.
"""
from __future__ import annotations

from typing import Callable, Hashable

import torch


class CapturedStep:
    def __init__(self, body: Callable[[Hashable], None], device: torch.device, warmup: int = 2,
                 enabled: bool = True, on_abort: Callable[[], None] | None = None):
        self.body = body
        self.on_abort = on_abort  # resets host-side state a half-captured body left behind
        self.device = torch.device(device)
        self.warmup = max(1, int(warmup))
        self.enabled = enabled and self.device.type == "cuda"
        self._graphs: dict = {}
        self._seen: dict = {}
        self._pool = None
        self.replays = 0
        self.fallback_reason: str | None = None

    def run(self, key: Hashable = None, warm_key: Hashable = None) -> None:
        """Replay ``key``'s graph (capturing it first).  ``warm_key``: the eager warm-up
        runs are counted per ``warm_key`` instead (several graph copies of one body:
        the first copy's warm-up serves them all)."""
        g = self._graphs.get(key)
        if g is not None and g is not False:
            g.replay()
            self.replays += 1
            return
        if g is False or not self.enabled:
            self.body(key)
            return
        wk = key if warm_key is None else warm_key
        n = self._seen.get(wk, 0)
        cur = torch.cuda.current_stream(self.device)
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(cur)
        if n < self.warmup:
            with torch.cuda.stream(side):
                self.body(key)
            cur.wait_stream(side)
            self._seen[wk] = n + 1
            return
        graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(graph, stream=side, pool=self._pool):
                self.body(key)
        except Exception as e:  # capture unsupported for this body: eager from here on
            self._graphs[key] = False
            self.fallback_reason = f"{type(e).__name__}: {e}"
            cur.wait_stream(side)
            torch.cuda.synchronize(self.device)
            if self.on_abort is not None:
                self.on_abort()
            self.body(key)
            return
        cur.wait_stream(side)
        if self._pool is None:
            self._pool = graph.pool()  # graphs of every key share one memory pool
        self._graphs[key] = graph
        graph.replay()
        self.replays += 1

    def reset(self) -> None:
        """Drop every captured graph (the body's launch arguments changed, e.g. new
        optimizer hyperparameters); the next ``run`` of a key captures it again."""
        self._graphs.clear()
        self._seen = {k: self.warmup for k in self._seen}

    def is_captured(self, key: Hashable) -> bool:
        g = self._graphs.get(key)
        return g is not None and g is not False

    @property
    def captured(self) -> int:
        return sum(1 for g in self._graphs.values() if g is not None and g is not False)
