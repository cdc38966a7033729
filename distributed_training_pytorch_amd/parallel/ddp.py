"""FlatDDP: the DDP Reducer re-built around one flat gradient buffer.

Reference behaviour reproduced (torch DDP as used at ``demo.py:69-72``):
* construction broadcasts rank 0's parameters (one coalesced flat broadcast);
* gradients are averaged (sum all-reduce, then 1/W) and the all-reduce is
  launched from autograd hooks as soon as a bucket's gradients are final, so it
  overlaps the rest of the backward on RCCL's stream;
* the optimizer sees the averaged gradient after ``backward()`` returns.

MI355X-first choices:
* gradients live in a flat buffer (parameters' ``.grad`` are views of it), so a
  bucket is a contiguous slice -- no per-bucket copy-in/copy-out;
* buckets: the first (last-produced) bucket small to start communication early,
  the rest 25 MB (torch DDP's defaults; see the class comment for the sizing
  argument on 7 point-to-point xGMI links);
* ``comm="auto"|"xgmi"`` routes buckets of up to 64 Ki floats through the
  one-shot xGMI all-reduce (``parallel/xgmi.py: XgmiAllReduce``) on a side HIP
  stream (one posted write per peer + one local read instead of a 2(W-1)-hop
  ring), after a self-test against the process group; larger buckets, CPU/gloo
  runs, more than 8 ranks or a failed self-test use RCCL (``comm="rccl"``).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops.gemm import add_grad_ready_hook, mark_fused_grad
from . import comm_util


class FlatDDP(nn.Module):
    # bucket_cap_mb / first_bucket_mb: "auto" (default) measures the all-reduce of this
    # process group on this node at construction (parallel/bucket_tuning.py: latency
    # alpha and bandwidth beta fitted to a few probe sizes; cap = 9 alpha beta, first =
    # alpha beta) when there are several ranks and a gradient bigger than the smallest
    # probe; otherwise -- and for any explicit number -- torch DDP's defaults (25 MB,
    # 1 MiB first bucket, torch/nn/parallel/distributed.py).  Why measure: on one MI355X
    # node a ring all-reduce of n bytes over W ranks moves 2 (W-1)/W n per rank and pays
    # 2 (W-1) hop latencies, each hop ONE point-to-point xGMI link; the crossover between
    # latency and bytes is a property of the node and RCCL version, not a constant.
    # Buckets <= 64 Ki floats take the one-shot xGMI all-reduce instead (one posted write
    # per peer, one hop).  ``bucket_plan`` records what was chosen and from what.
    def __init__(self, module: nn.Module, group=None, bucket_cap_mb: float | str = "auto",
                 first_bucket_mb: float | str = "auto",
                 flat_params: torch.Tensor | None = None, flat_grad: torch.Tensor | None = None,
                 broadcast: bool = True, comm: str = "auto"):
        super().__init__()
        self.module = module
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if comm not in ("auto", "rccl", "xgmi"):
            raise ValueError(f"FlatDDP comm must be auto|rccl|xgmi, got {comm!r}")
        params = [p for p in module.parameters() if p.requires_grad]
        if flat_params is None or flat_grad is None:
            flat_params, flat_grad = self._flatten(params)
        self.flat_params = flat_params
        self.flat_grad = flat_grad
        self._grad1d = flat_grad.view(-1)  # bucket spans index the flat ELEMENT space
        self._params = params
        # offsets of every param inside the flat grad
        base = flat_grad.data_ptr()
        self._offset = {}
        for p in params:
            if p.grad is None or p.grad.data_ptr() < base or \
                    p.grad.data_ptr() + p.numel() * p.element_size() > base + flat_grad.numel() * flat_grad.element_size():
                raise ValueError("parameter grads must be views of flat_grad")
            self._offset[p] = (p.grad.data_ptr() - base) // p.element_size()
        bucket_cap_mb, first_bucket_mb = self._resolve_buckets(params, bucket_cap_mb, first_bucket_mb)
        # buckets in reverse registration order (~ the order backward produces grads)
        self._buckets = []
        cur, cur_bytes = [], 0
        cap = int(first_bucket_mb * 2 ** 20)
        for p in reversed(params):
            cur.append(p)
            cur_bytes += p.numel() * p.element_size()
            if cur_bytes >= cap:
                self._buckets.append(cur)
                cur, cur_bytes = [], 0
                cap = int(bucket_cap_mb * 2 ** 20)
        if cur:
            self._buckets.append(cur)
        self._bucket_of = {p: i for i, b in enumerate(self._buckets) for p in b}
        self._spans = []
        for b in self._buckets:
            lo = min(self._offset[p] for p in b)
            hi = max(self._offset[p] + p.numel() for p in b)
            self._spans.append((lo, hi))
        self._pending = [0] * len(self._buckets)
        self._reduced = [False] * len(self._buckets)
        self._ready: set = set()
        self._works = []
        self._callback_queued = False
        for p in params:
            p.register_post_accumulate_grad_hook(self._hook)
            add_grad_ready_hook(p, self._hook)  # grads the GEMM backward accumulates in place
        if broadcast and self.world > 1:
            comm_util.broadcast_(self.flat_params, 0, group)
        self.comm = "rccl"
        self._xgmi = None
        self._side = None
        self._xgmi_buckets: set[int] = set()
        if comm in ("auto", "xgmi"):
            self._setup_xgmi(strict=comm == "xgmi")

    # ------------------------------------------------------------------ xGMI path
    def _setup_xgmi(self, strict: bool):
        from .xgmi import XgmiAllReduce

        dev = self.flat_grad.device
        why = ""
        if self.world == 1:
            why = "single rank"
        elif dev.type != "cuda":
            why = "needs GPU gradients"
        elif self.world > 8:
            why = "more than one node's worth of ranks"
        small = [b for b, (lo, hi) in enumerate(self._spans) if hi - lo <= XgmiAllReduce.MAX_CAP]
        if not why and not small:
            why = "no bucket small enough"
        if not why:
            cap = max(self._spans[b][1] - self._spans[b][0] for b in small)
            rank = dist.get_rank(self.group)
            probe = torch.full((cap,), float(rank + 1), device=dev)
            probe[::7] = 0.5 * (rank + 1)
            expect = probe.clone()
            comm_util.all_reduce_(expect, self.group)  # before anything that can fail: same collectives on all ranks
            ok, ar = False, None
            try:
                ar = XgmiAllReduce(cap, dev, self.group)
                ar.all_reduce_(probe)
                torch.cuda.synchronize(dev)
                ok = torch.equal(probe, expect) and not bool(ar.status[0].item())
                why = "" if ok else "self-test mismatch"
            except Exception as e:  # noqa: BLE001 - any mapping failure -> RCCL
                why = f"setup failed: {e}"
            flag = torch.tensor([1.0 if ok else 0.0], device=dev)
            comm_util.all_reduce_(flag, self.group, op=dist.ReduceOp.MIN)  # every rank takes the same path
            if flag.item() == 1.0:
                self._xgmi, self._side, self.comm = ar, torch.cuda.Stream(dev), "xgmi"
                self._xgmi_buckets = set(small)
                return
            if ar is not None:
                ar.close()
            why = why or "self-test failed on another rank"
        if strict and self.world > 1:
            raise RuntimeError(f"FlatDDP comm='xgmi' unavailable: {why}")

    def _resolve_buckets(self, params, cap_mb, first_mb) -> tuple[float, float]:
        """Numbers as given; "auto": the measured plan (bucket_tuning.plan) with several
        ranks and a gradient larger than the smallest probe, else torch's defaults."""
        from . import bucket_tuning

        self.bucket_plan = {"source": "default", "first_bucket_mb": 1.0, "bucket_cap_mb": 25.0}
        if "auto" in (cap_mb, first_mb):
            total = sum(p.numel() * p.element_size() for p in params)
            if self.world > 1 and total > min(bucket_tuning.DEFAULT_SIZES):
                dev = self.flat_grad.device
                backend = dist.get_backend(self.group)
                self.bucket_plan = dict(bucket_tuning.plan(self.group,
                                                           dev if backend == "nccl" else torch.device("cpu")))
        else:
            self.bucket_plan = {"source": "explicit"}
        cap = self.bucket_plan["bucket_cap_mb"] if cap_mb == "auto" else float(cap_mb)
        first = self.bucket_plan["first_bucket_mb"] if first_mb == "auto" else float(first_mb)
        self.bucket_plan.update(bucket_cap_mb=cap, first_bucket_mb=first)
        return cap, first

    @staticmethod
    def _flatten(params):
        n = sum(p.numel() for p in params)
        dev, dt = params[0].device, params[0].dtype
        flat = torch.empty(n, device=dev, dtype=dt)
        grad = torch.zeros(n, device=dev, dtype=dt)
        o = 0
        for p in params:
            k = p.numel()
            flat[o:o + k].copy_(p.data.reshape(-1))
            p.data = flat[o:o + k].view_as(p)
            p.grad = grad[o:o + k].view_as(p)
            mark_fused_grad(p)
            o += k
        return flat, grad

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def _hook(self, p):
        if not self._callback_queued:
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            self._callback_queued = True
            self._pending = [len(b) for b in self._buckets]
            self._reduced = [False] * len(self._buckets)
            self._ready = set()
        # one notification per parameter per backward: a fused-grad parameter is
        # reported by the kernel's grad-ready hook AND by torch's post-accumulate hook
        # (which fires even for a None gradient); counting both would release a bucket
        # before the last producing kernel was launched
        if id(p) in self._ready:
            return
        self._ready.add(id(p))
        b = self._bucket_of[p]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._reduce_bucket(b)

    def _reduce_bucket(self, b):
        self._reduced[b] = True
        if self.world == 1:
            return
        lo, hi = self._spans[b]
        view = self._grad1d[lo:hi]
        if b in self._xgmi_buckets:
            # grads of this bucket are final on the current (backward) stream: reduce
            # them on the side stream while the backward continues
            self._side.wait_stream(torch.cuda.current_stream(view.device))
            with torch.cuda.stream(self._side):
                self._xgmi.all_reduce_(view)
            self._works.append(("xgmi", view))
        elif dist.get_backend(self.group) == "nccl":
            self._works.append((dist.all_reduce(view, group=self.group, async_op=True), view))
        else:
            comm_util.all_reduce_(view, self.group)
            self._works.append((None, view))

    def _finalize(self):
        # parameters that got no gradient in this backward (find_unused_parameters
        # semantics): their bucket is reduced with whatever the buffer holds (zeros
        # after zero_grad).  One backward per iteration, as with torch DDP.
        for b, done in enumerate(self._reduced):
            if not done:
                self._reduce_bucket(b)
        for w, view in self._works:
            if w == "xgmi":
                torch.cuda.current_stream(view.device).wait_stream(self._side)
            elif w is not None:
                w.wait()
        if self.world > 1:
            self.flat_grad.mul_(1.0 / self.world)
        self._works = []
        self._callback_queued = False

    def zero_grad(self):
        """Zero the flat gradient -- unless the last optimizer step already did
        (``mark_grad_clean``: the flat optimizer zeroes what it consumed), which saves a
        fill launch per optimizer step."""
        if getattr(self, "_grad_clean", False):
            self._grad_clean = False
            return
        self.flat_grad.zero_()

    def mark_grad_clean(self):
        """The whole flat gradient is zero now (set by the caller that zeroed it)."""
        self._grad_clean = True

    def reset_hooks(self):
        """Forget a backward that never finished (e.g. an aborted graph capture)."""
        self._works = []
        self._callback_queued = False

    def graph_safe(self) -> bool:
        """Can a backward through this wrapper be captured into a hipGraph?  Yes with
        one rank, when every bucket goes through the in-kernel xGMI all-reduce (its
        exchange epochs are device counters, so each replay is a fresh exchange), or
        when the remaining buckets ride RCCL (capturable collectives); not when a
        bucket is staged through gloo on the host."""
        if self.world == 1:
            return True
        if all(b in self._xgmi_buckets for b in range(len(self._buckets))):
            return True
        return dist.get_backend(self.group) == "nccl"

    def check_comm(self):
        """Raise if an xGMI all-reduce timed out (one host sync; call at log points)."""
        if self._xgmi is not None:
            self._xgmi.check()
