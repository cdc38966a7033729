"""Gradient-bucket sizes for FlatDDP chosen by measuring the all-reduce on the node it
runs on.

The reference wraps its models in torch DDP with the default buckets (25 MB, first bucket
1 MiB; ``/root/reference/demo.py:69-72`` -> torch/nn/parallel/distributed.py).  Those
defaults were tuned for PCIe / NVLink rings.  On an MI355X node every ring hop is ONE
point-to-point xGMI link (7 per GPU, ~153 GB/s each way), so what a bucket costs is
RCCL's fixed per-collective latency (launch plus 2 (W-1) hops) against the bytes it moves
-- numbers this process can measure at start-up instead of assuming:

* every rank all-reduces buffers of a few sizes (all ranks, same order, max over ranks
  of the median of ``reps`` timed calls, so every rank sees the same numbers);
* the times are fitted to ``t(n) = alpha + n / beta`` (least squares);
* the bucket cap is the size whose fixed cost is ~10 % of its time (``n = 9 alpha
  beta``): larger buckets gain < 10 %, smaller ones pay the latency again per bucket;
* the first bucket (the last layers' gradients, reduced while the backward still runs)
  is the size where the transfer equals the fixed cost (``n = alpha beta``): as small as
  possible while still moving bytes half of its time.

Both are clipped to sane ranges (first 64 KiB .. cap, cap 1 MiB .. 256 MiB: 288 GB of
HBM per GPU makes large buckets cheap) and the plan is cached per (process group,
device).  FlatDDP runs this only with several ranks and a gradient larger than the
smallest probe (a model that fits one small bucket -- the toy MLP, 3 KB -- has nothing
to choose)."""
from __future__ import annotations

import statistics
import time

import torch
import torch.distributed as dist

from . import comm_util

DEFAULT_SIZES = (256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20)
_cache: dict = {}


def measure_allreduce(group=None, device=None, sizes=DEFAULT_SIZES, reps: int = 5, warmup: int = 2) -> list:
    """[(bytes, seconds)]: the slowest rank's median time of one SUM all-reduce of a
    float32 buffer of each size (every rank must call this with the same arguments)."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    sync = (lambda: torch.cuda.synchronize(device)) if device.type == "cuda" else (lambda: None)
    out = []
    for nbytes in sizes:
        buf = torch.ones(max(1, nbytes // 4), dtype=torch.float32, device=device)
        times = []
        for i in range(warmup + reps):
            comm_util.barrier(group)
            sync()
            t0 = time.perf_counter()
            dist.all_reduce(buf, group=group)
            sync()
            if i >= warmup:
                times.append(time.perf_counter() - t0)
        med = comm_util.all_reduce_scalar(statistics.median(times), dist.ReduceOp.MAX, group)
        out.append((int(nbytes), float(med)))
        del buf
    return out


def fit_latency_bandwidth(meas: list) -> tuple[float, float]:
    """Least-squares fit of t = alpha + n / beta; returns (alpha seconds, beta bytes/s)
    (alpha clamped >= 0, beta > 0)."""
    xs = [float(n) for n, _ in meas]
    ys = [float(t) for _, t in meas]
    k = len(xs)
    mx, my = sum(xs) / k, sum(ys) / k
    sxx = sum((x - mx) ** 2 for x in xs)
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx if sxx > 0 else 0.0
    if slope <= 0:  # latency-bound over the whole range: treat the largest probe as "bandwidth"
        slope = ys[-1] / xs[-1] if xs[-1] > 0 else 1e-12
    alpha = max(0.0, my - slope * mx)
    return alpha, 1.0 / slope


def choose_buckets(meas: list, min_first: int = 64 << 10, min_cap: int = 1 << 20,
                   max_cap: int = 256 << 20) -> dict:
    alpha, beta = fit_latency_bandwidth(meas)
    cap = int(min(max(9.0 * alpha * beta, min_cap), max_cap))
    first = int(min(max(alpha * beta, min_first), cap))
    return {"first_bucket_mb": first / 2 ** 20, "bucket_cap_mb": cap / 2 ** 20, "alpha_us": alpha * 1e6,
            "bandwidth_GBps": beta / 1e9, "measured": [(n, t * 1e6) for n, t in meas], "source": "measured"}


def plan(group=None, device=None, sizes=None, reps: int = 5) -> dict:
    """The (cached) bucket plan of this process group on this device (sizes: the probe
    sizes in bytes, default DEFAULT_SIZES as of the call)."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    sizes = tuple(sizes) if sizes is not None else tuple(DEFAULT_SIZES)
    key = (id(group), str(device), tuple(sizes), reps)
    p = _cache.get(key)
    if p is None:
        p = choose_buckets(measure_allreduce(group, device, sizes, reps))
        _cache[key] = p
    return p
