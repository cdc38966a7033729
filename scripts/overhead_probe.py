#!/usr/bin/env python3
"""Fixed per-call overhead of the persistent fused step (1 GPU).

``bench.py --steps K`` times ONE ``train(K)`` call: host argument marshalling,
the kernel launch, the kernel prologue (dataset -> LDS, weights, Adam table),
K steps, the epilogue, and ``torch.cuda.synchronize``.  At small K the fixed
part dominates.  This probe fits wall(K) = fixed + K * per_step over several K
and times the host-side pieces on their own.

Usage: python scripts/overhead_probe.py [--reps 30]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_training_pytorch_amd import _native as nat  # noqa: E402
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.models.toy import ToyModel  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import OptimConfig  # noqa: E402


def med(f, reps):
    xs = []
    for _ in range(reps):
        xs.append(f())
    return statistics.median(xs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--cold", action="store_true", help="only the bench sequence, first thing in the process")
    a = ap.parse_args()
    if a.cold:
        torch.cuda.set_device(0)
        print(json.dumps({"bench_sequence_cold": bench_sequence()}, indent=1))
        return
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ds = ToyData(n=512, seed=0)
    X, Y = ds.device_tensors(dev)
    geom = SamplerGeometry(n=512, world=1, rank=0, batch=256, seed=0)
    torch.manual_seed(0)
    init = [ToyModel().flat_params.detach().clone() for _ in range(2)]
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, OptimConfig(lr=1e-3), EngineConfig(), init_params=init)
    tr.train(5)
    tr.synchronize()

    out = {}

    def timed(k):
        def f():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.train(k)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e6
        return f

    ks = [1, 2, 5, 10, 20, 50, 100, 200, 1000]
    wall = {k: med(timed(k), a.reps) for k in ks}
    out["wall_us"] = wall
    # least squares over K >= 5
    xs = [k for k in ks if k >= 5]
    ys = [wall[k] for k in xs]
    mx, my = statistics.mean(xs), statistics.mean(ys)
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    out["fit_per_step_us"] = slope
    out["fit_fixed_us"] = my - slope * mx

    def sync_idle():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6
    out["sync_idle_us"] = med(sync_idle, a.reps)

    lib = nat.load()

    def args_only():
        t0 = time.perf_counter()
        for _ in range(100):
            tr._train_args(20, tr._update_mode(), None)
        return (time.perf_counter() - t0) * 1e4
    out["train_args_us"] = med(args_only, 5)

    def launch_host():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.train(1)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        return (t1 - t0) * 1e6
    out["train1_host_us"] = med(launch_host, a.reps)

    def empty_kernel():
        z = torch.empty(1, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        z.zero_()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6
    out["torch_tiny_kernel_roundtrip_us"] = med(empty_kernel, a.reps)

    # device-side time of one train(k) via events
    def ev(k):
        def f():
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            tr.train(k)
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) * 1e3
        return f
    out["event_us"] = {k: med(ev(k), a.reps) for k in (1, 20, 1000)}
    tr.close()
    out["bench_sequence"] = bench_sequence()
    print(json.dumps(out, indent=1))


def bench_sequence(reps: int = 3):
    """bench.py's exact sequence on fresh trainers: train(W); sync; t0; train(20); sync; t1."""
    dev = torch.device("cuda", 0)
    ds = ToyData(n=512, seed=0)
    X, Y = ds.device_tensors(dev)
    res = []
    for W in (5, 5, 50, 200, 2000, 5):
        for _ in range(reps):
            geom = SamplerGeometry(n=512, world=1, rank=0, batch=256, seed=0)
            torch.manual_seed(0)
            init = [ToyModel().flat_params.detach().clone() for _ in range(2)]
            tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, OptimConfig(lr=1e-3), EngineConfig(), init_params=init)
            tr.train(W)
            tr.synchronize()
            tr.synchronize()
            t0 = time.perf_counter()
            tr.train(20)
            tc = time.perf_counter()
            tr.synchronize()
            t1 = time.perf_counter()
            res.append({"W": W, "call_us": (tc - t0) * 1e6, "wall_us": (t1 - t0) * 1e6})
            tr.close()
    return res


if __name__ == "__main__":
    main()
