#!/usr/bin/env python3
"""Wide-MLP training throughput: the toy workload's structure (two independent
LeakyReLU MLPs X, Y on ToyData, MSE, Adam lr 1e-3, DDP) at widths where the
Linears are real GEMMs.

  ours  : ModelBank(2, hidden=W) -- every Linear on csrc/gemm.hip (bias/LeakyReLU
          epilogues, activation gradient fused into the dx GEMM), bf16 compute with
          fp32 master weights; FlatDDP (bucketed RCCL / xGMI all-reduce from the
          backward hooks); FlatOptimizer (one Adam launch for both models; with
          --shadow it also writes the bf16 weight operands, ops/gemm.py ComputeShadow)
  stock : nn.Sequential + torch.autocast(bf16) + torch DDP + torch.optim.Adam
          (hipBLASLt GEMMs, ATen elementwise) -- the same math on stock PyTorch-ROCm

usage: python scripts/bench_wide.py [--width 4096] [--depth 3] [--batch 8192] [--steps 20] [--impl ours|stock|both]
(N > 1 ranks: torch.distributed.run ... scripts/bench_wide.py).  Prints one JSON line per impl on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.parallel import comm_util  # noqa: E402
from distributed_training_pytorch_amd.runtime import bootstrap  # noqa: E402


def run_ours(a, X, Y, dev, world):
    from distributed_training_pytorch_amd.models.bank import ModelBank
    from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    torch.manual_seed(0)
    bank = ModelBank(2, hidden=a.width, depth=a.depth, compute_dtype=torch.bfloat16).to(dev)
    ddp = FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad, comm="rccl") if world > 1 else None
    # --shadow: Adam also writes the bf16 weight operands (no per-forward casts). Measured
    # at W = 4096 / 2048 / 1024: 4.52 / 1.78 / 1.28 ms vs 4.56 / 1.75 / 1.28 casting each
    # forward (profiles/r3_shadow/), so the cast stays the default
    opt = FlatOptimizer(bank.flat, bank.flat_grad, OptimConfig(lr=1e-3),
                        shadow=bank.compute_shadow() if a.shadow else None)
    mse = torch.nn.MSELoss()
    fwd = ddp if ddp is not None else bank

    def step(i):
        sl = slice((i * a.batch) % X.shape[0], (i * a.batch) % X.shape[0] + a.batch)
        x, y = X[sl], Y[sl]
        bank.zero_grad()
        ox, oy = fwd(x)
        (mse(ox, y) + mse(oy, y)).backward()
        opt.step()
    return step


def run_stock(a, X, Y, dev, world):
    from torch.nn.parallel import DistributedDataParallel as DDP

    def mk():
        mods = [torch.nn.Linear(2, a.width), torch.nn.LeakyReLU(0.01)]
        for _ in range(a.depth):
            mods += [torch.nn.Linear(a.width, a.width), torch.nn.LeakyReLU(0.01)]
        mods.append(torch.nn.Linear(a.width, 1))
        return torch.nn.Sequential(*mods).to(dev)

    torch.manual_seed(0)
    mx, my = mk(), mk()
    if world > 1:
        mx, my = DDP(mx, device_ids=[dev.index]), DDP(my, device_ids=[dev.index])
    try:
        ox_, oy_ = (torch.optim.Adam(m.parameters(), lr=1e-3, fused=True) for m in (mx, my))
    except (RuntimeError, TypeError):
        ox_, oy_ = (torch.optim.Adam(m.parameters(), lr=1e-3, foreach=True) for m in (mx, my))
    mse = torch.nn.MSELoss()

    def step(i):
        sl = slice((i * a.batch) % X.shape[0], (i * a.batch) % X.shape[0] + a.batch)
        x, y = X[sl], Y[sl]
        ox_.zero_grad(set_to_none=True)
        oy_.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lx, ly = mse(mx(x).float(), y), mse(my(x).float(), y)
        lx.backward()
        ly.backward()
        ox_.step()
        oy_.step()
    return step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--impl", choices=["ours", "stock", "both"], default="both")
    ap.add_argument("--shadow", action="store_true",
                    help="ours: the Adam kernel writes the bf16 weight operands (ops/gemm.py ComputeShadow) "
                         "instead of a cast before every forward")
    ap.add_argument("--gemm-backend", choices=["mfma", "blaslt"], default="mfma",
                    help="mfma: the library's kernels; blaslt: the large bf16 GEMMs on hipBLASLt + an epilogue "
                         "pass (scripts/blaslt_ref.py, an A/B reference outside the library)")
    a = ap.parse_args()
    if a.gemm_backend == "blaslt":
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from blaslt_ref import use_blaslt

        use_blaslt()
    env = bootstrap.detect()
    rank, world = env.rank, env.world_size
    dev = bootstrap.bind_device(env)
    if world > 1:
        bootstrap.init_process_group(env, "nccl", dev)
    X, Y = ToyData(n=a.batch * 4, seed=rank).device_tensors(dev)
    for impl in (["ours", "stock"] if a.impl == "both" else [a.impl]):
        step = (run_ours if impl == "ours" else run_stock)(a, X, Y, dev, world)
        for i in range(a.warmup):
            step(i)
        torch.cuda.synchronize()
        comm_util.barrier()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(i)
        torch.cuda.synchronize()
        comm_util.barrier()
        dt = comm_util.all_reduce_scalar(time.perf_counter() - t0, dist.ReduceOp.MAX)
        params = 2 * (2 * a.width + a.width + a.depth * (a.width * a.width + a.width) + a.width + 1)
        flops = 6.0 * params * a.batch * a.steps * world  # fwd + bwd (dx, dW) of both models
        if rank == 0:
            print(json.dumps({"impl": impl, "width": a.width, "depth": a.depth, "batch_per_rank": a.batch,
                              "world": world, "ms_per_step": 1e3 * dt / a.steps,
                              "samples_per_s": a.batch * world * a.steps / dt, "model_tflops": flops / dt / 1e12,
                              "dtype": "bf16 compute, fp32 master weights",
                              "gemm_backend": a.gemm_backend if impl == "ours" else "torch",
                              "weight_shadow": a.shadow if impl == "ours" else None}),
                  flush=True)
        del step
        torch.cuda.empty_cache()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
