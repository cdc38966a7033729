"""Diagnostic: FlatDDP xGMI buckets without host syncs between steps, two ranks on one
GPU.  Modes: side (default code: bucket reduced on a side stream from the grad-ready
hook), sync (device synchronize before each bucket reduction), inline (reduction on
the backward's own stream).  Prints whether the ranks' reduced gradients agree."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.dist_utils import run_ranks  # noqa: E402


def rank_fn(rank, world, mode, many, steps, graphs):
    from distributed_training_pytorch_amd.engine.graph_step import CapturedStep
    from distributed_training_pytorch_amd.models.bank import ModelBank
    from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig
    from distributed_training_pytorch_amd.parallel import ddp as ddp_mod

    orig = ddp_mod.FlatDDP._reduce_bucket

    def patched(self, b):
        if mode == "sync":
            torch.cuda.synchronize()
            return orig(self, b)
        if mode == "inline" and b in self._xgmi_buckets:
            self._reduced[b] = True
            lo, hi = self._spans[b]
            self._xgmi.all_reduce_(self._grad1d[lo:hi])
            self._works.append((None, self._grad1d[lo:hi]))
            return
        return orig(self, b)

    ddp_mod.FlatDDP._reduce_bucket = patched
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    bank = ModelBank(2).to(dev)
    kw = dict(first_bucket_mb=0.0005, bucket_cap_mb=0.001) if many else {}
    ddp = ddp_mod.FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad, comm="xgmi", **kw)
    opt = FlatOptimizer(bank.flat, bank.flat_grad, OptimConfig(lr=1e-2))
    g = torch.Generator().manual_seed(rank)
    xs = torch.randn(steps, 64, 2, generator=g).to(dev)
    ys = torch.randn(steps, 64, 1, generator=g).to(dev)
    x_st, y_st = xs[0].clone(), ys[0].clone()
    hist = torch.zeros(steps, 742, device=dev)
    slot = torch.zeros((), dtype=torch.long, device=dev)

    def body(_):
        bank.zero_grad()
        ox, oy = ddp(x_st)
        (torch.nn.functional.mse_loss(ox, y_st) + torch.nn.functional.mse_loss(oy, y_st)).backward()
        hist.index_copy_(0, slot.view(1), bank.flat_grad.view(1, -1))
        slot.add_(1)
        opt.step()

    stepper = CapturedStep(body, dev, enabled=graphs, on_abort=ddp.reset_hooks)
    for t in range(steps):
        x_st.copy_(xs[t])
        y_st.copy_(ys[t])
        stepper.run(0)
    torch.cuda.synchronize()
    return hist.cpu(), stepper.replays


def main():
    steps = 6
    for graphs in (False, True):
        for many in (False, True):
            for mode in ("sync", "side", "inline"):
                if graphs and mode == "sync":
                    continue
                r = run_ranks(rank_fn, 2, (mode, many, steps, graphs), timeout=300)
                eq = [torch.equal(r[0][0][t], r[1][0][t]) for t in range(steps)]
                print(f"graphs={graphs} many={many} mode={mode}: ranks equal per step {eq} replays={r[0][1]}",
                      flush=True)
                torch.save(r[0][0], f"gpurun_out/diag_{int(graphs)}{int(many)}_{mode}.pt")


if __name__ == "__main__":
    main()
