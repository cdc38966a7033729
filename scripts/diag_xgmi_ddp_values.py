"""Diagnostic: per step, the reduced gradient FlatDDP(xGMI) leaves in flat_grad on each
of two ranks (one GPU), against the mean of the ranks' local gradients computed on
the host from the same parameters (autograd on CPU)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.dist_utils import run_ranks  # noqa: E402


def rank_fn(rank, world, steps, comm, with_opt, many=False):
    from distributed_training_pytorch_amd.models.bank import ModelBank
    from distributed_training_pytorch_amd.ops.mlp import mlp_forward_ref
    from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    bank = ModelBank(2).to(dev)
    kw = dict(first_bucket_mb=0.0005, bucket_cap_mb=0.001) if many else {}
    ddp = FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad, comm=comm, **kw)
    calls = []
    orig = ddp._reduce_bucket

    def traced(b):
        calls.append((b, sorted(i for i, q in enumerate(ddp._params) if ddp._bucket_of[q] == b)))
        return orig(b)

    ddp._reduce_bucket = traced
    opt = FlatOptimizer(bank.flat, bank.flat_grad, OptimConfig(lr=1e-2))
    g = torch.Generator().manual_seed(rank)
    out = []
    for t in range(steps):
        x = torch.randn(64, 2, generator=g)
        y = torch.randn(64, 1, generator=g)
        p0 = bank.flat.detach().cpu().clone()
        local = []
        for i in range(2):
            q = p0[i].clone().requires_grad_(True)
            (gq,) = torch.autograd.grad(torch.nn.functional.mse_loss(mlp_forward_ref(q, bank.spec, x), y), q)
            local.append(gq)
        bank.zero_grad()
        ox, oy = ddp(x.to(dev))
        (torch.nn.functional.mse_loss(ox, y.to(dev)) + torch.nn.functional.mse_loss(oy, y.to(dev))).backward()
        red = bank.flat_grad.detach().cpu().clone()
        if with_opt:
            opt.step()
        out.append((p0, torch.stack(local), red, list(calls)))
        calls.clear()
    ddp.check_comm()
    return out, ddp.comm


def main():
    allres = {}
    for comm in ("xgmi", "rccl"):
        for many in (False, True):
            r = run_ranks(rank_fn, 2, (3, comm, False, many), timeout=300)
            allres[(comm, many)] = r
            print(f"== comm={comm}/{r[0][1]} many={many}", flush=True)
            for t in range(3):
                p00, l0, r0, c0 = r[0][0][t]
                p10, l1, r1, c1 = r[1][0][t]
                ref = (l0 + l1) / 2
                print(f"step {t}: params equal={torch.equal(p00, p10)} red equal={torch.equal(r0, r1)} "
                      f"|r0-ref|={(r0 - ref).abs().max():.3e} |r1-ref|={(r1 - ref).abs().max():.3e} "
                      f"|r0-l0|={(r0 - l0).abs().max():.3e} |ref|={(ref).abs().max():.3e} calls0={c0}", flush=True)
    torch.save({f"{k[0]}_{int(k[1])}": [[list(x[:3]) for x in v[r][0]] for r in range(2)] for k, v in allres.items()},
               "gpurun_out/diag_values.pt")


if __name__ == "__main__":
    main()
