"""Diagnostic: module step (ModelBank + FlatDDP xGMI buckets + FlatOptimizer) captured
as a hipGraph vs eager, two ranks on one GPU.  Records the reduced gradient of every
step inside the step itself and reports the first step / elements where graph and
eager differ, for one bucket and for many buckets."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.dist_utils import run_ranks  # noqa: E402


def rank_fn(rank, world, graphs, many, steps):
    from distributed_training_pytorch_amd.engine.graph_step import CapturedStep
    from distributed_training_pytorch_amd.models.bank import ModelBank
    from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    bank = ModelBank(2).to(dev)
    kw = dict(first_bucket_mb=0.0005, bucket_cap_mb=0.001) if many else {}
    ddp = FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad, comm="xgmi", **kw)
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
    st = ddp._xgmi.status[:2].tolist() if ddp._xgmi else None
    return hist.cpu(), bank.flat.cpu(), [(lo, hi) for lo, hi in ddp._spans], stepper.replays, st, \
        ddp._xgmi.epochs.cpu() if ddp._xgmi else None


def main():
    steps = 6
    for many in (False, True):
        e = run_ranks(rank_fn, 2, (False, many, steps), timeout=300)
        g = run_ranks(rank_fn, 2, (True, many, steps), timeout=300)
        print(f"== many_buckets={many} spans={e[0][2]} replays={g[0][3]} status e={e[0][4]} g={g[0][4]} "
              f"epochs e={e[0][5].tolist()} g={g[0][5].tolist()}", flush=True)
        for t in range(steps):
            d = (g[0][0][t] - e[0][0][t]).abs()
            bad = (d > 0).nonzero().view(-1).tolist()
            r01 = torch.equal(g[0][0][t], g[1][0][t])
            print(f"step {t}: max|g-e|={d.max().item():.3e} n_diff={len(bad)} first={bad[:8]} "
                  f"last={bad[-4:]} graph ranks equal={r01}", flush=True)


if __name__ == "__main__":
    main()
