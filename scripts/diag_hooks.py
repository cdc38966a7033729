"""Diagnostic: order of FusedMLP backward calls, in-place decisions and FlatDDP hook
calls in a 2-rank FlatDDP (gloo) backward on one GPU."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.dist_utils import run_ranks  # noqa: E402


def rank_fn(rank, world):
    from distributed_training_pytorch_amd.models.bank import ModelBank
    from distributed_training_pytorch_amd.ops import mlp as mlp_mod
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    log = []
    orig_bwd = mlp_mod.FusedMLPFunction.backward

    def bwd(ctx, grad_out):
        ids = [id(p) for p in ctx.params]
        import threading

        log.append(("bwd", ids[0] % 100000, ctx.needs_input_grad,
                    [mlp_mod._fused_grad_target(p) is not None for p in ctx.params], threading.get_ident() % 10000,
                    torch.cuda.current_stream().cuda_stream % 100000))
        return orig_bwd(ctx, grad_out)

    mlp_mod.FusedMLPFunction.backward = staticmethod(bwd)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    bank = ModelBank(2).to(dev)
    ddp = FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad, comm="rccl")
    orig_hook = ddp._hook

    def hook(p):
        import threading

        idx = next(i for i, q in enumerate(ddp._params) if q is p)
        log.append(("hook", idx, ddp._pending[0] if ddp._callback_queued else None, threading.get_ident() % 10000,
                    torch.cuda.current_stream().cuda_stream % 100000))
        return orig_hook(p)

    ddp._hook = hook
    orig_red = ddp._reduce_bucket

    def red(b):
        log.append(("reduce", b))
        return orig_red(b)

    ddp._reduce_bucket = red
    orig_fin = ddp._finalize

    def fin():
        log.append(("finalize",))
        return orig_fin()

    ddp._finalize = fin
    for p in ddp._params:  # re-point the registered grad-ready hooks at the tracer
        p._dtp_grad_ready_hooks = [hook]
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(64, 2, generator=g).to(dev)
    y = torch.randn(64, 1, generator=g).to(dev)
    bank.zero_grad()
    ox, oy = ddp(x)
    (torch.nn.functional.mse_loss(ox, y) + torch.nn.functional.mse_loss(oy, y)).backward()
    torch.cuda.synchronize()
    return log, [id(p) % 100000 for p in ddp._params]


if __name__ == "__main__":
    r = run_ranks(rank_fn, 2, (), timeout=200)
    for e in r[0][0]:
        print(e, flush=True)
    print("param ids", r[0][1])
