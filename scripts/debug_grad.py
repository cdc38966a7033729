"""Compare one fused MODE_GRAD step (gradients + loss) with torch autograd, per layer."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd import _native as nat  # noqa: E402
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC, mlp_forward_ref, unflatten  # noqa: E402

dev = torch.device("cuda", 0)
X, Y = ToyData(seed=3).device_tensors(dev)
for B in (256, 64, 100):
    geom = SamplerGeometry(n=512, batch=B, seed=11)
    g = torch.Generator().manual_seed(0)
    init = [(torch.randn(TOY_SPEC.P, generator=g) * 0.4).to(dev) for _ in range(2)]
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, cfg=EngineConfig(), init_params=init)
    lib = nat.load()
    a = tr._train_args(1, nat.MODE_GRAD, None)
    nat.check(lib.dtp_mlp_train(ctypes.byref(a), *TOY_SPEC.key[:4], nat.MODE_GRAD, nat.stream_ptr()), "grad")
    torch.cuda.synchronize()
    idx = torch.tensor(geom.indices(0), device=dev)
    for i in range(2):
        p = init[i].clone().requires_grad_(True)
        loss = torch.nn.functional.mse_loss(mlp_forward_ref(p, TOY_SPEC, X[idx]), Y[idx])
        (gr,) = torch.autograd.grad(loss, p)
        got = tr.comm_buf[i * TOY_SPEC.P:(i + 1) * TOY_SPEC.P]
        names = ["W0", "b0", "W1", "b1", "W2", "b2", "W3", "b3", "W4", "b4"]
        errs = {n: (a_ - b_).abs().max().item() for n, a_, b_ in zip(names, unflatten(got, TOY_SPEC), unflatten(gr, TOY_SPEC))}
        print(f"B={B} model {i}: loss got {tr.comm_buf[2 * TOY_SPEC.P + i].item():.6f} ref {loss.item():.6f}; "
              f"max|grad err| per tensor: " + ", ".join(f"{k}={v:.2e}" for k, v in errs.items()), flush=True)
