"""Host cost of torch ops alone vs interleaved with native (ctypes) launches (GPU box)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd import _native as nat  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC, stage_forward  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
a = torch.randn(256, 1, device=dev)
b = torch.randn(256, 1, device=dev)
x = torch.randn(256, 2, device=dev)
flat = torch.randn(TOY_SPEC.P, device=dev)


def bench(name, fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    host = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / n * 1e6
    print(f"{name:40s} host {host:7.2f} us/iter   wall {wall:7.2f} us/iter", flush=True)


bench("mse_loss", lambda: torch.nn.functional.mse_loss(a, b))
bench(".to(same device)", lambda: a.to(dev, non_blocking=True))
bench("current_stream()", lambda: torch.cuda.current_stream())
bench("is_available()", lambda: torch.cuda.is_available())
bench("stream_ptr()", lambda: nat.stream_ptr())
bench("stage_forward", lambda: stage_forward(x, flat, TOY_SPEC, save=True))


def mix():
    stage_forward(x, flat, TOY_SPEC, save=True)
    torch.nn.functional.mse_loss(a, b)


bench("stage_forward + mse_loss", mix)
bench("empty kernel (a.add_(0))", lambda: a.add_(0.0))
