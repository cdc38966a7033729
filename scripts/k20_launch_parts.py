"""Host cost of the pieces of FusedTrainer.train(20) on this box (us, median of 30
calls, each on an idle GPU): the ring check, the native launch call alone, and the
whole train(); plus a bare torch fill launch for scale."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd import _native as nat  # noqa: E402
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import OptimConfig  # noqa: E402

nat.set_wait_mode("spin")
dev = torch.device("cuda", 0)
X, Y = ToyData(n=512, seed=0).device_tensors(dev)
tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=256, seed=0), OptimConfig(lr=1e-3),
                  EngineConfig(steps_per_launch=1000))
tr.train(5)
torch.cuda.synchronize()
x = torch.zeros(1, device=dev)


def med(fn, n=30):
    ts = []
    for _ in range(n):
        time.sleep(0.005)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    return statistics.median(ts) * 1e6


print("ring check      %.1f us" % med(lambda: tr._ensure_epochs(20)))
raw = nat.raw_stream(0)
print("raw_stream      %.1f us" % med(lambda: nat.raw_stream(0)))
print("native launch   %.1f us" % med(lambda: tr._engine_run(tr._engine, 20, tr.t, raw)))
print("train(20)       %.1f us" % med(lambda: tr.train(20)))
print("torch fill      %.1f us" % med(lambda: x.fill_(1.0)))
print("empty sleep     %.1f us" % med(lambda: None))
