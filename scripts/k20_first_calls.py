"""Wall time (us) of the first eight 20-step calls of a fresh process after the bench's
warm-up (5 one-step launches), each on an idle GPU: is the first one the slow one?"""
import os
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
for _ in range(5):
    tr.train(1)
torch.cuda.synchronize()
out = []
for i in range(8):
    time.sleep(0.01 if os.environ.get("PAUSE", "1") == "1" else 0.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train(20)
    torch.cuda.synchronize()
    out.append((time.perf_counter() - t0) * 1e6)
print(" ".join(f"{v:.0f}" for v in out))
