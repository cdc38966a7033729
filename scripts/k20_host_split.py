"""Split the K=20 call's wall time into launch (train() returning), completion wait
(synchronize) and the kernel itself, in one process: the bench's setup, 5 warm-up steps,
then 12 timed 20-step calls with a pause between them (each starts on an idle GPU, as
the bench's single timed call does)."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import OptimConfig  # noqa: E402
from distributed_training_pytorch_amd import _native  # noqa: E402

_native.set_wait_mode("spin")
dev = torch.device("cuda", 0)
X, Y = ToyData(n=512, seed=0).device_tensors(dev)
tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=256, seed=0), OptimConfig(lr=1e-3),
                  EngineConfig(steps_per_launch=1000))
for _ in range(5):
    tr.train(1)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
rows = []
for i in range(12):
    time.sleep(0.01)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    tr.train(20)
    ev1.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    rows.append(((t1 - t0) * 1e6, (t2 - t1) * 1e6, (t2 - t0) * 1e6, ev0.elapsed_time(ev1) * 1e3))
for r in rows:
    print("launch %.1f us, wait %.1f us, total %.1f us, events %.1f us" % r)
print("median total %.1f us" % statistics.median(r[2] for r in rows))
