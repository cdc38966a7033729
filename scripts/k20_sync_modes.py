"""K=20 call wall time (us) by how the host waits for it, one process, alternating,
each call on an idle GPU: synchronize only; an event recorded behind the launch, then
synchronize; the event's own synchronize; the stream's synchronize."""
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

nat.set_wait_mode(os.environ.get("DTP_WAIT_MODE", "spin"))
dev = torch.device("cuda", 0)
X, Y = ToyData(n=512, seed=0).device_tensors(dev)
tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=256, seed=0), OptimConfig(lr=1e-3),
                  EngineConfig(steps_per_launch=1000))
tr.train(5)
torch.cuda.synchronize()
ev = torch.cuda.Event()
st = torch.cuda.current_stream()


def sync_only():
    tr.train(20)
    torch.cuda.synchronize()


def ev_then_sync():
    tr.train(20)
    ev.record()
    torch.cuda.synchronize()


def ev_sync():
    tr.train(20)
    ev.record()
    ev.synchronize()


def stream_sync():
    tr.train(20)
    st.synchronize()


modes = [sync_only, ev_then_sync, ev_sync, stream_sync]
res = {m.__name__: [] for m in modes}
for r in range(12):
    for m in modes:
        time.sleep(0.01)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m()
        res[m.__name__].append((time.perf_counter() - t0) * 1e6)
for k, v in res.items():
    print(f"{k:14s} median {statistics.median(v):.1f} us  min {min(v):.1f}  max {max(v):.1f}")
