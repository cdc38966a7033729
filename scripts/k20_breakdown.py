"""Where a short persistent launch's wall time goes (the driver's K = 20 bench call).

Same setup as ``bench.py`` (fp32, DistributedSampler order, 2 models, batch 256),
5 warm-up steps, then R fresh ``train(K)`` calls, each bracketed like the bench's
timed region (synchronize before and after).  Per call: the host time until
``train`` returns (argument marshalling + the launch) and the time until the
synchronize returns.  Kernel durations come from a rocprofv3 run of the same
script (``--kernel-trace``), so wall - kernel = launch + completion overhead.
"""
import json
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
from distributed_training_pytorch_amd.models.toy import ToyModel  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import OptimConfig  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    nat.set_wait_mode(os.environ.get("DTP_WAIT_MODE", "spin"))
    dev = torch.device("cuda", 0)
    X, Y = ToyData(n=512, seed=0).device_tensors(dev)
    torch.manual_seed(0)
    init = [ToyModel().flat_params.detach().clone() for _ in range(2)]
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=256, seed=0), OptimConfig(lr=1e-3),
                      EngineConfig(), init_params=init)
    tr.train(5)
    torch.cuda.synchronize(dev)
    host, wall = [], []
    for _ in range(R):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        tr.train(K)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e6)
        wall.append((t2 - t0) * 1e6)
    # an empty-kernel round trip on the same stream, for scale
    rt = []
    z = torch.zeros(1, device=dev)
    for _ in range(R):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        z.add_(1)
        torch.cuda.synchronize(dev)
        rt.append((time.perf_counter() - t0) * 1e6)
    med = statistics.median
    print(json.dumps({"K": K, "calls": R, "host_call_us_median": med(host), "wall_us_median": med(wall),
                      "wall_us_min": min(wall), "tiny_kernel_roundtrip_us_median": med(rt)}))


if __name__ == "__main__":
    main()
