"""Where a multi-rank K-step bench region goes, per rank (run under torchrun; --share-gpu
puts every rank on cuda:0).  Prints, per repetition, each rank's host launch time,
device time of the K-step kernel (events), and wall time of the barrier-bracketed region."""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd import _native  # noqa: E402
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.models.toy import ToyModel  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402
from distributed_training_pytorch_amd.parallel.xgmi import DeviceBarrier  # noqa: E402
from distributed_training_pytorch_amd.runtime import bootstrap  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--reps", type=int, default=6)
a = ap.parse_args()
_native.set_wait_mode(os.environ.get("DTP_WAIT_MODE", "spin"))
env = bootstrap.detect()
env.local_rank = 0
rank, world = env.rank, env.world_size
dev = bootstrap.bind_device(env)
bootstrap.init_process_group(env, "gloo", dev)
n = 512
X, Y = ToyData(n=n, seed=0).device_tensors(dev)
geom = SamplerGeometry(n=n, world=world, rank=rank, batch=256, seed=0)
torch.manual_seed(0)
tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, cfg=EngineConfig(),
                  init_params=[ToyModel().flat_params.detach().clone() for _ in range(2)])
bar = DeviceBarrier(dev)
tr.train(5)
bar()
torch.cuda.synchronize()
rows = []
for r in range(a.reps):
    bar()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    tr.train(a.steps)
    e1.record()
    tl = time.perf_counter()
    bar()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    rows.append({"launch_us": (tl - t0) * 1e6, "kernel_us": e0.elapsed_time(e1) * 1e3, "wall_us": (t1 - t0) * 1e6,
                 "t0_abs": t0})
allr = [None] * world
dist.all_gather_object(allr, rows)
if rank == 0:
    for r in range(a.reps):
        t0s = [allr[k][r]["t0_abs"] for k in range(world)]
        print(json.dumps({"rep": r, "t0_skew_us": round((max(t0s) - min(t0s)) * 1e6, 1),
                          "launch_us": [round(allr[k][r]["launch_us"], 1) for k in range(world)],
                          "kernel_us": [round(allr[k][r]["kernel_us"], 1) for k in range(world)],
                          "wall_us": [round(allr[k][r]["wall_us"], 1) for k in range(world)]}), flush=True)
tr.close()
bar.close()
dist.destroy_process_group()
