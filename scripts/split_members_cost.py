"""The fused layer split with split-batch stages (csrc/split_lanes.hip) against the
one-workgroup stages (csrc/split_train.hip): us per iteration at K = 1 / 2 / 3 / 5 stages
(all on one MI355X, per-device launch, device-scope links), members = 0 (one workgroup
per stage) / auto (ceil(batch / 64)) / 8, K = 2000-step launches, batch 256.
python scripts/split_members_cost.py -> JSON lines {K, members, us_per_step}."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import OptimConfig  # noqa: E402
from distributed_training_pytorch_amd.parallel.layer_split import FusedLayerSplit  # noqa: E402


def run(K, members, n=2000, launch="per_device", batch=256):
    dev = torch.device("cuda", 0)
    ds = ToyData(n=512, seed=2)
    init = torch.randn(TOY_SPEC.P, generator=torch.Generator().manual_seed(0)) * 0.4
    eng = FusedLayerSplit(TOY_SPEC, [dev] * K, ds.X, ds.Y, SamplerGeometry(n=512, batch=batch, seed=1),
                          OptimConfig(lr=1e-3), init, launch=launch, members=members)
    m = eng.members
    eng.train(50)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.train(n)
    eng.synchronize()
    us = (time.perf_counter() - t0) / n * 1e6
    eng.close()
    return m, us


if __name__ == "__main__":
    cases = [(2, 0), (2, "auto"), (1, "auto"), (3, "auto"), (5, "auto"), (2, 8), (2, "auto", "per_stage"),
             (2, 0), (2, "auto")]
    for c in cases:
        K, members = c[0], c[1]
        launch = c[2] if len(c) > 2 else "per_device"
        m, us = run(K, members, launch=launch)
        print(json.dumps({"K": K, "members": m, "launch": launch, "us_per_step": round(us, 3)}), flush=True)
