"""Where the fused layer-split iteration goes: the split stage kernel at K = 1 (the whole
model as one stage: no links), K = 2 (the reference split) and K = 5, per-device launch,
device-scope links (stages on one GPU) vs system-scope uncached links.
python scripts/split_cost.py  -> JSON lines {K, links, us_per_step}."""
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


def run(K, local, launch="per_device", n=2000):
    os.environ["DTP_SPLIT_LOCAL_LINKS"] = "1" if local else "0"
    dev = torch.device("cuda", 0)
    ds = ToyData(n=512, seed=2)
    init = torch.randn(TOY_SPEC.P, generator=torch.Generator().manual_seed(0)) * 0.4
    eng = FusedLayerSplit(TOY_SPEC, [dev] * K, ds.X, ds.Y, SamplerGeometry(n=512, batch=256, seed=1),
                          OptimConfig(lr=1e-3), init, launch=launch)
    eng.train(50)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.train(n)
    eng.synchronize()
    us = (time.perf_counter() - t0) / n * 1e6
    eng.close()
    return us


if __name__ == "__main__":
    for K, local, launch in [(1, True, "per_device"), (2, True, "per_device"), (2, False, "per_device"),
                             (2, True, "per_stage"), (3, True, "per_device"), (5, True, "per_device"),
                             (1, True, "per_device"), (2, True, "per_device")]:
        print(json.dumps({"lib": os.environ.get("DTP_LIB", "default"), "K": K, "links": "device" if local else "system", "launch": launch,
                          "us_per_step": round(run(K, local, launch), 3)}), flush=True)
