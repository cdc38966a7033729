"""How tight can the lanes / split-batch tests' parameter tolerances be?  Runs the
configurations of tests/test_lanes_gpu.py (fused step vs autograd + torch.optim in fp64,
tests/ref_train.py) and prints, per case, the largest parameter error and the smallest
rtol that passes with the tests' atol (2e-5).  GPU only; writes one JSON line per case."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_training_pytorch_amd.data.sampler import EpochIndexStream, SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC, MlpSpec  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import OptimConfig  # noqa: E402
from tests.ref_train import torch_train  # noqa: E402

DEV = torch.device("cuda", 0)


def _init(spec, seed, n=2, scale=0.4):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(spec.P, generator=g) * scale).to(DEV) for _ in range(n)]


def needed_rtol(got, ref, atol=2e-5):
    d = (got.double() - ref.double()).abs()
    r = torch.clamp(d - atol, min=0) / ref.double().abs().clamp_min(1e-30)
    return float(d.max()), float(r.max())


def case(spec, batch, seed_data, seed_geom, init_seed, scale, lr, steps, groups="auto", label=""):
    X, Y = ToyData(n=512, seed=seed_data).device_tensors(DEV)
    if spec.out_features > 1:
        Y = torch.randn(512, spec.out_features, device=DEV)
    geom = SamplerGeometry(n=512, batch=batch, seed=seed_geom)
    init = _init(spec, init_seed, scale=scale)
    ocfg = OptimConfig(lr=lr)
    tr = FusedTrainer(spec, 2, X, Y, geom, ocfg, EngineConfig(steps_per_launch=7, groups=groups), init_params=init)
    steps = steps if steps else 2 * geom.steps_per_epoch + 3
    tr.train(steps)
    tr.synchronize()
    ref_p, ref_l = torch_train(spec, init, X, Y, [EpochIndexStream(geom)], steps, ocfg)
    dmax, rt = needed_rtol(tr.params.cpu(), ref_p)
    print(json.dumps({"case": label, "batch": batch, "lanes": tr.lanes, "groups": tr.groups, "steps": steps,
                      "max_abs_err": dmax, "rtol_needed_at_atol_2e-5": rt}), flush=True)
    tr.close()


def main():
    for batch in (64, 50, 128, 100, 256, 200):
        case(TOY_SPEC, batch, 21, 3, batch, 0.4, 1e-2, 0, groups="on", label="toy")
    for spec, name in ((MlpSpec(2, 10, 3, 1), "nl3"), (MlpSpec(2, 15, 5, 1), "h15"), (MlpSpec(2, 10, 5, 4), "out4")):
        for batch in (64, 128):
            case(spec, batch, 5, 9, 7 + batch, 0.3, 5e-3, 12, label=name)


if __name__ == "__main__":
    main()
