"""Do two persistent split-stage kernels on separate streams of ONE GPU run at the same
time?  python scripts/diag_split_streams.py MODE  (MODE: per_device | cumask | torch | prio).  Prints one JSON line: whether stage 0's link timed out, and the per-stage launch
times; run it under rocprofv3 --kernel-trace to see each dispatch's queue and start/end."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd import _native as nat  # noqa: E402
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import OptimConfig  # noqa: E402
from distributed_training_pytorch_amd.parallel.layer_split import FusedLayerSplit  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "cumask"
    dev = torch.device("cuda", 0)
    ds = ToyData(n=512, seed=2)
    geom = SamplerGeometry(n=512, batch=256, seed=1)
    init = torch.randn(TOY_SPEC.P, generator=torch.Generator().manual_seed(0)) * 0.4
    eng = FusedLayerSplit(TOY_SPEC, [dev, dev], ds.X, ds.Y, geom, OptimConfig(lr=1e-3), init,
                          launch="per_device" if mode == "per_device" else "per_stage", timeout_us=200_000)
    if mode == "cumask":
        eng.streams = {k: nat.cu_masked_stream(dev, [2 * k, 2 * k + 1]) for k in eng.streams}
    elif mode == "torch":
        eng.streams = {k: torch.cuda.Stream(device=dev) for k in eng.streams}
    elif mode == "prio":
        eng.streams = {k: torch.cuda.Stream(device=dev, priority=-1 if k else 0) for k in eng.streams}
    t0 = time.perf_counter()
    eng.train(3)
    eng._join()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    status = [st[:4].tolist() for st in eng.status]  # per stage: link timeout flag / epoch, DP flag / epoch
    print(json.dumps({"mode": mode, "status": status, "seconds": round(dt, 4),
                      "streams": {str(k): hex(s.cuda_stream) for k, s in eng.streams.items()}}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
