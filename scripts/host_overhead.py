"""Host-side cost of one engine call (the bench's timed region is one train(K) call plus a
synchronize): FusedTrainer.train(1) vs the bare native call, and an idle synchronize."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd import _native as nat  # noqa: E402
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine.fused_trainer import FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402


def main():
    nat.set_wait_mode("spin")
    dev = torch.device("cuda", 0)
    X, Y = ToyData(seed=0).device_tensors(dev)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=256))
    tr.train(50)
    torch.cuda.synchronize()
    n = 200
    res = {}
    t0 = time.perf_counter()
    for _ in range(n):
        tr.train(1)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    res["train1_host_us"] = 1e6 * (t1 - t0) / n
    e = tr._engine_handle()
    run = tr._engine_run
    s = nat.raw_stream(0)
    t0 = time.perf_counter()
    for _ in range(n):
        run(e, 1, tr.t, s)
        tr.t += 1
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    res["native_call_host_us"] = 1e6 * (t1 - t0) / n
    t0 = time.perf_counter()
    for _ in range(n):
        torch.cuda.synchronize(dev)
    res["idle_sync_us"] = 1e6 * (time.perf_counter() - t0) / n
    # one call + synchronize, back to back (the bench's timed region at K = 1)
    ws = []
    for _ in range(50):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        tr.train(1)
        torch.cuda.synchronize(dev)
        ws.append(1e6 * (time.perf_counter() - t0))
    ws.sort()
    res["train1_plus_sync_us_median"] = ws[len(ws) // 2]
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
