"""What a launch + completion costs the host at all, against the bench's K = 20 call.

Medians over 300 repetitions, each bracketed like bench.py's timed region
(synchronize, perf_counter, work, synchronize, perf_counter), on a pool stream:
  sync          -- torch.cuda.synchronize() with nothing queued
  torch_tiny    -- one 1-element torch kernel + synchronize
  train_k       -- FusedTrainer.train(k) (the split-batch step, batch 256) + synchronize
GPU only; prints one JSON line."""
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
from distributed_training_pytorch_amd.engine.fused_trainer import FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.models.toy import ToyModel  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402


def med(fn, reps=300, pre_sync=None):
    """pre_sync: called before the closing torch.cuda.synchronize (e.g. the stream's own
    synchronize: whether waiting on the stream first shortens the device-wide wait)."""
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        if pre_sync is not None:
            pre_sync()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    return round(statistics.median(ts), 2)


def main():
    dev = torch.device("cuda", 0)
    nat.set_wait_mode("spin") if hasattr(nat, "set_wait_mode") else None
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        x = torch.zeros(1, device=dev)
        X, Y = ToyData(n=512, seed=0).device_tensors(dev)
        torch.manual_seed(0)
        init = [ToyModel().flat_params.detach().clone() for _ in range(2)]
        tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=256, seed=0), init_params=init)
        for _ in range(20):
            tr.train(1)
        out = {"sync": med(lambda: None), "torch_tiny": med(lambda: x.add_(1.0))}
        for k in (1, 20, 200):
            out[f"train_{k}"] = med(lambda k=k: tr.train(k), reps=100 if k == 200 else 300)
        out["train_20_stream_sync_first"] = med(lambda: tr.train(20), pre_sync=s.synchronize)
        ev = torch.cuda.Event()
        out["train_20_event_sync_first"] = med(lambda: (tr.train(20), ev.record(s)), pre_sync=ev.synchronize)
        out["train_20_again"] = med(lambda: tr.train(20))
        # the host's side alone: time to return from train(20) (enqueue), and from the bare
        # native call it ends in (same arguments, no Python bookkeeping)
        def host_only(fn, reps=300):
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                ts.append((time.perf_counter() - t0) * 1e6)
                torch.cuda.synchronize()
            return round(statistics.median(ts), 2)

        out["host_train_20"] = host_only(lambda: tr.train(20))
        e, run, di = tr._engine_handle(), tr._engine_run, tr._dev_index

        def bare():
            run(e, 20, tr.t, nat.raw_stream(di))
            tr.t += 20
        out["host_bare_engine_run_20"] = host_only(bare)
        tr.close()
    out["per_step_slope_us"] = round((out["train_200"] - out["train_20"]) / 180, 3)
    out["fixed_us"] = round(out["train_20"] - 20 * out["per_step_slope_us"], 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
