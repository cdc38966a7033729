#!/usr/bin/env python3
"""One model split by layers across several GPUs per process, data parallel on top.

Reference: demo_one_model_multi_gpu.py (MultiGPUModel: layers 0-1 on dev0, 2-4 on
dev1, activation moved with .to(dev1), DDP(device_ids=None) over processes,
launched with ``srun -n 2`` and TASKS_PER_NODE=1).

Here process p owns GPUs [p*K, p*K+K) (``--gpus_per_proc K``, default 2; the
reference's ``(rank*2) % local_world_size`` mapping put both stages on GPU 0 when
TASKS_PER_NODE=1).  Stage kernels hand activations to the next GPU by peer stores
over xGMI; ``--microbatches M`` turns the split into a GPipe pipeline.  Launch
with torchrun (``--torchrun``) or plain srun exactly like demo.py.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from argument_parser import build_parser  # noqa: E402
from distributed_training_pytorch_amd.data.sampler import BatchIndexer, SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine import runner  # noqa: E402
from distributed_training_pytorch_amd.models.toy import ToyModel  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig  # noqa: E402
from distributed_training_pytorch_amd.parallel.layer_split import LayerSplitDDP, LayerSplitMLP  # noqa: E402
from distributed_training_pytorch_amd.runtime.errors import FaultInjector, check_replicas, record  # noqa: E402
from distributed_training_pytorch_amd.utils.logging import LossRing, MetricLogger, rank_print  # noqa: E402


def get_args(argv=None):
    p = build_parser("layer-split model parallel + DDP demo")
    p.add_argument("--gpus_per_proc", type=int, default=2, help="pipeline stages (GPUs) per process")
    p.add_argument("--microbatches", type=int, default=1, help="GPipe micro-batches (1 = plain layer split)")
    p.add_argument("--split", type=str, default=None, help="layer ranges per stage, e.g. '0-1,2-4'")
    p.add_argument("--allow_shared_gpu", action="store_true",
                   help="map stages onto fewer visible GPUs (round robin) instead of failing")
    return p.parse_args(argv)


def stage_devices(config, env, device):
    K = config.gpus_per_proc
    if device.type == "cpu":
        return [torch.device("cpu")] * K
    n = torch.cuda.device_count()
    first = env.local_rank * K
    if first + K > n:
        if not config.allow_shared_gpu:
            raise RuntimeError(f"local rank {env.local_rank} needs GPUs {first}..{first + K - 1}, {n} visible "
                               "(use --allow_shared_gpu to co-locate stages)")
        return [torch.device("cuda", (first + s) % n) for s in range(K)]
    return [torch.device("cuda", first + s) for s in range(K)]


@record
def main(argv=None):
    config = get_args(argv)
    if config.dry_run:
        os.environ["WANDB_MODE"] = "dryrun"
    K = config.gpus_per_proc
    # the process binds its FIRST stage GPU; the others are addressed explicitly
    share = config.allow_shared_gpu and torch.cuda.is_available() and torch.cuda.device_count() < K
    env, device, rank, world = runner.setup(config, gpus_per_proc=1 if share else K)
    devs = stage_devices(config, env, device)
    rank_print(rank, f"stage devices: {[str(d) for d in devs]}")
    torch.manual_seed(config.seed)
    toy = ToyModel(hidden=config.hidden, depth=config.depth)
    bounds = None
    if config.split:
        bounds = [tuple(int(v) for v in r.split("-")) for r in config.split.split(",")]
    model = LayerSplitMLP(toy.spec, devs, bounds, config.microbatches, toy.flat_params.detach())
    ddp = LayerSplitDDP(model)
    opts = [FlatOptimizer(p.data, p.grad, OptimConfig(config.optimizer, config.lr, momentum=config.momentum))
            for p in model.params]
    ds = ToyData(n=config.n_samples, seed=config.seed, rank=rank, per_rank=config.per_rank_data)
    X, Y = ds.device_tensors(devs[0])
    Yl = Y.to(devs[-1])
    geom = SamplerGeometry(n=config.n_samples, world=world, rank=rank, batch=config.batch_size,
                           distributed=config.dataloader == "distributed", seed=0)
    indexer = BatchIndexer(geom, devs[0], exact_torch=config.sampler == "torch")
    logger = MetricLogger(project=config.project, group="multi-gpu-per-node", log_dir=config.log_dir, rank=rank)
    faults = FaultInjector(config.fail_at_iter, config.fail_rank, rank)
    lossf = torch.nn.MSELoss()
    pbar = runner._progress(rank, config.iters, config)
    # losses stay on the last stage's GPU; reduced and logged once per log_every steps
    ring = LossRing(max(1, config.log_every), 1, devs[-1], world)
    last = float("nan")

    def flush():
        nonlocal last
        for step, (v,) in ring.flush():
            if rank == 0:
                # the reference logs the local loss (demo_one_model_multi_gpu.py:129-130); this is the global mean
                logger.log({"loss/loss": v}, step=step)
            last = v

    t0 = time.perf_counter()
    for it in range(config.iters):
        faults.check(it)
        i0 = indexer(it)
        x = X.index_select(0, i0)
        y = Yl.index_select(0, i0.to(devs[-1]))
        model.zero_grad()
        out = model(x)
        loss = lossf(out, y)
        loss.backward()
        ddp.allreduce_grads()
        for o in opts:
            o.step()
        ring.put(it, loss)
        if ring.full():
            flush()
        if pbar is not None:
            pbar.update(1)
    flush()
    for d in set(devs):
        if d.type == "cuda":
            torch.cuda.synchronize(d)
    dt = time.perf_counter() - t0
    if pbar is not None:
        pbar.close()
    if config.check_replicas:
        check_replicas(model.flat_params_cpu())
    logger.finish()
    summary = {"final_loss": last, "iters": config.iters, "stages": len(devs),
               "microbatches": config.microbatches,
               "samples_per_s": geom.batch * config.iters * world / max(dt, 1e-9)}
    rank_print(rank, "Finished")
    if rank == 0:
        print(f"[Process {rank}] summary: {summary}", flush=True)
    runner.teardown()
    return summary


if __name__ == "__main__":
    main()
