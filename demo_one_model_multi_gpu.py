#!/usr/bin/env python3
"""One model split by layers across several GPUs per process, data parallel on top.

Reference: demo_one_model_multi_gpu.py (MultiGPUModel: layers 0-1 on dev0, 2-4 on
dev1, activation moved with .to(dev1), DDP(device_ids=None) over processes,
launched with ``srun -n 2`` and TASKS_PER_NODE=1).

Here process p owns GPUs [p*K, p*K+K) (``--gpus_per_proc K``, default 2; the
reference's ``(rank*2) % local_world_size`` mapping put both stages on GPU 0 when
TASKS_PER_NODE=1).  Two engines:

* ``--engine fused`` (default): ``FusedLayerSplit`` -- every stage ONE persistent
  kernel resident on its GPU for a whole chunk of iterations; activations and
  gradients go to the neighbour stage as epoch-tagged granules stored straight into
  its GPU's receive buffer over xGMI; each stage's gradient is all-reduced over
  the DP ranks inside its kernel (per-device buckets); Adam / SGD fused.
* ``--engine module``: the autograd path -- stage kernels whose epilogue stores the
  activation into the next GPU, GPipe micro-batches in wavefront issue order
  (``--microbatches``), per-device DDP buckets reduced from grad-ready hooks
  (``LayerSplitDDP``).
``--microbatches M`` on the fused engine: M member workgroups per stage
(``csrc/split_lanes.hip``), member k of every stage one micro-batch of batch / M <= 64
samples flowing through the pipeline on its own links (GPipe in space: the M hand-off
chains run side by side), each stage's member gradients summed on chip before its one
optimizer step (GPipe's math: the full-batch gradient, one step per iteration).  The
default (1) picks ceil(batch / 64) members wherever the split-batch stages apply, else
the one-workgroup stages.  Configurations the persistent kernels do not cover
(batch > 256, other losses) fall back to ``module`` with a printed reason.  Both engines draw the
reference's exact DistributedSampler order by default (``--sampler torch``).
Checkpoint / resume (``--checkpoint_dir --checkpoint_every --resume``) works for
both.  Launch with torchrun (``--torchrun``) or plain srun exactly like demo.py.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from argument_parser import build_parser  # noqa: E402
from distributed_training_pytorch_amd import _native as nat  # noqa: E402
from distributed_training_pytorch_amd.data.sampler import BatchIndexer, SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine import runner  # noqa: E402
from distributed_training_pytorch_amd.models.toy import ToyModel  # noqa: E402
from distributed_training_pytorch_amd.ops.loss import MSELoss  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig  # noqa: E402
from distributed_training_pytorch_amd.parallel import comm_util  # noqa: E402
from distributed_training_pytorch_amd.parallel.layer_split import (FusedLayerSplit, LayerSplitDDP,  # noqa: E402
                                                                   LayerSplitMLP)
from distributed_training_pytorch_amd.runtime import checkpoint  # noqa: E402
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


def _fused_reason(config, devs) -> str | None:
    """Why the persistent split engine cannot run this configuration (None: it can)."""
    if config.engine != "fused":
        return f"--engine {config.engine}"
    if devs[0].type != "cuda" or not nat.native_enabled():
        return "CPU run"
    if config.batch_size > 256:
        return "per-rank batch > 256 (one lane per sample)"
    if config.loss != "mse":
        return "the split stages implement the reference's MSE loss"
    return None


def _members(config, geom):
    """--microbatches M -> member workgroups per stage of the split-batch stages: M
    micro-batches of batch / M samples, at least ceil(batch / 64) (a member runs at most
    64); M = 1: "auto" (ceil(batch / 64) where the split-batch stages apply)."""
    if config.microbatches <= 1:
        return "auto"
    return max(config.microbatches, -(-geom.batch // 64))


def _ckpt_due(config, it):
    return bool(config.checkpoint_dir and config.checkpoint_every and it % config.checkpoint_every == 0)


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
    ds = ToyData(n=config.n_samples, seed=config.seed, rank=rank, per_rank=config.per_rank_data)
    geom = SamplerGeometry(n=config.n_samples, world=world, rank=rank, batch=config.batch_size,
                           distributed=config.dataloader == "distributed", seed=0)
    ocfg = OptimConfig(config.optimizer, config.lr, momentum=config.momentum, weight_decay=config.weight_decay)
    logger = MetricLogger(project=config.project, group="multi-gpu-per-node", log_dir=config.log_dir, rank=rank)
    faults = FaultInjector(config.fail_at_iter, config.fail_rank, rank)
    pbar = runner._progress(rank, config.iters, config)

    why = _fused_reason(config, devs)
    if why is None:
        try:
            eng = FusedLayerSplit(toy.spec, devs, ds.X, ds.Y, geom, ocfg, toy.flat_params.detach(), bounds,
                                  sampler=config.sampler,
                                  members=_members(config, geom))
        except (NotImplementedError, ValueError) as e:  # e.g. more micro-batches than the exchange serves
            why, eng = str(e), None
    if why is None:
        rank_print(rank, f"engine: fused layer split ({len(devs)} persistent stages, "
                         + (f"{eng.members} member workgroups each: micro-batches of "
                            f"{-(-geom.batch // eng.members)} samples)" if eng.members else "one workgroup each)"))
        summary = _run_fused(config, eng, geom, world, rank, logger, faults, pbar)
        summary["members"] = eng.members
    else:
        if config.engine == "fused":
            rank_print(rank, f"engine: module (autograd layer split): {why}")
        summary = _run_module(config, toy, devs, bounds, ds, geom, ocfg, world, rank, logger, faults, pbar)
    if pbar is not None:
        pbar.close()
    logger.finish()
    summary.update({"stages": len(devs), "microbatches": config.microbatches})
    rank_print(rank, "Finished")
    if rank == 0:
        print(f"[Process {rank}] summary: {summary}", flush=True)
    runner.teardown()
    return summary


def _run_fused(config, eng, geom, world, rank, logger, faults, pbar) -> dict:
    start = 0
    if config.resume and config.checkpoint_dir:
        st = checkpoint.load(config.checkpoint_dir)
        if st is not None:
            if st.get("engine") != "split-fused":
                raise RuntimeError(f"{config.checkpoint_dir} holds a {st.get('engine')!r} checkpoint")
            eng.load_state_dict(st)
            start = eng.t
            rank_print(rank, f"resumed from {config.checkpoint_dir} at iteration {start}")
            if pbar is not None:
                pbar.update(start)
    chunk = max(1, min(config.log_every, config.steps_per_launch))
    it = start
    pending = None
    last = float("nan")

    def process(p):
        nonlocal last
        it0, n, handle = p
        ls = handle.wait()
        # one block per launch (the reference logs the local loss every iteration,
        # demo_one_model_multi_gpu.py:129-130; this is the global mean, same key)
        logger.log_rows(list(range(it0, it0 + n)), ["loss/loss"], ls[:n])
        if n:
            last = ls[n - 1][0]
        if pbar is not None:
            pbar.update(n)

    t0 = time.perf_counter()
    while it < config.iters:
        n = min(chunk, config.iters - it)
        if faults.armed() and it <= config.fail_at_iter < it + n:
            n = config.fail_at_iter - it
        if n > 0:
            eng.train(n)
            handle = eng.losses_async(it, it + n)
            if pending is not None:
                process(pending)
            pending = (it, n, handle)
            it += n
        if pending is not None and (it >= config.iters or _ckpt_due(config, it) or
                                    (faults.armed() and it >= config.fail_at_iter)):
            process(pending)
            pending = None
            eng.check_comm()
        faults.check(it)
        if _ckpt_due(config, it):
            eng.synchronize()
            checkpoint.save({**eng.state_dict(), "engine": "split-fused"}, config.checkpoint_dir, it)
            comm_util.barrier()
    if pending is not None:
        process(pending)
    eng.synchronize()
    dt = time.perf_counter() - t0
    if config.check_replicas:
        check_replicas(eng.flat_params_cpu())
    if config.checkpoint_dir:
        checkpoint.save({**eng.state_dict(), "engine": "split-fused"}, config.checkpoint_dir, it)
    eng.close()
    return {"final_loss": last, "iters": it, "engine": "split-fused",
            "samples_per_s": geom.batch * (it - start) * world / max(dt, 1e-9),
            "us_per_step": dt / max(it - start, 1) * 1e6}


def _run_module(config, toy, devs, bounds, ds, geom, ocfg, world, rank, logger, faults, pbar) -> dict:
    model = LayerSplitMLP(toy.spec, devs, bounds, config.microbatches, toy.flat_params.detach())
    ddp = LayerSplitDDP(model, comm=config.comm if config.comm in ("auto", "rccl", "xgmi") else "rccl")
    opts = [FlatOptimizer(p.data, p.grad, ocfg) for p in model.params]
    X, Y = ds.device_tensors(devs[0])
    Yl = Y.to(devs[-1])
    indexer = BatchIndexer(geom, devs[0], exact_torch=config.sampler == "torch")
    lossf = MSELoss()  # nn.MSELoss drop-in, one fused launch each way (ops/loss.py)
    start = 0
    if config.resume and config.checkpoint_dir:
        st = checkpoint.load(config.checkpoint_dir)
        if st is not None:
            if st.get("engine") != "split-module":
                raise RuntimeError(f"{config.checkpoint_dir} holds a {st.get('engine')!r} checkpoint")
            with torch.no_grad():
                for p, sp in zip(model.params, st["params"]):
                    p.copy_(sp)
            for o, so in zip(opts, st["optim"]):
                o.load_state_dict(so)
            start = int(st["iteration"])
            rank_print(rank, f"resumed from {config.checkpoint_dir} at iteration {start}")
            if pbar is not None:
                pbar.update(start)

    def save(it_done):
        checkpoint.save({"engine": "split-module", "params": [p.detach() for p in model.params],
                         "optim": [o.state_dict() for o in opts]}, config.checkpoint_dir, it_done)

    # losses stay on the last stage's GPU; reduced and logged once per log_every steps
    ring = LossRing(max(1, config.log_every), 1, devs[-1], world)
    last = float("nan")

    def flush():
        nonlocal last
        ddp.check_comm()
        for step, (v,) in ring.flush():
            if rank == 0:
                # the reference logs the local loss (demo_one_model_multi_gpu.py:129-130); this is the global mean
                logger.log({"loss/loss": v}, step=step)
            last = v

    t0 = time.perf_counter()
    for it in range(start, config.iters):
        faults.check(it)
        i0 = indexer(it)
        x = X.index_select(0, i0)
        y = Yl.index_select(0, i0.to(devs[-1]))
        model.zero_grad()
        out = model(x)
        loss = lossf(out, y)
        loss.backward()  # per-device buckets reduced from the stages' grad-ready hooks
        ddp.finish()
        for o in opts:
            o.step()
        ring.put(it, loss)
        if ring.full():
            flush()
        if pbar is not None:
            pbar.update(1)
        if _ckpt_due(config, it + 1):
            flush()
            save(it + 1)
            comm_util.barrier()
    flush()
    for d in set(devs):
        if d.type == "cuda":
            torch.cuda.synchronize(d)
    dt = time.perf_counter() - t0
    if config.check_replicas:
        check_replicas(model.flat_params_cpu())
    if config.checkpoint_dir:
        save(config.iters)
    ddp.close()
    return {"final_loss": last, "iters": config.iters, "engine": "split-module",
            "samples_per_s": geom.batch * (config.iters - start) * world / max(dt, 1e-9)}


if __name__ == "__main__":
    main()
