"""The demo training loop shared by demo.py and demo_assume_started_with_mpiexec.py.

Reference: ``demo.py:19-137`` / ``demo_assume_started_with_mpiexec.py:29-127``:
two ToyModels (X, Y) trained on ToyData with DDP + Adam + MSE for 1000
iterations, the global mean loss of each model reduced every iteration and
logged by rank 0 (``loss/lossX``, ``loss/lossY``), tqdm on rank 0, rank-prefixed
status prints.

Engines (``--engine``):
* ``fused``  -- FusedTrainer: the whole iteration in one kernel (or one persistent
                kernel for many iterations); gradient all-reduce in-kernel over
                xGMI or through RCCL; losses read lazily from a device ring.
* ``module`` -- nn.Module path: ModelBank (both models in one flat buffer) with fused
                per-op kernels, FlatDDP (bucketed RCCL all-reduce overlapped with
                backward), FlatOptimizer (one Adam launch for both models).
* ``stock``  -- plain PyTorch eager DDP, the reference loop verbatim (baseline).
"""
from __future__ import annotations

import contextlib
import datetime
import os
import socket
import time

import torch
import torch.distributed as dist

from ..data.sampler import BatchIndexer, SamplerGeometry
from ..data.toy_data import ToyData
from ..ops.gather import gather_rows2, gather_rows2_ring, gather_rows2_sampler, ring_gather_ok
from ..ops.loss import MSELoss
from ..ops.mlp import ParamBackwardFusion
from ..ops.optim import OptimConfig
from ..parallel import comm_util
from ..runtime import bootstrap, checkpoint
from ..runtime.errors import FaultInjector, check_replicas
from ..utils.logging import LossRing, MetricLogger, rank_print
from ..utils.profiling import PhaseTimer
from ..utils.profiling import enabled as trace_enabled


def setup(config, launcher: str | None = None, gpus_per_proc: int = 1):
    """Discover ranks, bind the device, init the process group, print the reference's status lines."""
    bootstrap.configure_collective_env()
    if launcher == "mpi":
        env = bootstrap.detect(torchrun=False)
        if env.launcher == "single" and int(os.environ.get("WORLD_SIZE", "1")) > 1:
            raise RuntimeError("expected an MPI launch (OMPI_/PMI_ rank variables not found)")
    else:
        env = bootstrap.detect(torchrun=True if config.torchrun else None, use_node_rank=config.use_node_rank)
    device = bootstrap.bind_device(env, config.device, gpus_per_proc)
    backend = config.backend
    if device.type == "cpu" and backend == "nccl":
        backend = "gloo"
    bootstrap.init_process_group(env, backend, device, datetime.timedelta(minutes=config.timeout_min))
    rank, world = dist.get_rank(), dist.get_world_size()
    # the reference draws --seed independently in every process (argument_parser.py:17)
    # and never applies it; here rank 0's seed is broadcast so the data and model init
    # agree across ranks, and each worker gets seed + rank for its own randomness
    seed_t = torch.tensor([config.seed], dtype=torch.int64)
    comm_util.broadcast_(seed_t, 0)
    config.seed = int(seed_t.item())
    if rank == 0:
        rank_print(rank, f"World_size: {world}")
    rank_print(rank, f"Hello from {socket.gethostname()}")
    if env.local_rank == 0:
        n = torch.cuda.device_count() if torch.cuda.is_available() else 0
        rank_print(rank, f"Available devices on machine: {n}")
    base_seed = config.seed
    worker_seed = base_seed + rank
    rank_print(rank, f"Base seed: {base_seed} and  worker seed: {worker_seed}")
    torch.manual_seed(worker_seed)
    rank_print(rank, f"Using torchrun: {config.torchrun}")
    rank_print(rank, f"Using backend: {dist.get_backend()}")
    rank_print(rank, f"Launcher: {env.launcher}; device: {device}")
    return env, device, rank, world


def _dataset(config, rank):
    return ToyData(n=config.n_samples, seed=config.seed, rank=rank, per_rank=config.per_rank_data,
                   classes=4 if config.loss == "ce" else 0)


def _geom(config, rank, world):
    return SamplerGeometry(n=config.n_samples, world=world, rank=rank, batch=config.batch_size,
                           shuffle=True, distributed=config.dataloader == "distributed", seed=0)


def _compute_dtype(config) -> torch.dtype:
    return torch.bfloat16 if getattr(config, "precision", "fp32") == "bf16" else torch.float32


def _fused_supported(config) -> bool:
    from .. import _native as nat
    from ..ops.mlp import MlpSpec

    spec = MlpSpec(2, config.hidden, config.depth + 2, 4 if config.loss == "ce" else 1)
    if _compute_dtype(config) == torch.bfloat16:
        try:
            return bool(nat.load().dtp_mlp_train_bf16_supported(*spec.key[:4]))
        except nat.NativeUnavailable:
            return False
    return spec.native_supported()


def _optim(config) -> OptimConfig:
    return OptimConfig(config.optimizer, config.lr, momentum=config.momentum, weight_decay=config.weight_decay)


def _progress(rank, total, config):
    if rank != 0 or config.no_progress:
        return None
    try:
        from tqdm import tqdm

        return tqdm(total=total, desc="Iteration")
    except ImportError:  # pragma: no cover
        return None


def train(config, env, device, rank, world, group: str = "base-demo") -> dict:
    logger = MetricLogger(project=config.project, group=group, log_dir=config.log_dir, rank=rank,
                          config={k: v for k, v in vars(config).items() if isinstance(v, (int, float, str, bool))})
    faults = FaultInjector(config.fail_at_iter, config.fail_rank, rank)
    t_start = time.perf_counter()
    engine = config.engine
    if engine == "fused" and device.type == "cuda" and not _fused_supported(config):
        # widths / dtypes the fused step kernel is not instantiated for train through
        # nn.Modules whose Linears run on the MFMA GEMM (FlatDDP + FlatOptimizer)
        rank_print(rank, f"fused step kernel has no instance for hidden={config.hidden} depth={config.depth} "
                         f"precision={config.precision}: using the module engine (MFMA GEMM layers)")
        engine = "module"
    if engine == "fused":
        summary = _train_fused(config, device, rank, world, logger, faults)
    elif engine == "module":
        summary = _train_module(config, device, rank, world, logger, faults)
    else:
        summary = _train_stock(config, device, rank, world, logger, faults)
    wall = time.perf_counter() - t_start
    logger.finish()
    summary["wall_s"] = wall
    rank_print(rank, "Finished")
    return summary


# ----------------------------------------------------------------------------- fused engine
def _train_fused(config, device, rank, world, logger, faults) -> dict:
    from ..engine.fused_trainer import EngineConfig, FusedTrainer
    from ..models.toy import ToyModel
    from ..ops.mlp import MlpSpec

    ds = _dataset(config, rank)
    X, Y = ds.device_tensors(device)
    geom = _geom(config, rank, world)
    torch.manual_seed(config.seed)
    out_f = 4 if config.loss == "ce" else 1
    spec = MlpSpec(2, config.hidden, config.depth + 2, out_f)
    init = [ToyModel(hidden=config.hidden, depth=config.depth, out_features=out_f).flat_params.detach().clone()
            for _ in range(2)]
    ecfg = EngineConfig(comm=config.comm, launch=config.launch, steps_per_launch=config.steps_per_launch,
                        sampler=config.sampler, loss=config.loss, precision=config.precision)
    tr = FusedTrainer(spec, 2, X, Y, geom, _optim(config), ecfg, init_params=init)
    start = 0
    if config.resume and config.checkpoint_dir:
        st = checkpoint.load(config.checkpoint_dir)
        if st is not None:
            if st.get("engine", "fused") != "fused":
                raise RuntimeError(f"{config.checkpoint_dir} holds a {st['engine']!r}-engine checkpoint; "
                                   "resume it with the same engine")
            tr.load_state_dict(st)
            start = tr.t
            rank_print(rank, f"resumed from {config.checkpoint_dir} at iteration {start}")
    rank_print(rank, f"engine: fused ({tr.comm} comm, {config.launch} launch)")
    pbar = _progress(rank, config.iters, config)
    if pbar is not None and start:
        pbar.update(start)
    it = start
    chunk = max(1, min(config.log_every, config.steps_per_launch))
    timer = PhaseTimer(device)

    def ckpt_due(i):
        return bool(config.checkpoint_dir and config.checkpoint_every and i % config.checkpoint_every == 0)

    # Chunks are pipelined: chunk k+1 is queued on the GPU before the host logs chunk
    # k, whose losses (and the xGMI status word) were copied to pinned memory behind
    # it, so logging overlaps the next chunk instead of idling the GPU.
    pending = None

    def process(p):
        it0, n, handle = p
        with timer.phase("loss_readback"):
            ls = handle.wait_tensor()  # raises on a sticky xGMI timeout: never train on partial sums
        logger.log_rows(list(range(it0, it0 + n)), ["loss/lossX", "loss/lossY"], ls[:n])
        if pbar is not None:
            pbar.update(n)

    t0 = time.perf_counter()
    while it < config.iters:
        n = min(chunk, config.iters - it)
        if faults.armed() and it <= config.fail_at_iter < it + n:
            n = config.fail_at_iter - it
        if n > 0:
            with timer.phase("train_chunk"):
                tr.train(n)
            handle = tr.losses_async(it, it + n)
            if pending is not None:
                process(pending)
            pending = (it, n, handle)
            it += n
        if pending is not None and (it >= config.iters or ckpt_due(it) or
                                    (faults.armed() and it >= config.fail_at_iter)):
            process(pending)
            pending = None
        faults.check(it)
        if ckpt_due(it):
            tr.synchronize()
            checkpoint.save({**tr.state_dict(), "engine": "fused", "config": vars(config)},
                            config.checkpoint_dir, it)
            # the other ranks wait for rank 0's write on the host (process-group
            # timeout), not inside the next launch's first in-kernel xGMI exchange,
            # whose bounded spin a slow checkpoint filesystem could outlast
            comm_util.barrier()
    if pending is not None:
        process(pending)
    tr.synchronize()
    dt = time.perf_counter() - t0
    if pbar is not None:
        pbar.close()
    if config.check_replicas:
        check_replicas(tr.params)
    if config.checkpoint_dir:
        checkpoint.save({**tr.state_dict(), "engine": "fused", "config": vars(config)}, config.checkpoint_dir, it)
    final = tr.losses(it - 1, it)[0].tolist() if it > 0 else [float("nan")] * 2
    samples = geom.batch * (it - start) * world
    tr.close()
    return {"final_loss": final, "iters": it, "samples_per_s": samples / max(dt, 1e-9), "engine": "fused",
            **({"phases": timer.summary()} if trace_enabled() else {})}


# ----------------------------------------------------------------------------- module engine
def _train_module(config, device, rank, world, logger, faults) -> dict:
    from ..models.bank import ModelBank
    from ..ops.optim import FlatOptimizer
    from ..parallel.ddp import FlatDDP

    ds = _dataset(config, rank)
    X, Y = ds.device_tensors(device)
    geom = _geom(config, rank, world)
    # batch indices on the device: the native sampler kernel, or the exact torch order
    # uploaded once per epoch (no per-step host index math or copies)
    indexer = BatchIndexer(geom, device, exact_torch=config.sampler == "torch")
    torch.manual_seed(config.seed)
    out_f = 4 if config.loss == "ce" else 1
    bank = ModelBank(2, hidden=config.hidden, depth=config.depth, out_features=out_f,
                     compute_dtype=_compute_dtype(config)).to(device)
    ddp = FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad,
                  comm=config.comm if config.comm in ("auto", "rccl", "xgmi") else "rccl")
    rank_print(rank, f"engine: module (FlatDDP over {ddp.comm})")
    from .graph_step import CapturedStep
    opt = FlatOptimizer(bank.flat, bank.flat_grad, _optim(config))
    lossf = torch.nn.CrossEntropyLoss() if config.loss == "ce" else MSELoss()  # fused drop-in (ops/loss.py)
    start = 0
    if config.resume and config.checkpoint_dir:
        st = checkpoint.load(config.checkpoint_dir)
        if st is not None:
            if st.get("engine") != "module":
                raise RuntimeError(f"{config.checkpoint_dir} holds a {st.get('engine', 'fused')!r}-engine "
                                   "checkpoint; resume it with the same engine")
            with torch.no_grad():
                bank.flat.copy_(st["params"].to(bank.flat.dtype))
            opt.load_state_dict(st["optim_state"])
            start = int(st["iteration"])
            rank_print(rank, f"resumed from {config.checkpoint_dir} at iteration {start}")

    def _save(it_done):
        checkpoint.save({"engine": "module", "params": bank.flat.detach(), "optim_state": opt.state_dict(),
                         "config": vars(config)}, config.checkpoint_dir, it_done)

    pbar = _progress(rank, config.iters, config)
    if pbar is not None and start:
        pbar.update(start)
    timer = PhaseTimer(device)
    t0 = time.perf_counter()
    # per-step losses stay on the device; the global means are reduced and logged once
    # per log_every steps (one all-reduce of the chunk, one host sync), with the same
    # per-step values and keys as the reference's per-step gloo reduce + wandb.log
    ring = LossRing(max(1, config.log_every), 2, device, world)
    last = [float("nan")] * 2

    def _flush(wait: bool = True):
        nonlocal last
        # check the sticky xGMI timeout word at every log point (one host read, with
        # several ranks only), so a timed-out exchange stops the run there instead of
        # training on partial sums until the end
        ddp.check_comm()
        for step, (vx, vy) in ring.flush(wait):
            if rank == 0:
                logger.log({"loss/lossX": vx}, step=step, commit=False)
                logger.log({"loss/lossY": vy}, step=step)
            last = [vx, vy]

    # the batch indices of the current iteration, refreshed before each step (the
    # captured graph reads this static buffer)
    idx_static = torch.zeros(geom.batch, dtype=torch.int64, device=device)

    # the flat optimizer zeroes the gradient it consumed, so the next step's zero_grad fill
    # is skipped (reset whenever a capture is abandoned: its zeroing never ran)
    grads_clean = [False]
    xb = {}
    fuse_opt = world == 1 and os.environ.get("DTP_MODULE_FUSE_OPT", "1") != "0"
    seed = _Seeds(device)
    loss_log = os.environ.get("DTP_MODULE_LOSSLOG", "1") != "0"  # A/B: the separate ring put
    sync_flush = os.environ.get("DTP_MODULE_SYNC_FLUSH", "0") == "1"  # A/B: the blocking flush

    def step_body(size):
        with timer.phase("data"):
            if size not in xb:
                xb[size] = (torch.empty(size, X.shape[1], device=device), torch.empty(size, Y.shape[1], device=device))
            x, y = xb[size]
            if samp_cfg is not None:  # indices from the device sampler, step cursor advanced on the device
                gather_rows2_sampler(X, Y, samp_cfg, samp_cursor, x, y)
            elif epoch_ring is not None:  # indices from the device epoch ring, cursor advanced on the device
                gather_rows2_ring(X, Y, epoch_ring, geom.batch, geom.steps_per_epoch, x, y)
            else:
                gather_rows2(X, Y, idx_static[:size], x, y)  # both tensors in one launch
            if config.loss == "ce":
                y = y.view(-1).long()
        if not grads_clean[0]:
            bank.zero_grad()
        logged = False
        with timer.phase("forward"):
            ox, oy = ddp(x)  # both models' forwards in one launch (ModelBank.forward)
            if isinstance(lossf, MSELoss):
                # both losses, their sum and the loss-log row in one launch
                lx, ly, lsum = lossf.pair(ox, oy, y, log=ring.device_log() if loss_log else None)
                logged = loss_log
            else:
                lx, ly = lossf(ox, y), lossf(oy, y)
                lsum = lx + ly
        # one rank: both models' stage backwards and the flat Adam over both as ONE launch
        # (ParamBackwardFusion; nothing reads the gradient in between without an all-reduce)
        with (ParamBackwardFusion() if fuse_opt else contextlib.nullcontext()) as fus:
            with timer.phase("backward+allreduce"):
                # independent models: one backward, one bucketed all-reduce; the seed from a
                # cached tensor of ones (autograd's own is a fill launch per step)
                lsum.backward(seed.get(lsum.shape) if device.type == "cuda" else None)
            with timer.phase("optimizer"):
                grads_clean[0] = opt.step(zero_grad=True, fused=fus.take() if fus is not None else None)
        if not logged:
            ring.put_device(lx, ly)

    def _abort():
        grads_clean[0] = False
        ddp.reset_hooks()

    # hipGraph replay of the whole iteration (engine/graph_step.py) where it can be
    # captured: one rank, xGMI buckets (device-side exchange epochs) or RCCL buckets;
    # not gloo-staged buckets (host-driven)
    graphable = device.type == "cuda" and config.launch != "eager" and not trace_enabled() and ddp.graph_safe()
    stepper = CapturedStep(step_body, device, enabled=graphable, on_abort=_abort)
    # the device epoch ring {cursor, the epoch's indices} of the replayed step's gather: one
    # fill per epoch instead of an index copy per step (DTP_MODULE_RING=0: the copies, A/B)
    # better still, the step's indices computed on the device by the engine's own sampler
    # (sampler.h, reading the device permutation ring for DistributedSampler's exact order):
    # no host index work per epoch either (DTP_MODULE_RING=epoch: the epoch ring, A/B)
    epoch_ring, ring_epoch = None, None
    samp_cfg, samp_cursor, perm_ring = None, None, None
    ring_mode = os.environ.get("DTP_MODULE_RING", "sampler")
    if graphable and ring_gather_ok(X, Y, geom.batch) and ring_mode == "sampler" and geom.batch <= 1024:
        perm_ring = indexer.permutation_ring()
        if perm_ring is not None or not indexer.needs_ring():
            samp_cfg = geom.to_native()
            if perm_ring is not None:
                perm_ring.native(samp_cfg)
            samp_cursor = torch.full((1,), start, dtype=torch.int64, device=device)
    if (samp_cfg is None and graphable and indexer.can_fill_epoch() and ring_gather_ok(X, Y, geom.batch)
            and ring_mode != "0"):
        epoch_ring = torch.zeros(1 + geom.steps_per_epoch * geom.batch, dtype=torch.int64, device=device)
        epoch_ring[0] = geom.batch_pos(start)[1] // geom.batch  # the cursor: the first step's batch in its epoch
    # steady-state clock (the summary's steady_samples_per_s): from the end of step
    # steady_from on -- the first kernels' code-object loads, the warm-up runs and the
    # graph captures fall before it (they are a fixed cost that dominates short runs and
    # varies by box); synchronised at both ends
    steady_from = start + min(50, (config.iters - start) // 2)
    t_steady = None
    for it in range(start, config.iters):
        if it == steady_from and device.type == "cuda":
            torch.cuda.synchronize(device)
            t_steady = time.perf_counter()
        faults.check(it)
        size = geom.batch_size_at(it)
        if samp_cfg is not None:
            ep = geom.batch_pos(it)[0]
            if perm_ring is not None and ep != ring_epoch:  # resident before the replay that reads it
                perm_ring.ensure(ep, ep)
                ring_epoch = ep
        elif epoch_ring is not None:
            ep = geom.batch_pos(it)[0]
            if ep != ring_epoch:  # stream-ordered after the last replay that read the old epoch
                indexer.epoch_into(ep, epoch_ring[1:1 + geom.num_samples])
                ring_epoch = ep
        else:
            idx_static[:size].copy_(indexer(it))
        stepper.run(size)
        ring.mark(it)
        if ring.full():
            with timer.phase("loss_reduce"):
                _flush(wait=sync_flush)  # no device sync: the rows are logged when they arrive
        if pbar is not None:
            pbar.update(1)
        if config.checkpoint_dir and config.checkpoint_every and (it + 1) % config.checkpoint_every == 0:
            _flush()
            _save(it + 1)
            # as in the fused engine: the other ranks wait for rank 0's write on the host
            # (process-group timeout), not inside the next step's bounded xGMI spin
            comm_util.barrier()
    _flush()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    ddp.check_comm()
    t_end = time.perf_counter()
    dt = t_end - t0
    steady = None
    if t_steady is not None and config.iters > steady_from:
        steady = geom.batch * (config.iters - steady_from) * world / max(t_end - t_steady, 1e-9)
    if pbar is not None:
        pbar.close()
    if config.check_replicas:
        check_replicas(bank.flat)
    if config.checkpoint_dir:
        _save(config.iters)
    return {"final_loss": last, "iters": config.iters,
            "samples_per_s": geom.batch * (config.iters - start) * world / max(dt, 1e-9),
            "steady_samples_per_s": steady, "engine": "module",
            "graph_replays": stepper.replays,
            **({"phases": timer.summary()} if trace_enabled() else {})}


class _Seeds:
    """d loss / d loss: one cached tensor of ones per shape (a captured step replays it)."""

    def __init__(self, device):
        self.device = device
        self._t: dict = {}

    def get(self, shape):
        t = self._t.get(tuple(shape))
        if t is None:
            t = self._t[tuple(shape)] = torch.ones(shape, dtype=torch.float32, device=self.device)
        return t


# ----------------------------------------------------------------------------- stock engine
def _train_stock(config, device, rank, world, logger, faults) -> dict:
    from ..baselines.stock import StockLoop

    ds = _dataset(config, rank)
    loop = StockLoop(ds, device, batch=config.batch_size, seed=config.seed)
    pbar = _progress(rank, config.iters, config)
    timer = PhaseTimer(device)
    t0 = time.perf_counter()
    for it in range(config.iters):
        faults.check(it)
        with timer.phase("step"):
            loop.step()
        if rank == 0:
            logger.log({"loss/lossX": loop.last[0]}, step=it, commit=False)
            logger.log({"loss/lossY": loop.last[1]}, step=it)
        if pbar is not None:
            pbar.update(1)
    dt = time.perf_counter() - t0
    if pbar is not None:
        pbar.close()
    loop.close()
    return {"final_loss": list(loop.last), "iters": config.iters,
            "samples_per_s": loop.samples * world / max(dt, 1e-9), "engine": "stock",
            **({"phases": timer.summary()} if trace_enabled() else {})}


def teardown():
    if dist.is_initialized():
        comm_util.barrier()
        dist.destroy_process_group()
