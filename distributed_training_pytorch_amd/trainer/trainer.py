"""Trainer: a PyTorch-Lightning-1.5-compatible training driver (the parts the reference
uses: ``pl.Trainer(gpus, num_nodes, max_steps, precision=32, accelerator='gpu',
log_every_n_steps, strategy='ddp')`` + ``fit``, ``demo_pytorch_lightning.py:57-62``).

Semantics kept from PL 1.5.10:
* cluster environment: SLURM (SLURM_PROCID/LOCALID/NODEID/NTASKS + MASTER_ADDR/PORT)
  or torchrun env, else one process; backend from ``PL_TORCH_DISTRIBUTED_BACKEND``;
* ``strategy='ddp'``: rank-0 parameter broadcast, gradient averaging on every
  backward (FlatDDP: flat buffer, bucketed RCCL all-reduce overlapped with the
  backward, unused-parameter tolerant), DistributedSampler auto-injected into a
  sampler-less DataLoader;
* several optimizers: per batch, for each optimizer: toggle (only its params
  require grad), training_step(batch, batch_idx, optimizer_idx), backward, step,
  zero_grad; ``global_step`` advances once per BATCH (PL 1.5, not 1.6+);
* ``log_every_n_steps`` (a float in the reference, 0.03125) is clamped to an int >= 1;
* default checkpointing: ``{root}/lightning_logs/version_N/checkpoints/
  epoch={e}-step={s}.ckpt`` at the end of training; CSV metrics alongside.
MI355X-first: a dataset exposing device tensors (``ToyData``) is gathered on the GPU
(no collation/pin-memory per batch), the model's layers run as fused HIP kernels.
"""
from __future__ import annotations

import contextlib
import ctypes
import csv
import datetime
import math
import os
import time
from pathlib import Path

import torch
import torch.distributed as dist

from .. import _native as nat
from ..data.sampler import SamplerGeometry, torch_distributed_indices
from ..ops.mlp import ParamBackwardFusion
from ..parallel import comm_util
from ..parallel.ddp import FlatDDP
from ..runtime import bootstrap
from ..utils.logging import rank_print


class CSVLogger:
    def __init__(self, root: str, rank: int):
        self.rank = rank
        self.dir = None
        if rank != 0:
            return
        base = Path(root) / "lightning_logs"
        base.mkdir(parents=True, exist_ok=True)
        n = 0
        while (base / f"version_{n}").exists():
            n += 1
        self.dir = base / f"version_{n}"
        self.dir.mkdir(parents=True)
        self._f = open(self.dir / "metrics.csv", "w", newline="")
        self._w = None

    def log(self, step: int, metrics: dict):
        if self.dir is None:
            return
        row = {"step": step, **{k: float(v) for k, v in metrics.items()}}
        if self._w is None:
            self._w = csv.DictWriter(self._f, fieldnames=list(row.keys()), extrasaction="ignore")
            self._w.writeheader()
        self._w.writerow(row)

    def log_rows(self, steps, names, rows):
        """One row per (step, values): ``names[i]`` = ``values[i]`` plus their sum as
        ``train_loss`` (the fused engine's per-launch loss block, written in one call)."""
        if self.dir is None or not steps:
            return
        if self._w is None:
            self.log(steps[0], {**dict(zip(names, rows[0])), "train_loss": sum(rows[0])})
            steps, rows = steps[1:], rows[1:]
        if list(self._w.fieldnames) == ["step", *names, "train_loss"]:
            # the csv module's own text for these rows (floats as repr, excel's \r\n), formatted
            # directly: ~5 us per row through DictWriter made the host, not the GPU, the
            # limit of the fused engine's every-step logging (a step is ~3 us)
            self._f.write("".join(f"{s},{','.join(map(repr, r))},{sum(r)!r}\r\n" for s, r in zip(steps, rows)))
            return
        self._w.writerows({"step": s, **dict(zip(names, r)), "train_loss": sum(r)} for s, r in zip(steps, rows))

    def log_block(self, step0: int, every: int, names, rows: torch.Tensor, first: int = 0) -> None:
        """``log_rows`` for a host tensor of loss rows ([n, len(names)] fp32): rows
        ``first, first + every, ...`` at steps ``step0, step0 + every, ...``, formatted
        natively (``csrc/host_log.hip``, the csv module's exact text, ~0.5 us per row
        instead of ~5) when the library is loaded."""
        if self.dir is None:
            return
        sel = rows[first::every]
        n = sel.shape[0]
        if n == 0:
            return
        if self._w is None:
            self._w = csv.DictWriter(self._f, fieldnames=["step", *names, "train_loss"], extrasaction="ignore")
            self._w.writeheader()
        r = rows.detach()
        if (nat.native_enabled() and os.environ.get("DTP_NATIVE_LOG", "1") != "0"
                and r.device.type == "cpu" and r.dtype == torch.float32 and r.dim() == 2
                and r.is_contiguous() and r.shape[1] == len(names)
                and list(self._w.fieldnames) == ["step", *names, "train_loss"]):
            lib = nat.load()
            cap = lib.dtp_format_loss_rows_bound(len(names), n)
            buf = ctypes.create_string_buffer(cap)
            m = lib.dtp_format_loss_rows(nat.ptr(r), len(names), first, n, every, step0, every, 1, buf, cap)
            if m >= 0:
                self._f.write(buf.raw[:m].decode("ascii"))
                return
        self.log_rows(list(range(step0, step0 + n * every, every)), names, sel.tolist())

    def flush(self):
        if self.dir is not None:
            self._f.flush()

    def close(self):
        if self.dir is not None:
            self._f.close()


class _DeviceBatches:
    """Device-resident replacement for DataLoader(DistributedSampler(ds), batch_size).

    With ``use_ring()`` (a GPU and batches one workgroup gathers, the Trainer's replayed
    step) the epoch's indices live in a device ring ``{cursor, indices}`` that the
    replayed step's gather reads and advances itself (``ops.gather.gather_rows2_ring``):
    one asynchronous upload from pinned memory per epoch -- none at all while the order
    does not change (one rank: no shuffle) -- instead of a pageable upload per epoch and
    an index copy per batch.  ``skip`` (set before iterating) is the number of leading
    batches the caller will not run (a mid-epoch resume): the cursor starts there."""

    def __init__(self, X, Y, batch, world, rank, shuffle, seed=0):
        self.X, self.Y = X, Y
        self.geom = SamplerGeometry(n=X.shape[0], world=world, rank=rank, batch=batch, shuffle=shuffle, seed=seed)
        self.epoch = 0
        self.skip = 0
        self.ring = None  # int64 [1 + steps * batch] on the device: cursor, then the epoch's indices
        self._ring_idx = None  # the indices the ring holds (host copy)
        self._ring_clean = False  # the last epoch ran to its end: cursor mod steps == 0

    def __len__(self):
        return self.geom.steps_per_epoch

    def set_epoch(self, e):
        self.epoch = e

    def use_ring(self) -> bool:
        from ..ops.gather import ring_gather_ok

        if os.environ.get("DTP_TRAINER_RING", "1") == "0":  # A/B switch: the per-batch index copy
            return False
        if self.ring is None and ring_gather_ok(self.X, self.Y, self.geom.batch):
            self.ring = torch.zeros(1 + len(self) * self.geom.batch, dtype=torch.int64, device=self.X.device)
        return self.ring is not None

    def __iter__(self):
        g = self.geom
        idx = torch_distributed_indices(g.n, g.world, g.rank, self.epoch, g.seed, g.shuffle)
        skip, self.skip = self.skip, 0
        if self.ring is not None:
            idx_h = torch.tensor(idx, dtype=torch.int64)
            if not (self._ring_clean and skip == 0 and self._ring_idx is not None
                    and torch.equal(idx_h, self._ring_idx)):
                host = torch.empty(self.ring.numel(), dtype=torch.int64, pin_memory=self.ring.is_cuda)
                host.zero_()
                host[0] = skip
                host[1:1 + idx_h.numel()] = idx_h
                self.ring.copy_(host, non_blocking=True)  # stream-ordered after the last epoch's gathers
                self._ring_idx = idx_h
            idx_t = self.ring[1:1 + idx_h.numel()]
        else:
            idx_t = torch.tensor(idx, device=self.X.device)
        self._ring_clean = False
        for b in range(len(self)):
            yield _DevBatch(self.X, self.Y, idx_t[b * g.batch:(b + 1) * g.batch], self)
        self._ring_clean = True


class _DevBatch:
    """One batch of ``_DeviceBatches``: the sample indices, gathered on demand.  A
    replayed step gathers inside its graph into the static batch buffers: from the
    epoch ring (nothing per batch on the host side) or from a static index buffer the
    caller refreshes (one small index copy per batch)."""

    __slots__ = ("X", "Y", "sel", "src")

    def __init__(self, X, Y, sel, src):
        self.X, self.Y, self.sel, self.src = X, Y, sel, src

    @property
    def ring(self):
        return self.src.ring

    def materialize(self):
        return [self.X[self.sel], self.Y[self.sel]]

    def gather_into(self, idx, out):
        # both tensors in ONE launch (two index_selects otherwise): each launch costs ~4 us in
        # the replayed step
        from ..ops.gather import gather_rows2, gather_rows2_ring

        if idx is None:
            g = self.src.geom
            gather_rows2_ring(self.X, self.Y, self.src.ring, g.batch, g.steps_per_epoch, out[0], out[1])
        else:
            gather_rows2(self.X, self.Y, idx, out[0], out[1])


_STEADY_AFTER = 10  # batches excluded from Trainer.steady_time


class _MetricRing:
    """Logged metrics of many steps, reduced and written in one go.

    PL logs (``self.log``) every ``log_every_n_steps`` batches -- every batch in the
    reference (``log_every_n_steps=0.03125``).  Reducing and printing each of those on
    the host costs a collective and a device->host sync per batch, which would stall
    the replayed step after every batch.  Instead each logged step's values are stacked
    into a device row, and every ``rows`` logged steps -- and before a checkpoint and at
    the end of ``fit`` -- the block is averaged over ranks with ONE all-reduce, copied to
    the host once and written to ``metrics.csv`` row by row -- without a device sync:
    a block's rows are written once its copy has arrived (``flush``).
    ``callback_metrics`` is the last row of the newest written block, so it trails the
    live step by less than 2 x ``rows`` logged steps during training and is exact after
    ``fit``.

    The stack itself is deferred: a logged step's tensors are kept (``pending``) until
    ``defer`` steps are waiting or the graph copy that wrote them (``owner``) is about to
    be replayed again (``release``), then all waiting rows are stacked in ONE launch --
    with the Trainer's ``graph_copies`` replayed graphs per batch shape, one stack per
    ``graph_copies`` batches instead of one per batch."""

    def __init__(self, trainer, logger, rows: int = 64, defer: int = 1):
        self.tr = trainer
        self.logger = logger
        self.rows = rows
        self.defer = max(1, int(defer))
        self.buf = None
        self.keys: list = []
        self.steps: list = []
        self.pending: list = []  # (step, [tensors], owner)
        self._inflight: list = []  # (event, pinned rows, steps, keys) copied but not yet written
        self._sync_flush = os.environ.get("DTP_TRAINER_SYNC_FLUSH", "0") == "1"  # A/B: the blocking flush

    def push(self, step: int, logged: dict, owner=None) -> None:
        keys = list(logged.keys())
        if not keys:
            return
        if self.buf is None or keys != self.keys:
            self.flush()
            self.keys = keys
            self.buf = torch.empty(self.rows, len(keys), dtype=torch.float32, device=self.tr.device)
        self.pending.append((step, [v.detach() for v in logged.values()], owner))
        if len(self.pending) >= self.defer or len(self.steps) + len(self.pending) >= self.rows:
            self._stack_pending()
            if len(self.steps) == self.rows:
                self.flush(wait=self._sync_flush)

    def release(self, owner) -> None:
        """``owner``'s output tensors are about to be overwritten: stack what waits."""
        if any(o == owner for _, _, o in self.pending):
            self._stack_pending()

    def _stack_pending(self) -> None:
        if not self.pending:
            return
        n0, k = len(self.steps), len(self.pending)
        vals = [v.float().reshape(()) for _, vs, _ in self.pending for v in vs]
        torch.stack(vals, out=self.buf[n0:n0 + k].view(-1))
        self.steps.extend(st for st, _, _ in self.pending)
        self.pending = []

    def flush(self, wait: bool = True) -> None:
        """Reduce the block and start its copy to the host.  ``wait=False`` (the periodic
        flush inside training): no device sync -- the copy lands in pinned memory behind
        the queued batches and its rows are written at a later flush once it has arrived,
        so the replayed steps queued behind it keep the GPU busy while the host writes
        CSV.  ``wait=True`` (checkpoint, end of ``fit``): everything written now."""
        self._stack_pending()
        if self.steps:
            block = self.buf[:len(self.steps)]
            if self.tr.world_size > 1:
                comm_util.all_reduce_(block)
                block /= self.tr.world_size
            ev = None
            if block.is_cuda:
                host = torch.empty(block.shape, dtype=block.dtype, pin_memory=True)
                host.copy_(block, non_blocking=True)  # stream-ordered before the rows are reused
                ev = torch.cuda.Event()
                ev.record()
            else:
                host = block.clone()
            self._inflight.append((ev, host, self.steps, self.keys))
            self.steps = []
        while self._inflight and (wait or self._inflight[0][0] is None or self._inflight[0][0].query()):
            ev, host, steps, keys = self._inflight.pop(0)
            if ev is not None:
                ev.synchronize()
            rows = host.tolist()
            for step, vals in zip(steps, rows):
                self.logger.log(step, dict(zip(keys, vals)))
            self.logger.flush()
            self.tr.callback_metrics = dict(zip(keys, rows[-1]))


class Trainer:
    def __init__(self, gpus: int | None = None, num_nodes: int = 1, max_steps: int = -1, max_epochs: int | None = None,
                 precision: int = 32, accelerator: str | None = None, strategy: str | None = None,
                 log_every_n_steps: float = 50, default_root_dir: str | None = None,
                 enable_checkpointing: bool = True, enable_progress_bar: bool = True, seed: int | None = None,
                 use_graphs: bool = True, native_optimizers: bool = True, every_n_train_steps: int = 0,
                 engine: str = "auto", graph_copies: int | None = None, **unused):
        if precision in (32, "32", "32-true"):
            self.autocast_dtype = None
        elif precision in ("bf16", "bf16-mixed"):
            # PL: torch.autocast(bf16) around training_step; fp32 master weights and optimizer
            self.autocast_dtype = torch.bfloat16
        else:
            raise NotImplementedError(f"precision={precision!r}: supported are 32 and 'bf16'")
        self.precision = precision
        self.gpus = gpus
        self.num_nodes = num_nodes
        self.max_steps = -1 if max_steps is None else int(max_steps)  # PL 1.5: None = unbounded
        self.max_epochs = max_epochs if max_epochs is not None else (1000 if self.max_steps < 0 else None)
        self.accelerator = accelerator or ("gpu" if torch.cuda.is_available() and gpus else "cpu")
        self.strategy = strategy
        self.log_every_n_steps = max(1, int(log_every_n_steps))  # reference passes 0.03125
        self.root = default_root_dir or os.getcwd()
        self.enable_checkpointing = enable_checkpointing
        self.enable_progress_bar = enable_progress_bar
        self.seed = seed
        self.use_graphs = use_graphs  # replay each batch's optimizer steps as a hipGraph (GPU)
        # graphs captured per batch shape, replayed in turn: each keeps its logged outputs
        # until its next replay, so the metric rows are stacked once per `graph_copies` batches
        # (default 4; DTP_TRAINER_GRAPH_COPIES overrides the default, for A/Bs)
        if graph_copies is None:
            graph_copies = int(os.environ.get("DTP_TRAINER_GRAPH_COPIES", "4"))
        self.graph_copies = max(1, int(graph_copies))
        # run a plain torch Adam/SGD over a flat-buffer span as ONE flat-optimizer kernel (GPU)
        self.native_optimizers = native_optimizers
        self._flat_opts: list = []
        self._opt_zeroes = False  # the flat optimizers zero the gradient they consume (fit)
        # the backward's last stage kernel fused with the flat optimizer step (one rank);
        # DTP_TRAINER_FUSE_OPT=0 launches them separately (A/B)
        self._fuse_backward_opt = os.environ.get("DTP_TRAINER_FUSE_OPT", "1") != "0"
        self.graph_replays = 0
        self.global_step = 0
        self.current_epoch = 0
        self.callback_metrics: dict = {}
        self.checkpoint_path: str | None = None
        # ModelCheckpoint(every_n_train_steps=N): also save ``last.ckpt`` every N batches
        # (what a restarted job resumes from, fit(ckpt_path="last"))
        self.every_n_train_steps = int(every_n_train_steps or 0)
        # "auto": the fused train-step engine when the LightningModule declares its step
        # (``fused_spec``) and everything it needs matches; "module": always the
        # per-batch nn.Module path; "fused": the fused engine or an error
        if engine not in ("auto", "fused", "module"):
            raise ValueError(f"engine={engine!r}: auto, fused or module")
        self.engine = engine
        self.engine_used = "module"
        self.fused_refused: str | None = None  # why fused_spec() was not trusted (checked on the first batch)
        self._skip_batches = 0
        self._batch_in_epoch = 0
        self._log_dir = None

    # ------------------------------------------------------------------ distributed
    def _setup(self):
        bootstrap.configure_collective_env()  # before bind_device: HSA reads the IPC mode at its first touch
        env = bootstrap.detect()
        device = torch.device("cpu")
        if self.accelerator == "gpu" and torch.cuda.is_available():
            device = bootstrap.bind_device(env, "cuda")
        if self.strategy in ("ddp", "ddp_spawn", "ddp_find_unused_parameters_false") or env.world_size > 1:
            backend = os.environ.get("PL_TORCH_DISTRIBUTED_BACKEND", "nccl" if device.type == "cuda" else "gloo")
            bootstrap.init_process_group(env, backend, device, datetime.timedelta(minutes=60))
        self.env = env
        self.device = device
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        self.global_rank = dist.get_rank() if dist.is_initialized() else 0
        expected = (self.gpus or 1) * self.num_nodes
        if self.global_rank == 0 and dist.is_initialized() and self.world_size != expected:
            rank_print(0, f"note: world size {self.world_size} != gpus*num_nodes {expected}")

    def _loader(self, dl):
        ds = getattr(dl, "dataset", dl)
        bs = getattr(dl, "batch_size", None) or 1
        if hasattr(ds, "device_tensors"):
            X, Y = ds.device_tensors(self.device)
            return _DeviceBatches(X, Y, bs, self.world_size, self.global_rank, shuffle=self.world_size > 1)
        if self.world_size > 1 and not isinstance(getattr(dl, "sampler", None),
                                                   torch.utils.data.distributed.DistributedSampler):
            from torch.utils.data import DataLoader, DistributedSampler

            s = DistributedSampler(ds, shuffle=True)
            return DataLoader(ds, batch_size=bs, sampler=s, num_workers=getattr(dl, "num_workers", 0),
                              pin_memory=self.device.type == "cuda")
        return dl

    # ------------------------------------------------------------------ fit
    def fit(self, model, train_dataloaders=None, train_dataloader=None, ckpt_path: str | None = None):
        """Train ``model``.  ``ckpt_path`` resumes (PL's ``fit(ckpt_path=...)``): a
        checkpoint file, or ``"last"`` for the newest ``last.ckpt`` / final checkpoint
        under ``{root}/lightning_logs``; weights, optimizer states, ``global_step``,
        epoch and the position inside the epoch are restored, so a restarted job
        (torchrun ``--max_restarts``) continues where the checkpoint was taken."""
        dl = train_dataloaders if train_dataloaders is not None else train_dataloader
        self._setup()
        if self.seed is not None:
            torch.manual_seed(self.seed)
        model.trainer = self
        model.to(self.device)
        opts = model.configure_optimizers()
        if not isinstance(opts, (list, tuple)):
            opts = [opts]
        resume = self._resolve_ckpt(ckpt_path)
        if resume is not None:
            self._restore(model, opts, resume)
        plan = self._fused_plan(model, opts, dl)
        if plan is not None:
            done = self._fit_fused(model, opts, plan)
            if done is not None:
                return done
        # the flat gradient buffer of FlatDDP also serves one process: fused kernels add
        # their parameter gradients into its views in place (no AccumulateGrad adds)
        single_ok = self.device.type == "cuda" and all(
            p.dtype == torch.float32 and p.device == self.device for p in model.parameters() if p.requires_grad)
        ddp = FlatDDP(model) if (self.world_size > 1 or single_ok) else None
        loader = self._loader(dl)
        self._flat_opts = [_flat_optimizer_for(o, ddp) if self.native_optimizers else None for o in opts]
        # every trainable parameter under exactly one flat optimizer (one optimizer, or
        # several toggled per PL 1.5 so a backward touches only the stepping optimizer's
        # gradients): each flat step leaves the whole flat gradient zero
        self._opt_zeroes = False
        if ddp is not None and self._flat_opts and all(f is not None for f in self._flat_opts):
            owned = [id(p) for f in self._flat_opts for p in f.params]
            self._opt_zeroes = len(owned) == len(set(owned)) and set(owned) == {id(p) for p in ddp._params}
        stepper, static = self._batch_stepper(model, ddp, opts)
        if stepper is not None and isinstance(loader, _DeviceBatches):
            loader.use_ring()  # the replayed step reads its batches from the device epoch ring
        logged_by_key: dict = {}
        logger = CSVLogger(self.root, self.global_rank)
        self._log_dir = logger.dir
        copies = self.graph_copies if stepper is not None else 1
        metrics = _MetricRing(self, logger, defer=copies)
        pbar = None
        if self.enable_progress_bar and self.global_rank == 0:
            try:
                from tqdm import tqdm

                pbar = tqdm(total=self.max_steps if self.max_steps > 0 else None, desc="Epoch 0",
                            initial=self.global_step)
            except ImportError:  # pragma: no cover
                pbar = None
        model.on_train_start()
        t0 = time.perf_counter()
        # steady-state clock: from the end of batch _STEADY_AFTER on (warm-up batches,
        # graph capture and first kernel loads excluded); synchronised at both ends
        # (the warm-up runs and every graph copy's capture come first)
        self.steady_time, self.steady_steps, steady_t0 = None, 0, None
        steady_from = self.global_step + max(_STEADY_AFTER, copies + 6)
        done = 0 <= self.max_steps <= self.global_step or \
            (self.max_epochs is not None and self.current_epoch >= self.max_epochs)
        try:
            while not done:
                if isinstance(loader, _DeviceBatches):
                    loader.skip = self._skip_batches
                if hasattr(loader, "set_epoch"):
                    loader.set_epoch(self.current_epoch)
                elif hasattr(getattr(loader, "sampler", None), "set_epoch"):
                    loader.sampler.set_epoch(self.current_epoch)
                for batch_idx, batch in enumerate(loader):
                    if batch_idx < self._skip_batches:  # resumed mid-epoch: these already ran
                        continue
                    dev = batch if isinstance(batch, _DevBatch) else None
                    if dev is not None and stepper is None:
                        batch = dev.materialize()
                    elif dev is None:
                        batch = [b.to(self.device, non_blocking=True) for b in batch]
                    if self._refresh_flat_opts() and stepper is not None:
                        stepper.reset()  # the captured optimizer launches hold the old hyperparameters
                    if stepper is not None and (dev is not None or self._static_ok(static, batch)):
                        if dev is not None:  # gather inside the replayed step
                            key = ("idx", dev.sel.shape[0])
                            if key not in static:
                                static[key] = _StaticBatch(dev.materialize(),
                                                           None if dev.ring is not None else dev.sel.clone(), dev)
                            if static[key].idx is not None:  # no ring: the batch's indices in
                                static[key].idx.copy_(dev.sel)
                        else:
                            key = tuple(tuple(b.shape) for b in batch)
                            if key not in static:
                                static[key] = _StaticBatch([b.clone() for b in batch])
                            for dst, src in zip(static[key].tensors, batch):
                                dst.copy_(src)
                        self._cur_batch_idx = batch_idx  # read by the body only while capturing
                        # several graph copies per batch shape, replayed in turn: a copy's
                        # logged outputs stay valid until its next replay (_MetricRing.release)
                        gkey = (key, self.global_step % copies)
                        replay = stepper.is_captured(gkey)
                        if replay:
                            metrics.release(gkey)
                        stepper.run(gkey, warm_key=key)
                        # logged tensors of a replay are that copy's graph outputs (refreshed in place)
                        if replay:
                            model._logged.update(logged_by_key[gkey])
                        else:
                            logged_by_key[gkey] = dict(model._logged)
                        owner = gkey
                    else:
                        self._optimizer_steps(model, ddp, opts, batch, batch_idx)
                        owner = None
                    self.global_step += 1  # PL 1.5: once per batch, whatever the optimizer count
                    if self.global_step == steady_from:
                        if self.device.type == "cuda":
                            torch.cuda.synchronize(self.device)
                        steady_t0 = time.perf_counter()
                    self._batch_in_epoch = batch_idx + 1
                    if self.global_step % self.log_every_n_steps == 0:
                        metrics.push(self.global_step, model._logged, owner)
                    if pbar is not None:
                        pbar.update(1)
                    if self.every_n_train_steps and self.global_step % self.every_n_train_steps == 0:
                        metrics.flush()
                        self._save(model, opts, "last.ckpt")
                    if 0 <= self.max_steps <= self.global_step:
                        done = True
                        break
                else:
                    self.current_epoch += 1
                    self._batch_in_epoch = 0
                self._skip_batches = 0
                if self.max_epochs is not None and self.current_epoch >= self.max_epochs:
                    done = True
            metrics.flush()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.fit_time = time.perf_counter() - t0
            if steady_t0 is not None and self.global_step > steady_from:
                self.steady_time = time.perf_counter() - steady_t0
                self.steady_steps = self.global_step - steady_from
            if stepper is not None:
                self.graph_replays = stepper.replays
        finally:
            # the user's torch optimizers hold the trained state again -- before any
            # user hook runs, and also when training raised
            self._export_flat_opts()
            if pbar is not None:
                pbar.close()
        model.on_train_end()
        if self.enable_checkpointing:
            final = f"epoch={max(self.current_epoch - 1, 0) if self._batch_in_epoch == 0 else self.current_epoch}" \
                    f"-step={self.global_step}.ckpt"
            self._save(model, opts, final)
        logger.close()
        return self

    # ------------------------------------------------------------------ fused engine
    def _fused_plan(self, model, opts, dl):
        """The fused train-step engine (engine/fused_trainer.py) runs the fit when the
        LightningModule declares what its ``training_step`` computes --
        ``fused_spec() -> {"models": [m_0, ...], "loss": "mse", "metrics": [name_0, ...]}``:
        optimizer i trains ``models[i]`` (a ToyModel) on ``loss(models[i](x), y)`` of the
        same batch -- and the rest matches: a GPU, plain Adam / SGD optimizers with one
        param group over exactly one model's parameters each and equal hyperparameters,
        a dataset with ``device_tensors``, precision 32 or bf16.  Otherwise None (the
        per-batch module path); ``engine="fused"`` turns a mismatch into an error.

        PL-1.5 semantics kept: each optimizer's update uses the gradient of its own
        model's loss (the models are independent, so toggling the other optimizer's
        parameters changes nothing), ``global_step`` counts batches, the
        DistributedSampler order is exact at world > 1.  One difference in the logs:
        every model's loss is its loss BEFORE this batch's update, where Lightning's
        second ``training_step`` call would log the first model's post-update loss."""
        from ..models.toy import ToyModel

        if self.engine == "module":
            return None

        def no(why):
            if self.engine == "fused":
                raise RuntimeError(f"Trainer(engine='fused'): {why}")
            return None

        fs = getattr(model, "fused_spec", None)
        fs = fs() if callable(fs) else None
        if not fs:
            return no("the LightningModule defines no fused_spec()")
        if self.device.type != "cuda":
            return no("the fused engine needs a GPU")
        models, names = list(fs["models"]), list(fs.get("metrics") or [])
        loss = fs.get("loss", "mse")
        if loss not in ("mse", "ce") or len(names) != len(models) or len(opts) != len(models):
            return no("fused_spec must name one metric per model and match one optimizer per model")
        if not all(isinstance(m, ToyModel) for m in models) or any(m.spec != models[0].spec for m in models):
            return no("fused_spec models must be ToyModels of one architecture")
        cfgs = []
        for o, m in zip(opts, models):
            cfg = _optim_config(o)
            ps = list(m.parameters())
            if cfg is None or len(o.param_groups) != 1 or len(o.param_groups[0]["params"]) != len(ps) or \
                    any(a is not b for a, b in zip(o.param_groups[0]["params"], ps)):
                return no("each optimizer must be a plain Adam/SGD over exactly its model's parameters")
            cfgs.append(cfg)
        if any(c != cfgs[0] for c in cfgs):
            return no("the optimizers' hyperparameters differ")
        ds = getattr(dl, "dataset", None)
        if not hasattr(ds, "device_tensors"):
            return no("the dataset has no device_tensors()")
        prec = "fp32" if self.autocast_dtype is None else "bf16"
        return {"models": models, "names": names, "loss": loss, "optim": cfgs[0], "dataset": ds,
                "batch": int(getattr(dl, "batch_size", None) or 1), "precision": prec, "spec": models[0].spec}

    def _fit_fused(self, model, opts, plan):
        from ..engine.fused_trainer import EngineConfig, FusedTrainer

        models, names = plan["models"], plan["names"]
        X, Y = plan["dataset"].device_tensors(self.device)
        distributed = self.world_size > 1  # PL injects DistributedSampler(shuffle=True) under DDP
        geom = SamplerGeometry(n=X.shape[0], world=self.world_size, rank=self.global_rank, batch=plan["batch"],
                               shuffle=distributed, distributed=distributed, seed=0)
        ecfg = EngineConfig(loss=plan["loss"], precision=plan["precision"])
        tr = FusedTrainer(plan["spec"], len(models), X, Y, geom, plan["optim"], ecfg,
                          init_params=[m.flat_params.detach() for m in models])
        self._skip_batches = 0  # the engine positions its sampler from the step count
        # DDP construction semantics: the engine broadcast rank 0's weights; the modules
        # take them too, so the check below runs training_step on the weights the engine
        # trains (ranks that built their models from different seeds agree from here on)
        for i, m in enumerate(models):
            m.load_flat_(tr.model_params(i))
        why = None
        if self.global_step:  # resumed: the torch optimizers' state continues in the engine
            why = self._import_fused_state(tr, models, opts, self.global_step)
        # fused_spec() is a declaration: check it against training_step on the first batch
        # before the engine trains anything (every rank agrees on the outcome)
        if why is None:
            why = self._verify_fused_spec(model, opts, plan, tr, X, Y)
        if self.world_size > 1:  # every rank takes the same decision
            flag = torch.tensor([0.0 if why is None else 1.0])
            comm_util.all_reduce_(flag)
            if why is None and flag.item() > 0:
                why = "the fused engine was refused on another rank"
        if why is not None:
            tr.close()
            if self.engine == "fused":
                raise RuntimeError(f"Trainer(engine='fused'): {why}")
            if self.global_rank == 0:
                rank_print(0, f"Trainer: not using the fused engine ({why}); per-batch module path")
            self.fused_refused = why
            return None
        self.engine_used = "fused"
        spe = geom.steps_per_epoch
        # the same stopping rule as the module loop: whichever of max_steps / max_epochs
        # comes first (max_epochs defaults to 1000 when max_steps is unset, __init__)
        limits = [self.max_steps] if self.max_steps >= 0 else []
        if self.max_epochs is not None:
            limits.append(self.max_epochs * spe)
        total = min(limits)
        logger = CSVLogger(self.root, self.global_rank)
        self._log_dir = logger.dir
        model.on_train_start()
        if self.global_rank == 0:
            rank_print(0, f"Trainer: fused train-step engine ({tr.comm} comm, {plan['precision']})")
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        last = None
        # steady-state clock: the first launch runs _STEADY_AFTER steps (engine set-up and
        # first kernel loads), the clock runs from its end (synchronised by its loss readback)
        steady_t0, steady_from = None, None
        # launch k+1 is queued before launch k's loss rows are waited for and written
        # (losses_async: a pinned copy + event behind launch k), so the CSV writing
        # overlaps the next launch instead of idling the GPU
        pending = None

        def drain(p):
            nonlocal last
            s0_, s1_, handle = p
            rows = handle.wait_tensor()
            every = self.log_every_n_steps
            first = -(s0_ + 1) % every  # index of the first logged step of the launch
            logger.log_block(s0_ + first + 1, every, names, rows, first)
            last = rows[-1].tolist()

        try:
            while self.global_step < total:
                n = min(tr.cfg.steps_per_launch if steady_t0 is not None else _STEADY_AFTER, total - self.global_step)
                if self.every_n_train_steps:
                    n = min(n, self.every_n_train_steps - self.global_step % self.every_n_train_steps)
                s0 = self.global_step
                tr.train(n)
                self.global_step += n
                handle = tr.losses_async(s0, self.global_step)
                if pending is not None:
                    drain(pending)
                pending = (s0, self.global_step, handle)
                if steady_t0 is None:
                    drain(pending)
                    pending = None
                    steady_t0, steady_from = time.perf_counter(), self.global_step
                # PL's bookkeeping: the batch that reaches max_steps ends the fit inside its
                # epoch (epoch e, batch_in_epoch = its index + 1), it does not open the next
                e, b = divmod(self.global_step - 1, spe)
                self.current_epoch, self._batch_in_epoch = e, b + 1
                if self.every_n_train_steps and self.global_step % self.every_n_train_steps == 0:
                    if pending is not None:
                        drain(pending)
                        pending = None
                    self._export_fused_state(tr, models, opts)
                    self._save(model, opts, "last.ckpt")
            if pending is not None:
                drain(pending)
                pending = None
            torch.cuda.synchronize(self.device)
            t1 = time.perf_counter()
            self.fit_time = t1 - t0
            self.steady_time, self.steady_steps = None, 0
            if steady_t0 is not None and self.global_step > steady_from:
                self.steady_time, self.steady_steps = t1 - steady_t0, self.global_step - steady_from
            if last is not None:
                self.callback_metrics = {**dict(zip(names, last)), "train_loss": sum(last)}
        finally:
            self._export_fused_state(tr, models, opts)
            tr.close()
        model.on_train_end()
        if self.enable_checkpointing:
            final = f"epoch={max(self.current_epoch - 1, 0) if self._batch_in_epoch == 0 else self.current_epoch}" \
                    f"-step={self.global_step}.ckpt"
            self._save(model, opts, final)
        logger.close()
        return self

    def _verify_fused_spec(self, model, opts, plan, tr, X, Y) -> str | None:
        """Run ``training_step`` once on the batch the engine trains first (module path,
        autograd, no optimizer step) and compare every model's logged loss and parameter
        gradient with the engine's gradient-only launch of the same step (MODE_GRAD:
        local means, nothing updated).  Returns None when they agree (rtol 1e-4, atol
        1e-5: fp32 under different summation orders), else the reason (the caller makes
        every rank take the same decision)."""
        models, names = plan["models"], plan["names"]
        why = None
        try:
            idx = torch.as_tensor(tr.step_indices(self.global_step), dtype=torch.long, device=X.device)
            batch = [X[idx], Y[idx]]
            eng_g, eng_l = tr.local_gradients()
            saved = [p.requires_grad for p in model.parameters()]
            try:
                for oi, m in enumerate(models):
                    if len(opts) > 1:
                        model.toggle_optimizer(opts[oi], oi, opts)
                    with self._autocast():
                        out = model.training_step(batch, 0, oi) if len(opts) > 1 else model.training_step(batch, 0)
                    loss = out["loss"] if isinstance(out, dict) else out
                    ps = list(m.parameters())
                    gs = torch.autograd.grad(loss, ps, allow_unused=True)
                    g = torch.cat([(torch.zeros_like(p) if q is None else q).reshape(-1) for p, q in zip(ps, gs)])
                    logged = model._logged.get(names[oi])
                    if len(opts) > 1:
                        model.untoggle_optimizer(oi)
                    if logged is None:
                        why = f"training_step does not log {names[oi]!r}"
                        break
                    lv = float(torch.as_tensor(logged).detach().float().reshape(-1)[0])
                    tol = 1e-2 if plan["precision"] == "bf16" else 1e-4
                    if not math.isclose(lv, float(eng_l[oi]), rel_tol=tol, abs_tol=1e-5):
                        why = f"{names[oi]} of training_step is {lv:.6g}, the declared step gives {float(eng_l[oi]):.6g}"
                        break
                    if not torch.allclose(g.float(), eng_g[oi], rtol=tol, atol=1e-5 if tol < 1e-3 else 1e-3):
                        err = (g.float() - eng_g[oi]).abs().max().item()
                        why = f"model {oi}'s gradient from training_step differs from fused_spec's (max err {err:.3g})"
                        break
            finally:
                for p, r in zip(model.parameters(), saved):
                    p.requires_grad_(r)
                model._logged.clear()
        except Exception as e:  # noqa: BLE001 - any failure of the check refuses the engine
            why = f"fused_spec check failed: {e}"
        return why

    @staticmethod
    def _import_fused_state(tr, models, opts, global_step: int) -> str | None:
        """A resumed fit: the torch optimizers' restored moments (Adam exp_avg /
        exp_avg_sq, SGD momentum_buffer) and step count continue in the fused engine
        (the parameters came in through init_params); ``global_step`` batches ran.
        Returns None, or why the engine cannot continue this state (the caller refuses
        the engine: the module path under engine='auto', an error under 'fused')."""
        for i, (m, o) in enumerate(zip(models, opts)):
            st = [o.state.get(p, {}) for p in m.parameters()]
            keys = ("exp_avg", "exp_avg_sq") if isinstance(o, torch.optim.Adam) else ("momentum_buffer",)
            for key, dst in zip(keys, (tr.m[i], tr.v[i])):
                if all(s.get(key) is not None for s in st):
                    dst.copy_(torch.cat([s[key].reshape(-1).to(dst) for s in st]))
            steps = [s["step"] for s in st if "step" in s]
            step = int(float(steps[0])) if steps else global_step
            # the persistent engine positions its sampler AND its Adam bias corrections from
            # one step number (host_t0 = tr.t): a restored optimizer that stepped a different
            # number of times than the batches that ran cannot continue bit-exactly there
            if step != global_step:
                return (f"resumed optimizer {i} has step {step} but global_step is {global_step}: the fused "
                        "engine needs one optimizer step per batch")
            tr.step_ctr[i] = step
        tr.t = global_step
        return None

    @staticmethod
    def _export_fused_state(tr, models, opts) -> None:
        """Weights back into the modules and the optimizer state into torch format, so
        checkpoints, hooks and a later module-path fit see the trained state."""
        tr.synchronize()
        for i, (m, o) in enumerate(zip(models, opts)):
            m.load_flat_(tr.model_params(i))
            step = float(tr.step_ctr[i].item())
            off = 0
            for p in m.parameters():
                n = p.numel()
                if isinstance(o, torch.optim.Adam):
                    o.state[p] = {"step": torch.tensor(step), "exp_avg": tr.m[i, off:off + n].view_as(p).clone(),
                                  "exp_avg_sq": tr.v[i, off:off + n].view_as(p).clone()}
                elif o.param_groups[0].get("momentum", 0.0):
                    o.state[p] = {"momentum_buffer": tr.m[i, off:off + n].view_as(p).clone()}
                off += n

    # ------------------------------------------------------------------ checkpoints
    def _ckpt_dir(self) -> Path | None:
        if self._log_dir is None:
            return None
        d = self._log_dir / "checkpoints"
        d.mkdir(exist_ok=True)
        return d

    def _save(self, model, opts, name: str) -> None:
        """Rank-0 atomic save (tmp + rename) of weights, optimizer states and the loop
        position; every rank then waits for it (a barrier), so no rank can run ahead
        into a collective while rank 0 is still writing."""
        self._export_flat_opts()  # torch-format optimizer state of the flat-kernel optimizers
        d = self._ckpt_dir() if self.global_rank == 0 else None
        if d is not None:
            path = d / name
            tmp = path.with_suffix(".tmp")
            torch.save({"state_dict": {k: v.detach().cpu() for k, v in model.state_dict().items()},
                        "global_step": self.global_step, "epoch": self.current_epoch,
                        "batch_in_epoch": self._batch_in_epoch,
                        "optimizer_states": [_cpu_state(o.state_dict()) for o in opts]}, tmp)
            os.replace(tmp, path)
            self.checkpoint_path = str(path)
        if dist.is_initialized():
            comm_util.barrier()

    def _resolve_ckpt(self, ckpt_path):
        if ckpt_path is None:
            return None
        if ckpt_path != "last":
            return Path(ckpt_path)
        base = Path(self.root) / "lightning_logs"
        cands = sorted(base.glob("version_*/checkpoints/*.ckpt"), key=lambda p: p.stat().st_mtime)
        return cands[-1] if cands else None

    def _restore(self, model, opts, path: Path) -> None:
        ck = torch.load(path, map_location="cpu", weights_only=True)
        model.load_state_dict(ck["state_dict"])
        for o, st in zip(opts, ck["optimizer_states"]):
            o.load_state_dict(st)
        self.global_step = int(ck["global_step"])
        self.current_epoch = int(ck["epoch"])
        self._skip_batches = self._batch_in_epoch = int(ck.get("batch_in_epoch", 0))
        self.resumed_from = str(path)
        if self.global_rank == 0:
            rank_print(0, f"resumed from {path} at global_step {self.global_step}")

    def _refresh_flat_opts(self) -> bool:
        """Re-read every flat-kernel optimizer's param group (hooks may change lr, ...).
        True if a hyperparameter changed; an optimizer that left the flat kernel's
        domain hands its state back to torch and runs torch's own step from now on."""
        changed = False
        for i, fo in enumerate(self._flat_opts):
            if fo is None:
                continue
            r = fo.refresh()
            if r is None:
                fo.export_state()
                self._flat_opts[i] = None
                self._opt_zeroes = False  # torch's step leaves its gradient: zero_grad fills again
                changed = True
            else:
                changed |= r
        return changed

    def _export_flat_opts(self) -> None:
        for fo in self._flat_opts:
            if fo is not None:
                fo.export_state()

    def _optimizer_steps(self, model, ddp, opts, batch, batch_idx):
        """One batch: for each optimizer (PL 1.5): toggle, zero_grad, training_step,
        backward, step, untoggle."""
        for oi, opt in enumerate(opts):
            if len(opts) > 1:
                model.toggle_optimizer(opt, oi, opts)
            if ddp is not None:
                ddp.zero_grad()
            else:
                opt.zero_grad(set_to_none=False)
            with self._autocast():
                out = model.training_step(batch, batch_idx, oi) if len(opts) > 1 else \
                    model.training_step(batch, batch_idx)
            loss = out["loss"] if isinstance(out, dict) else out
            flat = self._flat_opts[oi] if oi < len(self._flat_opts) else None
            # one rank (nothing reads the gradient between the backward and the step): the
            # backward's last stage kernel and the flat optimizer step as ONE launch
            fuse = flat is not None and self._fuse_backward_opt and (ddp is None or ddp.world == 1)
            with (ParamBackwardFusion() if fuse else contextlib.nullcontext()) as fus:
                # the seed from a cached tensor of ones (autograd's own would be a fill launch per step)
                loss.backward(self._backward_seed(loss))
                if flat is not None:
                    # the flat kernel zeroes the gradient it consumed: the next zero_grad is free
                    if flat.step(zero_grad=self._opt_zeroes, fused=fus.take() if fus is not None else None) \
                            and ddp is not None:
                        ddp.mark_grad_clean()
                else:
                    opt.step()
            if len(opts) > 1:
                model.untoggle_optimizer(oi)
            model._logged[f"train_loss_opt{oi}"] = loss.detach()

    def _backward_seed(self, loss: torch.Tensor):
        """d loss / d loss for a scalar loss, cached per (dtype, device); None otherwise."""
        if loss.numel() != 1 or not loss.is_cuda:
            return None
        key = (loss.dtype, loss.device, tuple(loss.shape))
        seeds = self.__dict__.setdefault("_seeds", {})
        t = seeds.get(key)
        if t is None:
            t = seeds[key] = torch.ones_like(loss)
        return t

    def _autocast(self):
        """precision='bf16': torch.autocast around the forward (PL's bf16 plugin); the
        weight-cast cache stays off so a captured hipGraph re-reads the live weights."""
        if self.autocast_dtype is None:
            return contextlib.nullcontext()
        return torch.autocast(self.device.type, dtype=self.autocast_dtype, cache_enabled=False)

    @staticmethod
    def _static_ok(static, batch) -> bool:
        return all(isinstance(b, torch.Tensor) and b.is_cuda for b in batch)

    def _batch_stepper(self, model, ddp, opts):
        """A CapturedStep replaying one batch's optimizer steps as a hipGraph, when the
        run allows it: a GPU, buckets that can be captured (one rank, the in-kernel xGMI
        all-reduce, or RCCL: ``FlatDDP.graph_safe``), and optimizers that can keep
        their step counts on the device (torch's ``capturable`` param-group flag).

        What a replay repeats is what the capture recorded: device work on the static
        batch buffers.  Host-side decisions inside ``training_step`` (e.g. on
        ``batch_idx`` or a Python counter) are frozen at capture time, and a step that
        syncs with the host cannot be captured (that batch shape then runs eagerly);
        ``Trainer(use_graphs=False)`` runs every batch eagerly."""
        if not (self.use_graphs and self.device.type == "cuda"):
            return None, None
        if ddp is not None and not ddp.graph_safe():
            return None, None
        for opt in opts:
            if not all("capturable" in g for g in opt.param_groups) and not isinstance(opt, torch.optim.SGD):
                return None, None
        for opt in opts:
            for g in opt.param_groups:
                if "capturable" in g:
                    g["capturable"] = True
        from ..engine.graph_step import CapturedStep

        static: dict = {}

        def body(gkey):
            sb = static[gkey[0]]  # (batch shape, graph copy)
            if sb.src is not None:  # device batch: the gather is part of the replayed step
                sb.src.gather_into(sb.idx, sb.tensors)
            self._optimizer_steps(model, ddp, opts, sb.tensors, self._cur_batch_idx)

        def abort():
            if getattr(model, "_toggled", None):
                model.untoggle_optimizer(-1)
            if ddp is not None:
                ddp.reset_hooks()
                ddp._grad_clean = False  # the abandoned capture's gradient zeroing never ran

        stepper = CapturedStep(body, self.device, on_abort=abort)
        self._stepper = stepper
        return stepper, static

    def teardown(self):
        if dist.is_initialized():
            comm_util.barrier()
            dist.destroy_process_group()


class _StaticBatch:
    """The batch buffers a captured step reads (and, for device batches, the index
    buffer it gathers them with)."""

    __slots__ = ("tensors", "idx", "src")

    def __init__(self, tensors, idx=None, src=None):
        self.tensors, self.idx, self.src = tensors, idx, src


def _cpu_state(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: _cpu_state(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_cpu_state(v) for v in x)
    return x


_GROUP_KEYS = ("lr", "betas", "eps", "weight_decay", "momentum", "dampening", "nesterov", "amsgrad", "maximize",
               "differentiable", "decoupled_weight_decay")


def _group_key(opt):
    g = opt.param_groups[0]
    return (type(opt), len(opt.param_groups)) + tuple(g.get(k) for k in _GROUP_KEYS)


def _optim_config(opt):
    """OptimConfig of a plain Adam/SGD's single param group, or None if the flat kernel
    cannot run it (several groups, tensor lr, amsgrad, nesterov, ...)."""
    from ..ops.optim import OptimConfig

    if len(opt.param_groups) != 1:
        return None
    g = opt.param_groups[0]
    lr = g.get("lr")
    if isinstance(lr, torch.Tensor) or g.get("maximize") or g.get("differentiable"):
        return None
    if type(opt) is torch.optim.Adam:
        if g.get("amsgrad") or g.get("decoupled_weight_decay"):
            return None
        return OptimConfig("adam", float(lr), tuple(float(b) for b in g["betas"]), float(g["eps"]),
                           float(g["weight_decay"]))
    if type(opt) is torch.optim.SGD:
        if g.get("nesterov") or g.get("dampening", 0):
            return None
        return OptimConfig("sgd", float(lr), weight_decay=float(g["weight_decay"]), momentum=float(g["momentum"]))
    return None


class _FlatTorchOptimizer:
    """A user's plain ``torch.optim.Adam`` / ``SGD`` run as ONE flat-optimizer kernel
    (``csrc/optim.hip``, the element-for-element mirror of torch's math) over the span
    of the flat parameter buffer its single param group covers, instead of torch's
    ~5 multi-tensor launches plus per-parameter step bookkeeping.  The moments live
    in flat buffers (imported from ``opt.state`` when the optimizer was restored from
    a checkpoint); ``export_state`` writes them back into ``opt.state`` in torch's own
    format (checkpoints, continued use of the optimizer).  ``refresh`` re-reads the
    param group, so hyperparameter edits between steps (manual LR decay) apply."""

    def __init__(self, opt, params, flat_p, flat_g, cfg):
        from ..ops.optim import FlatOptimizer

        self.opt = opt
        self.params = params
        self.cfg = cfg
        self.flat = FlatOptimizer(flat_p, flat_g, cfg)
        self._key = _group_key(opt)
        self._import_state()

    def _import_state(self):
        st0 = [self.opt.state.get(p) for p in self.params]
        if not any(st0):
            return
        steps = {int(float(st["step"])) if st and "step" in st else 0 for st in st0}
        o = 0
        m, v = self.flat.m.view(-1), self.flat.v.view(-1)
        with torch.no_grad():
            for p, st in zip(self.params, st0):
                n = p.numel()
                if st:
                    if self.cfg.name == "adam":
                        m[o:o + n].copy_(st["exp_avg"].reshape(-1))
                        v[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                    elif st.get("momentum_buffer") is not None:
                        m[o:o + n].copy_(st["momentum_buffer"].reshape(-1))
                o += n
        # SGD keeps no step count in torch: a restored momentum buffer means "not the first step"
        step = max(steps) if self.cfg.name == "adam" else (1 if any(st0) else 0)
        self.flat.step_ctr.fill_(step)
        self.opt.state.clear()  # the flat buffers are the live state until export_state

    def refresh(self):
        """True if the param group's hyperparameters changed (now applied), False if
        not, None if the optimizer no longer fits the flat kernel.  Called every batch:
        an unchanged param group is recognised from a tuple of its entries."""
        key = _group_key(self.opt)
        if key == self._key:
            return False
        self._key = key
        cfg = _optim_config(self.opt)
        if cfg is None or cfg.name != self.cfg.name:
            return None
        if cfg == self.cfg:
            return False
        self.cfg = self.flat.cfg = cfg
        return True

    def step(self, zero_grad: bool = False, fused=None) -> bool:
        return self.flat.step(zero_grad=zero_grad, fused=fused)

    def export_state(self):
        step = int(self.flat.step_ctr[0].item())
        if step == 0:
            return
        group = self.opt.param_groups[0]
        o = 0
        m, v = self.flat.m.view(-1), self.flat.v.view(-1)
        for p in self.params:
            n = p.numel()
            st = self.opt.state[p]
            if self.cfg.name == "adam":
                cap = bool(group.get("capturable", False))
                st["step"] = torch.tensor(float(step), dtype=torch.float32, device=p.device if cap else "cpu")
                st["exp_avg"] = m[o:o + n].view_as(p).clone()
                st["exp_avg_sq"] = v[o:o + n].view_as(p).clone()
            elif self.cfg.momentum:
                st["momentum_buffer"] = m[o:o + n].view_as(p).clone()
            o += n


def _flat_optimizer_for(opt, ddp):
    """_FlatTorchOptimizer for ``opt`` if it is a plain Adam/SGD whose one param group
    is a contiguous span of the flat buffers on a GPU, else None (torch's step runs)."""
    from ..ops.mlp import _flat_view_of

    if ddp is None or not ddp.flat_params.is_cuda:
        return None
    cfg = _optim_config(opt)
    if cfg is None:
        return None
    params = list(opt.param_groups[0]["params"])
    if not params or any(p.dtype != torch.float32 or p.grad is None for p in params):
        return None
    flat_p = _flat_view_of([p.data for p in params])
    flat_g = _flat_view_of([p.grad for p in params])
    if flat_p is None or flat_g is None:
        return None
    return _FlatTorchOptimizer(opt, params, flat_p, flat_g, cfg)
