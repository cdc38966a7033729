#!/usr/bin/env python3
"""Lightning-style demo: two ToyModels, two Adams, DDP strategy.

Reference: demo_pytorch_lightning.py (``pl.Trainer(gpus, num_nodes, max_steps,
precision=32, accelerator='gpu', strategy='ddp')``, backend from
PL_TORCH_DISTRIBUTED_BACKEND, launched one task per GPU by srun).  Uses the in-repo
Trainer (distributed_training_pytorch_amd.trainer), which follows PyTorch-Lightning
1.5.10 semantics; when pytorch_lightning is importable and ``--use_lightning`` is
given, the real Lightning Trainer is used instead.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

from distributed_training_pytorch_amd.ops.loss import MSELoss  # noqa: E402
from distributed_training_pytorch_amd.runtime import bootstrap  # noqa: E402
from distributed_training_pytorch_amd.runtime.errors import record  # noqa: E402
from distributed_training_pytorch_amd.trainer import LightningModule, Trainer  # noqa: E402
from toy_model_and_data import ToyData, ToyModel  # noqa: E402


class LitToyModel(LightningModule):
    def __init__(self, lr: float = 1e-3):
        super().__init__()
        self.model_X = ToyModel()
        self.model_Y = ToyModel()
        self.loss = MSELoss()  # nn.MSELoss drop-in: one fused launch each way (ops/loss.py)
        self.lr = lr

    def forward(self, x):
        # both models on the same batch: one fused forward launch on the GPU (models/toy.py)
        return ToyModel.forward_many([self.model_X, self.model_Y], x)

    def training_step(self, batch, batch_idx, optimizer_idx=0):
        x, y = batch
        out_x, out_y = self(x)
        # loss_x, loss_y and loss_x + loss_y of the reference's step, as ONE fused launch
        # (ops/loss.py:MSELoss.pair; the same values as two MSELoss calls and an add)
        loss_x, loss_y, loss = self.loss.pair(out_x, out_y, y)
        self.log("loss/lossX", loss_x)
        self.log("loss/lossY", loss_y)
        return loss

    def fused_spec(self):
        """What training_step computes, for the in-repo Trainer's fused train-step engine:
        optimizer i trains models[i] on MSE(models[i](x), y) of the same batch (the
        returned loss_X + loss_Y over two independent models), logged as metrics[i]."""
        return {"models": [self.model_X, self.model_Y], "loss": "mse", "metrics": ["loss/lossX", "loss/lossY"]}

    def configure_optimizers(self):
        return [torch.optim.Adam(self.model_X.parameters(), lr=self.lr),
                torch.optim.Adam(self.model_Y.parameters(), lr=self.lr)]


def get_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--nnodes", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--num_workers", type=int, default=0)
    p.add_argument("--batch_size", type=int, default=128)
    p.add_argument("--accelerator", choices=["gpu", "cpu"], default=None)
    p.add_argument("--root_dir", type=str, default=None)
    p.add_argument("--no_progress", action="store_true")
    p.add_argument("--use_lightning", action="store_true", help="use pytorch_lightning if it is installed")
    p.add_argument("--engine", default="auto", choices=["auto", "fused", "module"],
                   help="in-repo Trainer: the fused train-step engine (from LitToyModel.fused_spec) or the "
                        "per-batch nn.Module path (auto: fused when it applies)")
    p.add_argument("--no_graphs", action="store_true",
                   help="in-repo Trainer, module path: run every batch eagerly instead of replaying it as a hipGraph")
    p.add_argument("--torch_optimizers", action="store_true",
                   help="in-repo Trainer: step the torch optimizers themselves, not the flat-optimizer kernel")
    p.add_argument("--precision", default="32", choices=["32", "bf16"],
                   help="32 (the reference's precision=32) or bf16 autocast (fp32 master weights)")
    p.add_argument("--ckpt_path", default=None,
                   help="resume: a checkpoint file, or 'last' for the newest one under <root_dir>/lightning_logs")
    p.add_argument("--every_n_train_steps", type=int, default=0,
                   help="also save lightning_logs/version_N/checkpoints/last.ckpt every N batches")
    return p.parse_args(argv)


@record
def main(argv=None):
    a = get_args(argv)
    # before the first GPU touch (torch.cuda.is_available below): HSA reads the IPC mode once
    bootstrap.configure_collective_env()
    torch.manual_seed(a.seed)
    ds = ToyData(seed=a.seed)
    dl = DataLoader(ds, batch_size=a.batch_size, pin_memory=torch.cuda.is_available(), num_workers=a.num_workers)
    model = LitToyModel()
    accel = a.accelerator or ("gpu" if torch.cuda.is_available() else "cpu")
    TrainerCls = Trainer
    if a.use_lightning:
        try:
            import pytorch_lightning as pl

            TrainerCls = pl.Trainer
        except ImportError:
            print("pytorch_lightning not installed; using the in-repo Trainer", flush=True)
    engine = "module" if (a.no_graphs or a.torch_optimizers) and a.engine == "auto" else a.engine
    extra = {"seed": a.seed, "use_graphs": not a.no_graphs, "native_optimizers": not a.torch_optimizers,
             "every_n_train_steps": a.every_n_train_steps, "engine": engine} if TrainerCls is Trainer else {}
    precision = 32 if a.precision == "32" else "bf16"
    trainer = TrainerCls(gpus=a.gpus, num_nodes=a.nnodes, max_steps=a.steps, precision=precision, accelerator=accel,
                         log_every_n_steps=min(50, len(dl) / a.batch_size), strategy="ddp",
                         default_root_dir=a.root_dir, enable_progress_bar=not a.no_progress, **extra)
    trainer.fit(model, dl, ckpt_path=a.ckpt_path)
    if getattr(trainer, "global_rank", 0) == 0:
        sps = None
        if getattr(trainer, "fit_time", None):
            sps = trainer.global_step * a.batch_size * getattr(trainer, "world_size", 1) / trainer.fit_time
        # steady state: module path after the first 10 batches (eager warm-up, graph capture,
        # first kernel loads); fused engine after its first launch of 10 steps
        steady = None
        if getattr(trainer, "steady_time", None):
            steady = trainer.steady_steps * a.batch_size * getattr(trainer, "world_size", 1) / trainer.steady_time
        print(f"[Process 0] summary: {{'global_step': {trainer.global_step}, 'metrics': {trainer.callback_metrics}, "
              f"'checkpoint': {trainer.checkpoint_path!r}, 'samples_per_s': {sps}, 'steady_samples_per_s': {steady}, "
              f"'graph_replays': {getattr(trainer, 'graph_replays', 0)}, "
              f"'engine': {getattr(trainer, 'engine_used', None)!r}}}", flush=True)
    if hasattr(trainer, "teardown"):
        trainer.teardown()


if __name__ == "__main__":
    main()
