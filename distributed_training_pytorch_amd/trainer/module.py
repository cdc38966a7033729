"""LightningModule-style base class (the subset demo_pytorch_lightning.py uses).

Reference: ``LitToyModel(pl.LightningModule)`` with ``forward``,
``training_step(batch, batch_idx, optimizer_idx)`` and ``configure_optimizers``
returning two Adams (``demo_pytorch_lightning.py:16-40``), PyTorch-Lightning 1.5.10
semantics.  pytorch_lightning is not installed on the MI355X image, so the
Trainer in ``trainer.py`` drives this class directly.
"""
from __future__ import annotations

import torch
import torch.nn as nn


class LightningModule(nn.Module):
    def __init__(self):
        super().__init__()
        self.trainer = None
        self._logged: dict[str, float] = {}

    # ---- user hooks -----------------------------------------------------------
    def training_step(self, batch, batch_idx, optimizer_idx=0):  # pragma: no cover - abstract
        raise NotImplementedError

    def configure_optimizers(self):  # pragma: no cover - abstract
        raise NotImplementedError

    def on_train_start(self):
        pass

    def on_train_end(self):
        pass

    # ---- services ---------------------------------------------------------------
    def log(self, name: str, value, prog_bar: bool = False, sync_dist: bool = False, **_):
        v = value.detach() if isinstance(value, torch.Tensor) else torch.tensor(float(value))
        self._logged[name] = v

    @property
    def global_step(self) -> int:
        return self.trainer.global_step if self.trainer else 0

    @property
    def current_epoch(self) -> int:
        return self.trainer.current_epoch if self.trainer else 0

    @property
    def device(self) -> torch.device:
        for p in self.parameters():
            return p.device
        return torch.device("cpu")

    def toggle_optimizer(self, optimizer, optimizer_idx: int, optimizers) -> None:
        """PL 1.5: only the current optimizer's params require grad during its step."""
        own = {id(p) for g in optimizer.param_groups for p in g["params"]}
        self._toggled = {}
        for opt in optimizers:
            for g in opt.param_groups:
                for p in g["params"]:
                    self._toggled[p] = p.requires_grad
                    p.requires_grad_(id(p) in own)

    def untoggle_optimizer(self, optimizer_idx: int) -> None:
        for p, rg in getattr(self, "_toggled", {}).items():
            p.requires_grad_(rg)
        self._toggled = {}
