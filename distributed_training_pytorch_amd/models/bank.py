"""ModelBank: N ToyModels whose parameters (and gradients) are rows of ONE
[N, P] buffer.

The reference trains two independent models per iteration with two DDP
wrappers, two NCCL all-reduces and two Adam optimizers (``demo.py:22-23,69-72,
80-81,110-111``).  Laid out as one bank, both models' gradients leave the GPU in
a single all-reduce and both optimizers are one kernel launch -- fewer, larger
collectives (the MI355X rule), while each ``bank[i]`` is still an ordinary
``nn.Module`` with the reference's state_dict keys.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.gemm import ComputeShadow, mark_fused_grad
from .toy import ToyModel


class ModelBank(nn.Module):
    def __init__(self, n: int = 2, **toy_kwargs):
        super().__init__()
        self.models = nn.ModuleList([ToyModel(**toy_kwargs) for _ in range(n)])
        self.rebind()

    @property
    def spec(self):
        return self.models[0].spec

    def rebind(self) -> None:
        """(Re)pack every model's params into rows of one buffer and grads likewise."""
        P = self.spec.P
        n = len(self.models)
        ref = self.models[0].flat_params
        flat = torch.empty(n, P, dtype=ref.dtype, device=ref.device)
        grad = torch.zeros(n, P, dtype=ref.dtype, device=ref.device)
        for i, m in enumerate(self.models):
            flat[i].copy_(m.flat_params)
            o = 0
            for p in m.layers.parameters():
                k = p.numel()
                p.data = flat[i, o:o + k].view_as(p)
                p.grad = grad[i, o:o + k].view_as(p)
                mark_fused_grad(p)
                o += k
            m._flat = flat[i]
        self.flat = flat
        self.flat_grad = grad
        if getattr(self, "_shadow", None) is not None:  # the old shadow's views point at the old buffer
            self._shadow.detach_()
            self._shadow = None

    def compute_shadow(self):
        """A bf16 ``ComputeShadow`` of the bank's weight matrices (the GEMM path's
        operands), for ``FlatOptimizer(..., shadow=bank.compute_shadow())``.  Rebuilt
        after ``.to()`` / ``rebind()``."""
        if getattr(self, "_shadow", None) is None:
            weights = [p for m in self.models for n, p in m.layers.named_parameters() if n.endswith("weight")]
            self._shadow = ComputeShadow(self.flat, weights)
        return self._shadow

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn, recurse)
        self.rebind()
        return out

    def zero_grad(self, set_to_none: bool = False) -> None:  # grads are views: zero in place
        self.flat_grad.zero_()

    def forward(self, x):
        # the models' forwards in one launch on the GPU (ToyModel.forward_many)
        return list(ToyModel.forward_many(list(self.models), x))

    def __getitem__(self, i) -> ToyModel:
        return self.models[i]
