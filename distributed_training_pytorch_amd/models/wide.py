"""WideMLP: the ToyModel architecture (Linear + LeakyReLU stack, ``toy_model_and_data.py:8-25``)
at widths where the matmuls are real GEMMs -- every Linear runs through ``ops.gemm``:
the LDS-tiled MFMA GEMMs of ``csrc/gemm.hip`` / ``csrc/gemm_ph8.hip`` (bias +
activation fused into the epilogue, activation gradient fused into the input-gradient
GEMM); fp32 or bf16 compute.

Same ``layers.{2i}.{weight,bias}`` state-dict layout as ``ToyModel``; parameters
are views into one flat fp32 buffer, so ``FlatDDP`` all-reduces them as one
bucket list and checkpoints interchange with plain ``nn.Sequential`` MLPs.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.gemm import mlp


class WideMLP(nn.Module):
    def __init__(self, widths=(2, 1024, 1024, 1024, 1024, 1), slope: float = 0.01,
                 compute_dtype: torch.dtype = torch.float32):
        super().__init__()
        if len(widths) < 2:
            raise ValueError("WideMLP needs at least an input and an output width")
        self.widths = tuple(int(w) for w in widths)
        self.slope = slope
        self.compute_dtype = compute_dtype
        mods: list[nn.Module] = []
        for i in range(len(widths) - 1):
            mods.append(nn.Linear(widths[i], widths[i + 1]))
            if i < len(widths) - 2:
                mods.append(nn.LeakyReLU(slope))
        self.layers = nn.Sequential(*mods)
        self._flatten()

    def _flatten(self):
        ps = list(self.layers.parameters())
        flat = torch.empty(sum(p.numel() for p in ps), dtype=ps[0].dtype, device=ps[0].device)
        o = 0
        for p in ps:
            n = p.numel()
            flat[o:o + n].copy_(p.data.reshape(-1))
            p.data = flat[o:o + n].view_as(p)
            o += n
        self._flat = flat

    @property
    def flat_params(self) -> torch.Tensor:
        return self._flat

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn, recurse)
        self._flatten()
        return out

    def linears(self) -> list[nn.Linear]:
        return [m for m in self.layers if isinstance(m, nn.Linear)]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        lin = self.linears()
        return mlp(x, [m.weight for m in lin], [m.bias for m in lin], self.slope, self.compute_dtype)

    def reference_forward(self, x: torch.Tensor) -> torch.Tensor:
        """Plain PyTorch forward of the same module tree (tests / stock baseline)."""
        return self.layers(x)
