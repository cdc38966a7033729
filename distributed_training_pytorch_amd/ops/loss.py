"""Fused MSE loss for the module (autograd) path.

``nn.MSELoss()`` in the reference's training step (``/root/reference/demo.py:103-104``,
``/root/reference/demo_pytorch_lightning.py:27-33``) is, on torch, an elementwise square
plus a mean reduction forward (two launches) and its own backward launch.  Inside the
Trainer's replayed hipGraph every launch costs ~4 us whatever it does
(``docs/perf_notes.md``, "the Trainer's generic (module) path"), so the loss is ONE
launch forward (``csrc/loss.hip``: sum of squares in one workgroup, divided by n) and one
backward (``ga = g * 2 (a - b) / n``, the incoming gradient read on the device).

``MSELoss`` / ``mse_loss`` are drop-ins for reduction="mean" on fp32 CUDA tensors of the
same shape; anything else (CPU, other dtypes or reductions, broadcasting, more than 2^20
elements) runs ``torch.nn.functional.mse_loss``.
"""
from __future__ import annotations

import torch
from torch import nn

from .. import _native as nat


def _fused_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    return (a.is_cuda and b.is_cuda and a.dtype == torch.float32 and b.dtype == torch.float32
            and a.shape == b.shape and a.device == b.device and 0 < a.numel() <= (1 << 16)
            and nat.native_enabled())


class _FusedMSE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a_ = a.contiguous()
        b_ = b.contiguous()
        out = torch.empty((), dtype=torch.float32, device=a.device)
        lib = nat.load()
        nat.check(lib.dtp_mse_fwd(nat.ptr(a_), nat.ptr(b_), a_.numel(), nat.ptr(out), nat.stream_ptr()), "dtp_mse_fwd")
        ctx.save_for_backward(a_, b_)
        ctx.shape = a.shape
        return out

    @staticmethod
    def backward(ctx, g):
        a_, b_ = ctx.saved_tensors
        need_a, need_b = ctx.needs_input_grad
        ga = torch.empty_like(a_) if need_a else None
        gb = torch.empty_like(b_) if need_b else None
        if ga is None and gb is None:
            return None, None
        g_ = g.reshape(1).contiguous().float()
        lib = nat.load()
        nat.check(lib.dtp_mse_bwd(nat.ptr(a_), nat.ptr(b_), nat.ptr(g_), a_.numel(), nat.ptr(ga), nat.ptr(gb),
                                  nat.stream_ptr()), "dtp_mse_bwd")
        return (ga.view(ctx.shape) if ga is not None else None,
                gb.view(ctx.shape) if gb is not None else None)


def mse_loss(input: torch.Tensor, target: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    """``torch.nn.functional.mse_loss`` with the fused one-launch path for the common case."""
    if reduction == "mean" and _fused_ok(input, target):
        return _FusedMSE.apply(input, target)
    return nn.functional.mse_loss(input, target, reduction=reduction)


class MSELoss(nn.Module):
    """Drop-in ``nn.MSELoss`` (reduction="mean" fused on the GPU, see module docstring)."""

    def __init__(self, reduction: str = "mean"):
        super().__init__()
        self.reduction = reduction

    def forward(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        return mse_loss(input, target, self.reduction)
