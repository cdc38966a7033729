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


class _FusedMSEPair(torch.autograd.Function):
    """(mse(a1, b), mse(a2, b), their sum) in one launch; backward in one launch."""

    @staticmethod
    def forward(ctx, a1, a2, b, log):
        ctx.set_materialize_grads(False)  # unused outputs' gradients stay None (no zero fills)
        a1_, a2_, b_ = a1.contiguous(), a2.contiguous(), b.contiguous()
        o1, o2, osum = (torch.empty((), dtype=torch.float32, device=a1.device) for _ in range(3))
        ring, slot = log if log is not None else (None, None)
        nat.check(nat.load().dtp_mse_pair_fwd(nat.ptr(a1_), nat.ptr(a2_), nat.ptr(b_), b_.numel(), nat.ptr(o1),
                                              nat.ptr(o2), nat.ptr(osum), nat.ptr(ring), nat.ptr(slot),
                                              0 if ring is None else ring.shape[1], nat.stream_ptr()),
                  "dtp_mse_pair_fwd")
        ctx.save_for_backward(a1_, a2_, b_)
        ctx.shape = b.shape
        return o1, o2, osum

    @staticmethod
    def backward(ctx, g1, g2, gsum):
        a1_, a2_, b_ = ctx.saved_tensors
        n1, n2, nb, _ = ctx.needs_input_grad
        if (g1 is None and g2 is None and gsum is None) or not (n1 or n2 or nb):
            return None, None, None, None
        ga1 = torch.empty_like(a1_) if n1 else None
        ga2 = torch.empty_like(a2_) if n2 else None
        gb = torch.empty_like(b_) if nb else None
        dev = lambda g: None if g is None else g.reshape(1).contiguous().float()  # noqa: E731
        g1_, g2_, gs_ = dev(g1), dev(g2), dev(gsum)
        nat.check(nat.load().dtp_mse_pair_bwd(nat.ptr(a1_), nat.ptr(a2_), nat.ptr(b_), nat.ptr(g1_), nat.ptr(g2_),
                                              nat.ptr(gs_), b_.numel(), nat.ptr(ga1), nat.ptr(ga2), nat.ptr(gb),
                                              nat.stream_ptr()), "dtp_mse_pair_bwd")
        view = lambda t: None if t is None else t.view(ctx.shape)  # noqa: E731
        return view(ga1), view(ga2), view(gb), None


def mse_loss_pair(input1: torch.Tensor, input2: torch.Tensor, target: torch.Tensor, log=None):
    """(mse(input1, target), mse(input2, target), their sum): the reference's two models'
    losses on one batch (``loss_X + loss_Y``) in ONE launch forward and one backward on
    the GPU (the unfused form is 2 forward launches, an add and 2 backward launches);
    torch's ops elsewhere.  The same values, bit for bit, as the separate calls.

    ``log``: a device loss log ``(rows [cap, >= 2] fp32, slot [1] int64)`` -- the
    engine's ``LossRing`` -- into whose row ``slot`` the two losses are also written (slot
    advanced) by the same launch; the caller keeps the slot within ``cap``."""
    if _fused_ok(input1, target) and _fused_ok(input2, target) and (
            log is None or (log[0].is_cuda and log[0].dtype == torch.float32 and log[0].dim() == 2
                            and log[0].shape[1] >= 2 and log[0].is_contiguous() and log[1].dtype == torch.int64)):
        return _FusedMSEPair.apply(input1, input2, target, log)
    l1 = nn.functional.mse_loss(input1, target)
    l2 = nn.functional.mse_loss(input2, target)
    if log is not None:
        rows, slot = log
        rows[:, :2].index_copy_(0, slot, torch.stack([l1.detach(), l2.detach()]).view(1, 2).to(rows.dtype))
        slot.add_(1)
    return l1, l2, l1 + l2


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

    def pair(self, input1: torch.Tensor, input2: torch.Tensor, target: torch.Tensor, log=None):
        """Two predictions against one target: (loss1, loss2, loss1 + loss2) in one fused
        launch (``mse_loss_pair``; reduction="mean" only; ``log``: see there)."""
        if self.reduction != "mean":
            if log is not None:
                raise ValueError("MSELoss.pair(log=...) needs reduction='mean'")
            l1, l2 = self(input1, target), self(input2, target)
            return l1, l2, l1 + l2
        return mse_loss_pair(input1, input2, target, log)
