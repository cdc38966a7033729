"""Flat-buffer optimizers (Adam / SGD) over [n_models, P] parameters.

The math is the element-for-element mirror of torch.optim.Adam / SGD
(``csrc/optim_core.h``); the PyTorch reference below is used on CPU and by the
numerics tests.  The reference trains with Adam(lr=1e-3) (``demo.py:80-81``).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

import torch

from .. import _native as nat


@dataclass
class OptimConfig:
    name: str = "adam"  # "adam" | "sgd"
    lr: float = 1e-3
    betas: tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    momentum: float = 0.0

    @property
    def kind(self) -> int:
        if self.name == "adam":
            return nat.MODE_ADAM
        if self.name == "sgd":
            return nat.MODE_SGD
        raise ValueError(f"unknown optimizer {self.name!r}")

    def hyper(self, slope: float = 0.01, grad_scale: float = 1.0) -> nat.Hyper:
        return nat.Hyper(self.lr, self.betas[0], self.betas[1], self.eps, self.weight_decay, self.momentum,
                         slope, grad_scale)

    def torch_optimizer(self, params):
        if self.name == "adam":
            return torch.optim.Adam(params, lr=self.lr, betas=self.betas, eps=self.eps,
                                    weight_decay=self.weight_decay)
        return torch.optim.SGD(params, lr=self.lr, momentum=self.momentum, weight_decay=self.weight_decay)


def adam_update_ref(p: torch.Tensor, m: torch.Tensor, v: torch.Tensor, g: torch.Tensor, t1: int,
                    cfg: OptimConfig) -> None:
    """In-place Adam step number t1 (1-based) with torch's operation order (fp32)."""
    b1, b2 = cfg.betas
    if cfg.weight_decay:
        g = g + cfg.weight_decay * p
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** t1
    bc2 = 1 - b2 ** t1
    denom = (v.sqrt() / math.sqrt(bc2)).add_(cfg.eps)
    p.addcdiv_(m, denom, value=-(cfg.lr / bc1))


def adam_bias_table(cfg: "OptimConfig", max_len: int = 1 << 22):
    """Adam's per-step scalars as the fused kernels use them: row t = {lr / (1 - b1^t),
    sqrt(1 - b2^t)} in float32, formed in float64 exactly as the kernels' own fill does
    (``pow_int``: repeated squaring, ``csrc/dtp_common.h``), so a launch reading this
    table is bitwise the launch that forms the scalars itself.  The table ends at the
    first t where both corrections are exactly 1.0 in float64; every later step uses
    that last row.  None if that takes more than ``max_len`` steps (beta ~ 1)."""
    import numpy as np

    b1, b2 = float(cfg.betas[0]), float(cfg.betas[1])

    def pow_int(b: float, t: "np.ndarray") -> "np.ndarray":
        r = np.ones(t.shape, dtype=np.float64)
        base = np.full(t.shape, b, dtype=np.float64)
        e = t.copy()
        while e.any():
            r = np.where(e & 1, r * base, r)
            base = base * base
            e >>= 1
        return r

    n = 1024
    while True:
        t = np.arange(n, dtype=np.int64)
        bc1 = 1.0 - pow_int(b1, t)
        bc2 = 1.0 - pow_int(b2, t)
        done = np.nonzero((bc1 == 1.0) & (bc2 == 1.0))[0]
        if done.size or n >= max_len:
            break
        n *= 2
    if not done.size:
        return None
    T = int(done[0])
    with np.errstate(divide="ignore"):
        tab = np.stack([(float(cfg.lr) / bc1[:T + 1]).astype(np.float32),
                        np.sqrt(bc2[:T + 1]).astype(np.float32)], axis=1)
    return tab


def sgd_update_ref(p: torch.Tensor, buf: torch.Tensor, g: torch.Tensor, first: bool, cfg: OptimConfig) -> None:
    if cfg.weight_decay:
        g = g + cfg.weight_decay * p
    if cfg.momentum:
        if first:
            buf.copy_(g)
        else:
            buf.mul_(cfg.momentum).add_(g)
        g = buf
    p.add_(g, alpha=-cfg.lr)


def flat_optimizer_step(params, m, v, step, grad, cfg: OptimConfig, grad_scale: float = 1.0,
                        loss_log=None, loss_scale: float = 1.0, slope: float = 0.01, shadow=None,
                        zero_grad: bool = False, fused=None) -> None:
    """One optimizer step over [n_models, P] flat buffers.

    ``grad`` is [n_models*P (+ n_models losses)] -- the all-reduced comm buffer;
    ``step`` is the per-model int32 step counter (device or CPU); ``shadow`` (optional,
    bf16 [n_models, >= P], unit column stride) receives the updated parameters rounded
    to bf16 in the same pass, row i at ``shadow[i, :P]``.  ``zero_grad``: the gradient
    rows are zeroed in the same pass once read (the loss slots are not).  ``fused``: a
    deferred stage backward (``ops.mlp.ParamBackwardFusion``) whose span is exactly this
    optimizer's rows (row i = stage i): the backwards and this step run as one launch.
    """
    n_models, P = params.shape
    if shadow is not None and (shadow.dtype != torch.bfloat16 or shadow.dim() != 2 or shadow.shape[0] != n_models
                               or shadow.shape[1] < P or shadow.stride(1) != 1 or shadow.device != params.device):
        raise ValueError("flat_optimizer_step: shadow must be a bf16 [n_models, >= P] tensor with unit column stride")
    if params.is_cuda and nat.native_enabled():
        lib = nat.require(params.device)
        a = nat.OptArgs(nat.ptr(params), nat.ptr(m), nat.ptr(v), nat.ptr(step), nat.ptr(grad),
                        nat.ptr(loss_log), 0 if loss_log is None else loss_log.shape[0], n_models, P, cfg.kind,
                        loss_scale, 1 if zero_grad else 0, cfg.hyper(slope, grad_scale), nat.ptr(shadow),
                        0 if shadow is None else shadow.stride(0))
        if fused is not None:  # the stage backwards that produced `grad`, in the same launch
            from .mlp import launch_fused_with_optimizer

            launch_fused_with_optimizer(fused, a)
            return
        nat.check(lib.dtp_flat_optimizer(ctypes.byref(a), nat.stream_ptr()), "dtp_flat_optimizer")
        return
    if fused is not None:
        for p in fused:
            p.launch()
    g = grad[: n_models * P].view(n_models, P) * grad_scale
    for i in range(n_models):
        t = int(step[i])
        if cfg.name == "adam":
            adam_update_ref(params[i], m[i], v[i], g[i], t + 1, cfg)
        else:
            sgd_update_ref(params[i], m[i], g[i], t == 0, cfg)
        if loss_log is not None:
            loss_log[t % loss_log.shape[0], i] = grad[n_models * P + i] * loss_scale
        step[i] = t + 1
    if zero_grad:
        grad[: n_models * P].zero_()
    if shadow is not None:
        shadow[:, :P].copy_(params)


class FlatOptimizer:
    """Adam/SGD over flat [n_models, P] (or [P]) params + grads in one kernel launch
    (replaces the reference's two torch.optim.Adam, each ~7 kernels x 10 tensors)."""

    def __init__(self, flat_params: torch.Tensor, flat_grad: torch.Tensor, cfg: OptimConfig | None = None,
                 slope: float = 0.01, shadow=None):
        """``shadow``: an ``ops.gemm.ComputeShadow`` of ``flat_params``; every step also
        writes its bf16 copy (the bf16-compute forward then needs no weight casts)."""
        self.shadow = shadow
        if shadow is not None and shadow.flat.data_ptr() != flat_params.data_ptr():
            raise ValueError("FlatOptimizer: the shadow must be of flat_params")
        self.params = flat_params if flat_params.dim() == 2 else flat_params.view(1, -1)
        self.grad = flat_grad if flat_grad.dim() == 2 else flat_grad.view(1, -1)
        self.cfg = cfg or OptimConfig()
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step_ctr = torch.zeros(self.params.shape[0], dtype=torch.int32, device=self.params.device)
        n, P = self.params.shape
        self._buf = None if self.grad.is_contiguous() else \
            torch.zeros(n * P + n, dtype=self.params.dtype, device=self.params.device)
        self.slope = slope

    @torch.no_grad()
    def step(self, zero_grad: bool = False, fused=None) -> bool:
        """One step; ``zero_grad``: zero the gradient in the same launch (no separate fill
        before the next backward).  ``fused``: deferred stage backwards
        (``ops.mlp.ParamBackwardFusion.take()``): run in the same launch when their spans
        are exactly this optimizer's rows, else launched first.  Returns whether the
        gradient was zeroed (not when it had to be staged through a copy)."""
        # the kernel reads grad[i*P : (i+1)*P] only (the loss slots behind them are
        # read only with a loss log), so a contiguous [n, P] gradient is used in place
        n, P = self.params.shape
        sh = self.shadow
        fresh = sh is not None and sh._token == sh._current()  # else the next forward re-casts anyway
        if fused is not None:
            from .mlp import fused_rows_match

            if fresh or not fused_rows_match(fused, self.params, self.grad):
                for p in fused:
                    p.launch()
                fused = None
        if self.grad.is_contiguous() and self.grad.device == self.params.device:
            buf = self.grad.view(-1)
        else:
            self._buf[: n * P].copy_(self.grad.reshape(-1))
            buf = self._buf
            zero_grad = False
        flat_optimizer_step(self.params, self.m, self.v, self.step_ctr, buf, self.cfg, slope=self.slope,
                            shadow=sh.buf if fresh else None, zero_grad=zero_grad, fused=fused)
        if fresh:
            sh.mark_fresh()
        return zero_grad

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.grad.zero_()

    def state_dict(self) -> dict:
        return {"m": self.m.cpu(), "v": self.v.cpu(), "step": self.step_ctr.cpu()}

    def load_state_dict(self, sd: dict) -> None:
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.step_ctr.copy_(sd["step"])
