"""Fused MLP ops: spec, PyTorch reference, native HIP wrappers, autograd Function.

The toy network of the reference (``toy_model_and_data.py:8-25``: Linear(2,10),
LeakyReLU, 3x[Linear(10,10), LeakyReLU], Linear(10,1)) is described by an
:class:`MlpSpec`.  Parameters live in ONE flat fp32 buffer in torch's
``parameters()`` order (W0, b0, W1, b1, ...), which is what every kernel reads
and what the data-parallel all-reduce moves in a single message.

CUDA tensors go through the HIP kernels in ``csrc/mlp_train.hip``;
CPU tensors (gloo tests, ``--device cpu``) through the PyTorch reference below.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, replace

import torch
import torch.nn.functional as F

from .. import _native as nat
from .gemm import _fused_grad_target, _grad_ready


@dataclass(frozen=True)
class MlpSpec:
    in_features: int = 2
    hidden: int = 10
    n_layers: int = 5
    out_features: int = 1
    final_act: bool = False
    slope: float = 0.01

    def dims(self) -> list[tuple[int, int]]:
        out = []
        for l in range(self.n_layers):
            din = self.in_features if l == 0 else self.hidden
            dout = self.out_features if l == self.n_layers - 1 else self.hidden
            out.append((din, dout))
        return out

    @property
    def P(self) -> int:
        return sum(o * (i + 1) for i, o in self.dims())

    def param_shapes(self) -> list[tuple[int, ...]]:
        shapes: list[tuple[int, ...]] = []
        for i, o in self.dims():
            shapes += [(o, i), (o,)]
        return shapes

    def act(self, l: int) -> bool:
        return l < self.n_layers - 1 or self.final_act

    def substage(self, a: int, b: int) -> "MlpSpec":
        """Spec of layers a..b (inclusive) as a stand-alone stage."""
        dims = self.dims()
        return replace(self, in_features=dims[a][0], out_features=dims[b][1], n_layers=b - a + 1,
                       final_act=(b < self.n_layers - 1) or self.final_act)

    def param_range(self, a: int, b: int) -> tuple[int, int]:
        """Flat-parameter slice [lo, hi) of layers a..b."""
        dims = self.dims()
        lo = sum(o * (i + 1) for i, o in dims[:a])
        hi = lo + sum(o * (i + 1) for i, o in dims[a:b + 1])
        return lo, hi

    @property
    def key(self) -> tuple[int, int, int, int, int]:
        return (self.in_features, self.hidden, self.n_layers, self.out_features, int(self.final_act))

    def native_supported(self, bf16: bool = False) -> bool:
        try:
            lib = nat.load()
        except nat.NativeUnavailable:
            return False
        return bool(lib.dtp_mlp_supported_bf16(*self.key) if bf16 else lib.dtp_mlp_supported(*self.key))


TOY_SPEC = MlpSpec()


# ----------------------------------------------------------------------------- reference
def unflatten(flat: torch.Tensor, spec: MlpSpec) -> list[torch.Tensor]:
    out, o = [], 0
    for shp in spec.param_shapes():
        n = 1
        for s in shp:
            n *= s
        out.append(flat[o:o + n].view(*shp))
        o += n
    return out


def mlp_forward_ref(flat: torch.Tensor, spec: MlpSpec, x: torch.Tensor) -> torch.Tensor:
    ps = unflatten(flat, spec)
    h = x
    for l in range(spec.n_layers):
        h = F.linear(h, ps[2 * l], ps[2 * l + 1])
        if spec.act(l):
            h = F.leaky_relu(h, spec.slope)
    return h


# ----------------------------------------------------------------------------- native
def _check_f32_cuda(name: str, t: torch.Tensor, device: torch.device, numel: int | None = None):
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"{name} must be on {device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name} must have {numel} elements, got {t.numel()}")


def stage_forward(x: torch.Tensor, flat: torch.Tensor, spec: MlpSpec, save: bool = True,
                  peer_device: torch.device | None = None, force_peer: bool = False, bf16: bool = False):
    """Native forward of one MLP stage. Returns (out [B,OUT], saved [B,(NL-1)*H] or None)
    or, with peer_device, (out, saved, out_peer) where out_peer lives on peer_device and is
    written by the same kernel over xGMI (peer access must be enabled).  ``force_peer``
    makes the epilogue's second store target a distinct buffer even when peer_device is
    x's own device (tests of the hand-off path on a one-GPU box)."""
    lib = nat.require(x.device)
    if x.dim() != 2 or x.shape[1] != spec.in_features:
        raise ValueError(f"input must be [B, {spec.in_features}], got {tuple(x.shape)}")
    dev = x.device
    _check_f32_cuda("x", x, dev)
    _check_f32_cuda("params", flat, dev, spec.P)
    B = x.shape[0]
    out = torch.empty(B, spec.out_features, device=dev, dtype=torch.float32)
    saved = torch.empty(B, (spec.n_layers - 1) * spec.hidden, device=dev, dtype=torch.float32) \
        if (save and spec.n_layers > 1) else None
    out_peer = None
    if peer_device is not None and (torch.device(peer_device) != dev or force_peer):
        out_peer = torch.empty(B, spec.out_features, device=peer_device, dtype=torch.float32)
    a = nat.StageArgs(nat.ptr(x), nat.ptr(flat), nat.ptr(out), nat.ptr(saved), None, None, None, nat.ptr(out_peer),
                      B, spec.slope, 0, int(bf16))
    nat.check(lib.dtp_mlp_stage_fwd(ctypes.byref(a), *spec.key, nat.stream_ptr()), "dtp_mlp_stage_fwd")
    if peer_device is not None:
        return out, saved, (out_peer if out_peer is not None else out)
    return out, saved


class ParamBackwardFusion:
    """A window in which whole-model stage backwards that add into persistent flat
    gradient spans (and want no input gradient) are not launched at once but handed to the
    next flat optimizer step over exactly those spans, which runs them and itself as ONE
    launch (``csrc/mlp_stage.hip:mlp_stage_bwd_opt_kernel``, one block per model;
    ``FlatOptimizer.step(fused=...)``): the Trainer's toggled model (its backward + its
    optimizer: 2 launches -> 1), the module engine's ModelBank (both backwards + the one
    flat Adam over both models: 3 -> 1).

    Opened around ``loss.backward()`` + the optimizer step at one rank: there nothing
    reads the gradient in between (no all-reduce).  Whatever is still pending when the
    window closes normally -- an optimizer over other spans, none at all -- is launched
    as it was; an exception drops it (that backward's gradient is abandoned anyway).
    Reference: PL 1.5's per-optimizer backward + step,
    ``/root/reference/demo_pytorch_lightning.py:27-40``; ``demo.py:105-111``."""

    def __init__(self):
        self.pending: list = []
        self._prev = None

    def __enter__(self):
        global _FUSION
        self._prev, _FUSION = _FUSION, self
        return self

    def __exit__(self, et, ev, tb):
        global _FUSION
        _FUSION = self._prev
        p, self.pending = self.pending, []
        if p and et is None:
            _launch_pending(p)
        return False

    def defer(self, pend) -> None:
        if self.pending and (len(self.pending) >= nat.STAGE_MULTI_MAX or not self.pending[0].compatible(pend)):
            _launch_pending(self.pending)
            self.pending = []
        self.pending.append(pend)

    def take(self):
        """The deferred backwards (model order), or None; the caller launches them."""
        p, self.pending = self.pending, []
        return p or None


_FUSION: ParamBackwardFusion | None = None  # read from autograd's device thread too


class _PendingStageBackward:
    """A deferred ``dtp_mlp_stage_bwd`` launch (its operands kept alive until it runs)."""

    __slots__ = ("args", "key", "keep", "device")

    def __init__(self, args, key, keep, device):
        self.args, self.key, self.keep, self.device = args, key, keep, device

    def compatible(self, other) -> bool:
        return other.key == self.key and other.device == self.device

    def launch(self) -> None:
        nat.check(nat.require(self.device).dtp_mlp_stage_bwd(ctypes.byref(self.args), *self.key, nat.stream_ptr()),
                  "dtp_mlp_stage_bwd")


def _launch_pending(pends) -> None:
    for p in pends:
        p.launch()


def fused_rows_match(pends, params: torch.Tensor, grad: torch.Tensor) -> bool:
    """Whether an optimizer over [n, P] (params, grad) rows is exactly these deferred stage
    backwards, row i = stage i."""
    if not pends or params.dim() != 2 or grad.dim() != 2 or params.shape[0] != len(pends) \
            or grad.shape != params.shape or not grad.is_contiguous() or not params.is_contiguous():
        return False
    P = params.shape[1]
    for i, p in enumerate(pends):
        if (p.keep[1].numel() != P or p.args.params != params[i].data_ptr()
                or p.args.grad_params != grad[i].data_ptr() or not p.compatible(pends[0])):
            return False
    return True


def launch_fused_with_optimizer(pends, opt_args) -> None:
    """The deferred stage backwards and the optimizer step (``opt_args``, one row per
    stage) as ONE launch."""
    m = nat.StageMulti()
    m.n = len(pends)
    for i, p in enumerate(pends):
        m.stage[i] = p.args
    nat.check(nat.require(pends[0].device).dtp_mlp_stage_bwd_opt(ctypes.byref(m), ctypes.byref(opt_args),
                                                                 *pends[0].key, nat.stream_ptr()),
              "dtp_mlp_stage_bwd_opt")


def stage_backward(x, flat, spec: MlpSpec, out, saved, grad_out, need_grad_in: bool = True,
                   grad_params: torch.Tensor | None = None, bf16: bool = False):
    """Native backward of one stage. Returns (grad_in or None, grad_params [P]).

    With ``grad_params`` (a contiguous fp32 [P] span, e.g. the parameters' persistent
    ``.grad`` views in a flat gradient buffer) the kernel ADDS the parameter gradient
    into it instead of returning a fresh tensor for autograd to add."""
    lib = nat.require(x.device)
    dev = x.device
    B = x.shape[0]
    grad_out = grad_out.contiguous()
    if grad_out.device != dev and grad_out.device.type == "cuda":
        pass  # peer read over xGMI (layer split): the kernel loads it through the peer mapping
    else:
        _check_f32_cuda("grad_out", grad_out, dev, B * spec.out_features)
    grad_in = torch.empty(B, spec.in_features, device=dev, dtype=torch.float32) if need_grad_in else None
    nblk = (B + 1023) // 1024
    acc = grad_params is not None
    if acc:
        _check_f32_cuda("grad_params", grad_params, dev, spec.P)
        gp = grad_params
    else:
        gp = torch.zeros(spec.P, device=dev, dtype=torch.float32) if nblk > 1 else \
            torch.empty(spec.P, device=dev, dtype=torch.float32)
    a = nat.StageArgs(nat.ptr(x), nat.ptr(flat), nat.ptr(out), nat.ptr(saved), nat.ptr(grad_out),
                      nat.ptr(grad_in), nat.ptr(gp), None, B, spec.slope, int(acc), int(bf16))
    fus = _FUSION
    if fus is not None and acc and not need_grad_in and not bf16 and nblk == 1 and grad_out.device == dev \
            and gp.numel() == spec.P:
        # handed to the next flat optimizer step over this span (ParamBackwardFusion)
        fus.defer(_PendingStageBackward(a, spec.key, (x, flat, out, saved, grad_out, gp), dev))
        return grad_in, gp
    nat.check(lib.dtp_mlp_stage_bwd(ctypes.byref(a), *spec.key, nat.stream_ptr()), "dtp_mlp_stage_bwd")
    return grad_in, gp


def _flat_view_of(params: list[torch.Tensor]) -> torch.Tensor | None:
    """If params are consecutive views of one contiguous storage, return that flat span."""
    if not params:
        return None
    p0 = params[0]
    base = p0.data_ptr()
    off = 0
    for p in params:
        if not p.is_contiguous() or p.data_ptr() != base + off * 4 or p.dtype != torch.float32:
            return None
        off += p.numel()
    st = p0.untyped_storage()
    start = (base - st.data_ptr()) // 4
    full = torch.empty(0, dtype=torch.float32, device=p0.device).set_(st, start, (off,), (1,))
    return full


class FusedMLPFunction(torch.autograd.Function):
    """y = MLP(x) with the forward and the whole backward (dX chain + MFMA dW
    reduction) each in ONE kernel, instead of ~9 GEMM + ~10 elementwise launches."""

    @staticmethod
    def forward(ctx, x, spec: MlpSpec, bf16: bool, *params):
        flat = _flat_view_of(list(params))
        if flat is None:
            flat = torch.cat([p.detach().reshape(-1) for p in params])
        flat = flat.detach()
        x = x.contiguous()
        out, saved = stage_forward(x, flat, spec, save=True, bf16=bf16)
        ctx.spec = spec
        ctx.bf16 = bf16
        ctx.shapes = [p.shape for p in params]
        ctx.params = params
        ctx.save_for_backward(x, flat, out, saved if saved is not None else torch.empty(0, device=x.device))
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, flat, out, saved = ctx.saved_tensors
        spec = ctx.spec
        params = ctx.params
        # parameters whose .grad is a persistent view of one flat gradient span
        # (ModelBank / FlatDDP, ops.gemm.mark_fused_grad): the kernel adds into it, so
        # autograd runs no AccumulateGrad add kernel per parameter tensor
        target = None
        if all(ctx.needs_input_grad[3:]) and all(_fused_grad_target(p) is not None for p in params):
            target = _flat_view_of([p.grad for p in params])
        gin, gp = stage_backward(x, flat, spec, out, saved if saved.numel() else None, grad_out.float(),
                                 need_grad_in=ctx.needs_input_grad[0], grad_params=target, bf16=ctx.bf16)
        if target is not None:
            for p in params:
                _grad_ready(p)
            return (gin, None, None, *([None] * len(params)))
        grads, o = [], 0
        for shp in ctx.shapes:
            n = 1
            for s in shp:
                n *= s
            grads.append(gp[o:o + n].view(shp))
            o += n
        return (gin, None, None, *grads)


def _stage_param_grads(spec, x, flat, out, saved, grad_out, params, shapes, need_params: bool, need_x: bool):
    """One model's backward (FusedMLPFunction.backward's body): (grad_in, [param grads]
    or [None]*n when added in place into persistent flat .grad views)."""
    target = None
    if need_params and all(_fused_grad_target(p) is not None for p in params):
        target = _flat_view_of([p.grad for p in params])
    gin, gp = stage_backward(x, flat, spec, out, saved if saved.numel() else None, grad_out.float(),
                             need_grad_in=need_x, grad_params=target)
    if target is not None:
        for p in params:
            _grad_ready(p)
        return gin, [None] * len(params)
    if not need_params:
        return gin, [None] * len(params)
    grads, o = [], 0
    for shp in shapes:
        n = 1
        for d in shp:
            n *= d
        grads.append(gp[o:o + n].view(shp))
        o += n
    return gin, grads


class FusedMLPMultiFunction(torch.autograd.Function):
    """(MLP_0(x), ..., MLP_{n-1}(x)) for n models of ONE shape on the same input: the n
    forwards in ONE launch (``dtp_mlp_stage_fwd_multi``), each backward its own launch,
    only for the models whose outputs get a gradient and whose parameters want one (the
    Trainer toggles the other optimizer's models off)."""

    @staticmethod
    def forward(ctx, x, spec: MlpSpec, n: int, *params):
        ctx.set_materialize_grads(False)
        k = len(params) // n
        groups = [params[i * k:(i + 1) * k] for i in range(n)]
        x = x.contiguous()
        dev = x.device
        B = x.shape[0]
        m = nat.StageMulti()
        m.n = n
        flats, outs, saveds = [], [], []
        for i, ps in enumerate(groups):
            flat = _flat_view_of(list(ps))
            if flat is None:
                flat = torch.cat([p.detach().reshape(-1) for p in ps])
            flat = flat.detach()
            out = torch.empty(B, spec.out_features, device=dev, dtype=torch.float32)
            saved = torch.empty(B, (spec.n_layers - 1) * spec.hidden, device=dev, dtype=torch.float32) \
                if spec.n_layers > 1 else torch.empty(0, device=dev)
            m.stage[i] = nat.StageArgs(nat.ptr(x), nat.ptr(flat), nat.ptr(out), nat.ptr(saved) if saved.numel() else None,
                                       None, None, None, None, B, spec.slope, 0, 0)
            flats.append(flat)
            outs.append(out)
            saveds.append(saved)
        nat.check(nat.require(dev).dtp_mlp_stage_fwd_multi(ctypes.byref(m), *spec.key, nat.stream_ptr()),
                  "dtp_mlp_stage_fwd_multi")
        ctx.spec, ctx.n, ctx.k = spec, n, k
        ctx.groups = groups
        ctx.shapes = [p.shape for p in groups[0]]
        ctx.save_for_backward(x, *flats, *outs, *saveds)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        n, k = ctx.n, ctx.k
        saved_t = ctx.saved_tensors
        x = saved_t[0]
        flats, outs, saveds = saved_t[1:1 + n], saved_t[1 + n:1 + 2 * n], saved_t[1 + 2 * n:1 + 3 * n]
        need = ctx.needs_input_grad
        gx = None
        grads = []
        for i in range(n):
            g = gouts[i]
            need_p = any(need[3 + i * k:3 + (i + 1) * k])
            if g is None or not (need_p or need[0]):
                grads.extend([None] * k)
                continue
            gin, gp = _stage_param_grads(ctx.spec, x, flats[i], outs[i], saveds[i], g, ctx.groups[i], ctx.shapes,
                                         need_p, need[0])
            if gin is not None:
                gx = gin if gx is None else gx + gin
            grads.extend(gp)
        return (gx, None, None, *grads)


def fused_mlp_multi(x: torch.Tensor, spec: MlpSpec, param_lists: list[list[torch.Tensor]]) -> tuple:
    """n models of one shape on the same input, forwards in one launch (fp32 GPU);
    elsewhere the models' forwards one by one."""
    if x.is_cuda and nat.native_enabled() and spec.native_supported() and 1 <= len(param_lists) <= nat.STAGE_MULTI_MAX:
        return FusedMLPMultiFunction.apply(x, spec, len(param_lists), *[p for ps in param_lists for p in ps])
    return tuple(fused_mlp(x, spec, ps) for ps in param_lists)


def fused_mlp(x: torch.Tensor, spec: MlpSpec, params: list[torch.Tensor], bf16: bool = False) -> torch.Tensor:
    """The whole MLP as one fused forward and one fused backward kernel.  ``bf16``:
    bf16 compute (bf16 weights / activations / gradients as matmul operands, fp32
    accumulation, fp32 weight gradients -- torch.autocast's recipe)."""
    if x.is_cuda and nat.native_enabled():
        lib = nat.require(x.device)  # raises if the library is missing
        ok = lib.dtp_mlp_supported_bf16(*spec.key) if bf16 else spec.native_supported()
        if not ok:
            raise NotImplementedError(f"no fused {'bf16 ' if bf16 else ''}kernel instantiated for {spec}")
        return FusedMLPFunction.apply(x, spec, bool(bf16), *params)
    flat = torch.cat([p.reshape(-1) for p in params])
    return mlp_forward_ref(flat, spec, x)


def bf16_round(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(t.dtype)


def mlp_forward_ref_bf16(flat: torch.Tensor, spec: MlpSpec, x: torch.Tensor) -> torch.Tensor:
    """PyTorch reference of the bf16-compute kernels (fp32 tensors holding bf16 values:
    bf16 operands, fp32 accumulation, bf16 rounding of every matmul output and
    activation) -- differentiable, its backward rounds the gradients the same way."""
    class _R(torch.autograd.Function):
        @staticmethod
        def forward(ctx, t):
            return bf16_round(t)

        @staticmethod
        def backward(ctx, g):
            return bf16_round(g)

    ps = unflatten(flat, spec)
    h = _R.apply(x)
    for l in range(spec.n_layers):
        h = _R.apply(F.linear(h, _R.apply(ps[2 * l]), _R.apply(ps[2 * l + 1])))
        if spec.act(l):
            h = _R.apply(F.leaky_relu(h, spec.slope))
    return h
