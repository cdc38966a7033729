"""MFMA GEMM with fused Linear epilogues (``csrc/gemm.hip``) and the wide-MLP op built on it.

The toy model's 10-wide layers run inside the fused train-step kernel
(``ops/mlp.py``); any wider MLP -- ``models/wide.py`` -- runs its Linear layers
through this op: an LDS-tiled MFMA GEMM with the Linear epilogues fused (or, for the
large bf16 problems, hipBLASLt plus one epilogue pass -- see below):

* forward    ``h' = LeakyReLU(h W^T + b)``       bias + activation in the epilogue;
* grad input ``dz' = (dz W) * LeakyReLU'(h)``    activation gradient in the epilogue;
* grad W     ``dW = dz^T h``                     transposed operands staged through
  registers, split-K over blocks when the output has too few tiles;
* grad b     ``db = sum_m dz``                   column-sum kernel.

Replaces the reference's cuBLAS ``addmm``/``mm`` + ATen ``leaky_relu(_backward)``
/ ``sum`` kernels (``toy_model_and_data.py:12-25``).
On CPU tensors every function runs the PyTorch reference of the same math (the
gloo test paths); on a GPU the HIP kernels are required.

One backend: the HIP kernels of this library.  The 256x256 bf16 layer GEMMs run on
the eight-phase LDS-DMA kernel (``csrc/gemm_ph8.hip``), few-tile long-K problems (the
weight gradient of a <= 2048-wide layer) on its split-K plan.  Measured end to end
(``profiles/gemm_r3_ph8/``): 1.30 / 1.81 / 4.64 ms per step on the 1024 / 2048 / 4096-
wide MLPs vs 1.63 / 1.92 / 4.90 with hipBLASLt + an epilogue pass and 2.47 / 2.32 /
5.82 stock.  The hipBLASLt variant used for that A/B lives outside the library
(``scripts/blaslt_ref.py``).
"""
from __future__ import annotations

import math

import torch

from .. import _native as nat

_DT = {torch.float32: nat.DT_F32, torch.bfloat16: nat.DT_BF16}
_BM = 128

def _ld(t: torch.Tensor, name: str) -> int:
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D, got {tuple(t.shape)}")
    if t.stride(1) != 1 and t.shape[1] > 1:
        raise ValueError(f"{name} needs a unit-stride last dimension (got strides {t.stride()})")
    return max(t.stride(0), 1) if t.shape[0] > 1 else max(t.shape[1], 1)


def _ref(a, b, trans_a, trans_b, bias, aux, act, slope, alpha):
    A = (a.t() if trans_a else a).float()
    B = (b.t() if trans_b else b).float()  # [N, K]
    r = alpha * (A @ B.t())
    if bias is not None:
        r = r + bias.float()
    if aux is not None:
        r = r * torch.where(aux.float() > 0, 1.0, slope)
    if act:
        r = torch.nn.functional.leaky_relu(r, slope)
    return r


def _auto_splitk(M: int, N: int, K: int, dtype: torch.dtype) -> int:
    tiles = math.ceil(M / _BM) * math.ceil(N / _BM)
    ktiles = math.ceil(K / (64 if dtype == torch.bfloat16 else 32))
    if tiles >= 128 or ktiles < 8:
        return 1
    return max(1, min(256 // tiles, ktiles // 4))


def gemm(a: torch.Tensor, b: torch.Tensor, *, trans_a: bool = False, trans_b: bool = False,
         out: torch.Tensor | None = None, bias: torch.Tensor | None = None, aux: torch.Tensor | None = None,
         act: bool = False, slope: float = 0.01, accumulate: bool = False, alpha: float = 1.0,
         splitk: int | None = None, out_dtype: torch.dtype | None = None, force_big: bool = False,
         fast: bool | int | None = None) -> torch.Tensor:
    """C[M,N] (+)= epilogue(alpha * A(m,k) B(n,k)).

    ``a`` is [M,K] (or [K,M] with ``trans_a``); ``b`` is [N,K] (or [K,N] with ``trans_b``).
    Epilogue order: + bias[n], * LeakyReLU'(aux[m,n]), LeakyReLU, (+ old C), cast.
    ``fast``: None = pick the kernel by shape; True = the LDS-DMA 256x256 bf16 kernel
    whenever its preconditions hold (K % 64 == 0, aligned rows); False = never.
    """
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    N, Kb = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    if K != Kb:
        raise ValueError(f"gemm: inner dimensions differ ({K} vs {Kb})")
    if a.dtype != b.dtype or a.dtype not in _DT:
        raise ValueError(f"gemm: operands must share dtype float32 or bfloat16 (got {a.dtype}, {b.dtype})")
    out_dtype = out_dtype or (out.dtype if out is not None else a.dtype)
    if out is None:
        out = (torch.zeros if accumulate else torch.empty)(M, N, dtype=out_dtype, device=a.device)
        if not accumulate and nat.debug_enabled():
            out.fill_(float("nan"))  # poisoned: any element the kernel fails to write shows up
    if out.shape != (M, N) or out.dtype != out_dtype:
        raise ValueError(f"gemm: out must be [{M},{N}] {out_dtype}")
    if aux is not None and (aux.shape != (M, N) or aux.dtype != a.dtype):
        raise ValueError("gemm: aux must be [M,N] with the operands' dtype")
    if a.device.type != "cuda" or not nat.native_enabled():
        r = _ref(a, b, trans_a, trans_b, bias, aux, act, slope, alpha)
        if accumulate:
            r = r + out.float()
        out.copy_(r.to(out_dtype))
        return out
    lib = nat.require(a.device)  # loud on a GPU box without the extension
    return _gemm_native(lib, a, b, M, N, K, trans_a, trans_b, out, bias, aux, act, slope, accumulate, alpha,
                        splitk, out_dtype, force_big, fast)


def _gemm_native(lib, a, b, M, N, K, trans_a, trans_b, out, bias, aux, act, slope, accumulate, alpha, splitk,
                 out_dtype, force_big, fast):
    split_ok = out_dtype == torch.float32 and not act and aux is None
    if bias is not None and (bias.dtype != torch.float32 or not bias.is_contiguous()):
        bias = bias.float().contiguous()
    args = nat.GemmArgs()
    args.A, args.B, args.C = nat.ptr(a), nat.ptr(b), nat.ptr(out)
    args.bias = nat.ptr(bias)
    args.aux = nat.ptr(aux)
    args.lda, args.ldb, args.ldc = _ld(a, "a"), _ld(b, "b"), _ld(out, "out")
    args.ldaux = _ld(aux, "aux") if aux is not None else 0
    args.M, args.N, args.K = M, N, K
    args.dtype, args.out_dtype = _DT[a.dtype], _DT[out_dtype]
    args.trans_a, args.trans_b = int(trans_a), int(trans_b)
    args.act, args.accumulate = int(act), int(accumulate)
    args.alpha, args.slope = float(alpha), float(slope)
    args.force_big = int(force_big)
    # int >= 2: force the fast kernel with schedule variant fast - 2 (experiments / benches)
    args.fast = 0 if fast is None else (int(fast) if fast is not True and fast is not False else (1 if fast else -1))
    work = None
    if splitk is None and split_ok:
        # few output tiles, long K (the weight gradient of a <= 2048-wide layer): the
        # library's 8-phase split-K plan, partial sums in a workspace from torch's
        # caching allocator (stream-ordered, hipGraph-capturable); else the classic
        # kernel's atomic split-K
        args.splitk = 0
        nbytes = lib.dtp_gemm_workspace(args)
        if nbytes > 0:
            work = torch.empty(nbytes, dtype=torch.uint8, device=out.device)
            args.work, args.work_bytes = work.data_ptr(), nbytes
        else:
            splitk = _auto_splitk(M, N, K, a.dtype)
    if work is None:
        args.splitk = int(splitk if splitk is not None else 1)
    nat.check(lib.dtp_gemm(args, nat.stream_ptr()), "dtp_gemm")
    return out


def colsum(x: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False) -> torch.Tensor:
    """out[n] (+)= sum_m x[m, n] in fp32 (bias gradients)."""
    M, N = x.shape
    if out is None:
        out = torch.zeros(N, dtype=torch.float32, device=x.device)
    if x.device.type != "cuda" or not nat.native_enabled():
        s = x.float().sum(0)
        out.copy_(out + s if accumulate else s)
        return out
    lib = nat.require(x.device)
    nat.check(lib.dtp_colsum(nat.ptr(x), _ld(x, "x"), M, N, _DT[x.dtype], nat.ptr(out), int(accumulate),
                             nat.stream_ptr()), "dtp_colsum")
    return out


def mark_fused_grad(p: torch.Tensor, on: bool = True) -> None:
    """Let the GEMM backward accumulate this parameter's gradient straight into
    ``p.grad`` (the dW GEMM's epilogue adds into it; the bias column sum likewise)
    instead of returning a fresh tensor that autograd then adds in a separate
    kernel.  For parameters whose ``.grad`` is a persistent view of a flat gradient
    buffer (``ModelBank``, ``FlatDDP``).  Because autograd never sees such a
    gradient, its post-accumulate hooks do not run; hooks registered with
    ``add_grad_ready_hook`` run instead, once the in-place write is enqueued."""
    p._dtp_fused_grad = on


def add_grad_ready_hook(p: torch.Tensor, fn) -> None:
    hooks = getattr(p, "_dtp_grad_ready_hooks", None)
    if hooks is None:
        hooks = p._dtp_grad_ready_hooks = []
    hooks.append(fn)


def _fused_grad_target(p: torch.Tensor) -> torch.Tensor | None:
    g = p.grad
    if (getattr(p, "_dtp_fused_grad", False) and g is not None and g.dtype == torch.float32
            and g.shape == p.shape and g.is_contiguous() and g.device == p.device):
        return g
    return None


def _grad_ready(p: torch.Tensor) -> None:
    for fn in getattr(p, "_dtp_grad_ready_hooks", ()):
        fn(p)


class ComputeShadow:
    """A bf16 copy of a flat fp32 parameter buffer, for the bf16-compute GEMM path.

    ``MLPFunction`` casts every fp32 master weight to bf16 before each forward: one
    launch and 6 B of traffic per parameter.  With a shadow attached, the optimizer
    kernel writes the rounded weights in the same pass as the update (2 B per
    parameter, ``flat_optimizer_step(shadow=...)``) and the forward reads its operands
    from the shadow's views.  The copy is bit-identical to ``w.to(torch.bfloat16)``
    (both round to nearest even).

    Staleness: the shadow is trusted only while the version counters of the flat
    buffer and of every attached parameter are the ones recorded when it was last
    written.  Any torch in-place write (``load_state_dict``, ``copy_``, a broadcast)
    bumps one of them, and the next forward re-casts the whole buffer once.  The
    native optimizer writes through raw pointers (no version bump) and calls
    ``mark_fresh`` after it has written both.

    Layout: a flat [n, P] buffer's shadow is [n, P rounded up to 256] (512-byte rows).
    With an odd P (every bias-terminated MLP row) the rows of a same-shaped bf16 copy
    would start at odd element offsets: the GEMM's 16-byte operand loads need aligned
    rows, and its weight tiles should not straddle cache lines (a 16-byte-aligned but
    not line-aligned shadow ran the W = 4096 forward GEMMs 10 % slower)."""

    def __init__(self, flat: torch.Tensor, params, dtype: torch.dtype = torch.bfloat16):
        if dtype != torch.bfloat16 or flat.dtype != torch.float32 or not flat.is_contiguous():
            raise ValueError("ComputeShadow: a contiguous fp32 flat buffer and a bf16 shadow")
        self.flat, self.params = flat, list(params)
        self._rows = flat if flat.dim() == 2 else flat.view(1, -1)
        n, P = self._rows.shape
        self.buf = torch.empty(n, -(-P // 256) * 256, dtype=dtype, device=flat.device)
        base, es = flat.data_ptr(), flat.element_size()
        for p in self.params:
            r, c = divmod((p.data_ptr() - base) // es, P)
            if p.dtype != flat.dtype or not p.is_contiguous() or not 0 <= r < n or c + p.numel() > P:
                raise ValueError("ComputeShadow: every parameter must be a contiguous view of one flat row")
            p._dtp_shadow = (self, self.buf[r, c:c + p.numel()].view_as(p))
        self._token = None

    def _current(self):
        return (self.flat._version, *(p._version for p in self.params))

    def view(self, p: torch.Tensor) -> torch.Tensor:
        """The bf16 operand for parameter ``p``, re-cast first if the masters changed."""
        if self._token != self._current():
            with torch.no_grad():
                self.buf[:, :self._rows.shape[1]].copy_(self._rows)
            self._token = self._current()
        return p._dtp_shadow[1]

    def mark_fresh(self) -> None:
        self._token = self._current()

    def detach_(self) -> None:
        for p in self.params:
            if getattr(p, "_dtp_shadow", (None,))[0] is self:
                del p._dtp_shadow


def _compute_weight(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    sh = getattr(w, "_dtp_shadow", None)
    if sh is not None and sh[0].buf.dtype == dtype:
        return sh[0].view(w)
    return w.detach().to(dtype).contiguous()


class MLPFunction(torch.autograd.Function):
    """y = L_{n-1}(... LeakyReLU(L_0(x)) ...) with every matmul through ``gemm``.

    ``compute_dtype`` bf16 = autocast-style mixed precision: fp32 master weights
    cast once per forward, bf16 activations, fp32 accumulation and fp32 weight /
    bias gradients; fp32 = exact-fp32 MFMA throughout.
    """

    @staticmethod
    def forward(ctx, x, slope, compute_dtype, *params):
        weights, biases = params[0::2], params[1::2]
        L = len(weights)
        ws = [_compute_weight(w, compute_dtype) for w in weights]
        h = x.detach().to(compute_dtype).contiguous()
        hs = [h]
        for l in range(L):
            last = l == L - 1
            h = gemm(h, ws[l], bias=biases[l].detach(), act=not last, slope=slope,
                     out_dtype=torch.float32 if last else compute_dtype)
            if not last:
                hs.append(h)
        ctx.save_for_backward(*hs, *ws)
        # leaf parameters (not saved tensors): the backward may accumulate into their .grad
        ctx.params = [q if q.is_leaf else None for q in params]
        ctx.L, ctx.slope, ctx.x_dtype = L, slope, x.dtype
        ctx.x_needs = ctx.needs_input_grad[0]
        return h

    @staticmethod
    def backward(ctx, gy):
        L, slope = ctx.L, ctx.slope
        saved = ctx.saved_tensors
        hs, ws = saved[:L], saved[L:]
        cd = ws[0].dtype
        dz = gy.to(cd).contiguous()
        gW: list[torch.Tensor | None] = [None] * L
        gb: list[torch.Tensor | None] = [None] * L
        dx = None
        need = ctx.needs_input_grad[3:]
        for l in range(L - 1, -1, -1):
            pw, pb = ctx.params[2 * l], ctx.params[2 * l + 1]
            tw = _fused_grad_target(pw) if (pw is not None and need[2 * l]) else None
            tb = _fused_grad_target(pb) if (pb is not None and need[2 * l + 1]) else None
            if tw is not None:  # dW += dz^T h in the GEMM epilogue (no separate add kernel)
                gemm(dz, hs[l], trans_a=True, trans_b=True, out=tw, accumulate=True)
            else:
                gW[l] = gemm(dz, hs[l], trans_a=True, trans_b=True, out_dtype=torch.float32)
            if tb is not None:
                colsum(dz, out=tb, accumulate=True)
            else:
                gb[l] = colsum(dz)
            for q, t in ((pw, tw), (pb, tb)):
                if t is not None:
                    _grad_ready(q)
            if l > 0:
                dz = gemm(dz, ws[l], trans_b=True, aux=hs[l], slope=slope, out_dtype=cd)
            elif ctx.x_needs:
                dx = gemm(dz, ws[0], trans_b=True, out_dtype=torch.float32).to(ctx.x_dtype)
        grads = []
        for l in range(L):
            grads += [gW[l], gb[l]]
        return (dx, None, None, *grads)


def mlp(x: torch.Tensor, weights: list[torch.Tensor], biases: list[torch.Tensor], slope: float = 0.01,
        compute_dtype: torch.dtype = torch.float32) -> torch.Tensor:
    params = []
    for w, b in zip(weights, biases):
        params += [w, b]
    return MLPFunction.apply(x, slope, compute_dtype, *params)
