"""hipBLASLt A/B reference for the wide-MLP GEMMs -- NOT part of the library.

``ops/gemm.py`` has one backend (the HIP kernels).  For the A/B measurements in
``profiles/gemm_r3_ph8/`` the same ``gemm`` contract runs here on hipBLASLt
(``torch.mm`` / ``addmm``, fp32 output through ``out_dtype``) with the epilogue as one
extra in-place elementwise pass.  ``use_blaslt()`` swaps it in for the large bf16
problems of a benchmark process (``scripts/bench_wide.py --gemm-backend blaslt``).
"""
from __future__ import annotations

import torch

from distributed_training_pytorch_amd.ops import gemm as gemm_mod

_MIN_FLOP = 4e9  # smaller problems keep the fused kernel (no extra epilogue pass)


def gemm_blaslt(a, b, trans_a, trans_b, out, bias, aux, act, slope, accumulate, out_dtype):
    """The library's gemm contract, GEMM on hipBLASLt, epilogue in place after it."""
    A = a.t() if trans_a else a        # [M, K]
    Bt = b if trans_b else b.t()       # [K, N]
    lowp = out_dtype == a.dtype
    if accumulate:
        if lowp:
            out.add_(torch.mm(A, Bt))
        else:
            torch.addmm(out, A, Bt, out_dtype=out_dtype, out=out)
        if bias is not None:
            out.add_(bias)
    elif bias is not None:
        if lowp:
            torch.addmm(bias.to(out_dtype), A, Bt, out=out)
        else:
            torch.addmm(bias.float(), A, Bt, out_dtype=out_dtype, out=out)
    elif lowp:
        torch.mm(A, Bt, out=out)
    else:
        torch.mm(A, Bt, out_dtype=out_dtype, out=out)
    if aux is not None:  # out *= LeakyReLU'(aux), one pass, in place
        aux = aux if aux.dtype == out.dtype else aux.to(out.dtype)
        torch.ops.aten.leaky_relu_backward.grad_input(out, aux, slope, False, grad_input=out)
    if act:
        torch.nn.functional.leaky_relu_(out, slope)
    return out


def use_blaslt() -> None:
    """Route this process's large bf16 GEMMs (>= 4 GFLOP, no pinned kernel options)
    through ``gemm_blaslt``; everything else keeps the library kernels."""
    native = gemm_mod.gemm

    def gemm(a, b, *, trans_a=False, trans_b=False, out=None, bias=None, aux=None, act=False, slope=0.01,
             accumulate=False, alpha=1.0, splitk=None, out_dtype=None, force_big=False, fast=None):
        M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
        N = b.shape[1] if trans_b else b.shape[0]
        big = (a.is_cuda and a.dtype == torch.bfloat16 and alpha == 1.0 and K > 16 and min(M, N) > 1
               and 2.0 * M * N * K >= _MIN_FLOP and splitk is None and fast is None and not force_big
               and not (accumulate and (aux is not None or act)))
        if not big:
            return native(a, b, trans_a=trans_a, trans_b=trans_b, out=out, bias=bias, aux=aux, act=act, slope=slope,
                          accumulate=accumulate, alpha=alpha, splitk=splitk, out_dtype=out_dtype,
                          force_big=force_big, fast=fast)
        out_dtype = out_dtype or (out.dtype if out is not None else a.dtype)
        if out is None:
            out = (torch.zeros if accumulate else torch.empty)(M, N, dtype=out_dtype, device=a.device)
        return gemm_blaslt(a, b, trans_a, trans_b, out, bias, aux, act, slope, accumulate, out_dtype)

    gemm_mod.gemm = gemm
