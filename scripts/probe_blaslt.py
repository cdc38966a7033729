"""Wide-MLP layer GEMMs: the fused MFMA kernel vs hipBLASLt (torch) + a separate epilogue.

Shapes are the 2->W^4->1 MLP's hidden layers at batch B: forward (bias + LeakyReLU),
grad input (x LeakyReLU'(h)), grad weight (fp32 accumulate).  One JSON line per case.
Usage: python scripts/probe_blaslt.py [B W]...
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd.ops.gemm import gemm  # noqa: E402

DEV = torch.device("cuda", 0)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def run(B, W):
    bf = torch.bfloat16
    h = (torch.rand(B, W, device=DEV) * 2 - 1).to(bf)
    w = ((torch.rand(W, W, device=DEV) * 2 - 1) / W ** 0.5).to(bf)
    bias = torch.rand(W, device=DEV) - 0.5
    dz = (torch.rand(B, W, device=DEV) * 2 - 1).to(bf)
    gw = torch.zeros(W, W, device=DEV)
    slope = 0.01
    res = {"B": B, "W": W}
    fl = 2.0 * B * W * W

    # forward
    out = torch.empty(B, W, device=DEV, dtype=bf)
    t_ours = timeit(lambda: gemm(h, w, bias=bias, act=True, slope=slope, out=out))
    bb = bias.to(bf)
    out2 = torch.empty(B, W, device=DEV, dtype=bf)

    def fwd_lt():
        torch.addmm(bb, h, w.t(), out=out2)
        F.leaky_relu_(out2, slope)
    t_lt = timeit(fwd_lt)
    ref = F.leaky_relu(h.float() @ w.float().t() + bias, slope)
    res["fwd"] = {"ours_ms": round(t_ours, 4), "lt_ms": round(t_lt, 4), "ours_tf": round(fl / t_ours / 1e9),
                  "lt_tf": round(fl / t_lt / 1e9),
                  "err_ours": (out.float() - ref).abs().max().item(), "err_lt": (out2.float() - ref).abs().max().item()}

    # grad input: dz' = (dz W) * LeakyReLU'(h)
    t_ours = timeit(lambda: gemm(dz, w, trans_b=True, aux=h, slope=slope, out=out))

    def dx_lt():
        torch.mm(dz, w, out=out2)
        return torch.ops.aten.leaky_relu_backward(out2, h, slope, False)
    t_lt = timeit(dx_lt)
    r2 = dx_lt()
    ref = (dz.float() @ w.float()) * torch.where(h.float() > 0, 1.0, slope)
    res["dx"] = {"ours_ms": round(t_ours, 4), "lt_ms": round(t_lt, 4), "ours_tf": round(fl / t_ours / 1e9),
                 "lt_tf": round(fl / t_lt / 1e9),
                 "err_ours": (out.float() - ref).abs().max().item(), "err_lt": (r2.float() - ref).abs().max().item()}

    # grad weight: gw += dz^T h  (fp32 out)
    t_ours = timeit(lambda: gemm(dz, h, trans_a=True, trans_b=True, out=gw, accumulate=True))
    gw2 = torch.zeros(W, W, device=DEV)
    mode = "addmm.dtype"
    try:
        torch.addmm(gw2, dz.t(), h, out_dtype=torch.float32, out=gw2)

        def dw_lt():
            torch.addmm(gw2, dz.t(), h, out_dtype=torch.float32, out=gw2)
    except Exception as e:  # noqa: BLE001
        res["addmm_dtype_error"] = str(e)[:200]
        mode = "mm bf16 + add"

        def dw_lt():
            gw2.add_(torch.mm(dz.t(), h))
    t_lt = timeit(dw_lt)
    gw.zero_()
    gw2.zero_()
    gemm(dz, h, trans_a=True, trans_b=True, out=gw, accumulate=True)
    dw_lt()
    ref = dz.float().t() @ h.float()
    res["dw"] = {"mode": mode, "ours_ms": round(t_ours, 4), "lt_ms": round(t_lt, 4),
                 "ours_tf": round(fl / t_ours / 1e9), "lt_tf": round(fl / t_lt / 1e9),
                 "err_ours": (gw - ref).abs().max().item(), "err_lt": (gw2 - ref).abs().max().item()}
    try:
        o = torch.mm(dz, w, out_dtype=torch.float32)
        res["mm_dtype"] = str(o.dtype)
    except Exception as e:  # noqa: BLE001
        res["mm_dtype_error"] = str(e)[:200]
    return res


def main():
    args = [int(x) for x in sys.argv[1:]] or [8192, 4096, 16384, 1024, 8192, 2048, 4096, 8192]
    for i in range(0, len(args), 2):
        print(json.dumps(run(args[i], args[i + 1])), flush=True)


if __name__ == "__main__":
    main()
