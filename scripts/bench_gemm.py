"""GEMM microbenchmark: the MFMA GEMM of csrc/gemm.hip vs torch.matmul (hipBLASLt)
on the three Linear-layer layouts, bf16 and f32.  Prints one JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd.ops.gemm import gemm  # noqa: E402

DEV = torch.device("cuda", 0)


def timeit(fn, iters):
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


def case(M, N, K, ta, tb, dtype, iters):
    a = (torch.rand(*((K, M) if ta else (M, K)), device=DEV) * 2 - 1).to(dtype)  # uniform [-1, 1): DVFS-honest
    b = (torch.rand(*((K, N) if tb else (N, K)), device=DEV) * 2 - 1).to(dtype)
    out = torch.empty(M, N, device=DEV, dtype=torch.float32 if ta else dtype)
    A = a.t() if ta else a
    Bt = b if tb else b.t()  # [K, N]
    ours = timeit(lambda: gemm(a, b, trans_a=ta, trans_b=tb, out=out), iters)
    classic = timeit(lambda: gemm(a, b, trans_a=ta, trans_b=tb, out=out, fast=False), iters)
    theirs = timeit(lambda: torch.matmul(A, Bt), iters)
    gemm(a, b, trans_a=ta, trans_b=tb, out=out)
    err = (out.float() - torch.matmul(A.float(), Bt.float())).abs().max().item()
    fl = 2.0 * M * N * K
    return {"M": M, "N": N, "K": K, "layout": f"{'T' if ta else 'N'}{'T' if tb else 'N'}", "dtype": str(dtype),
            "ours_ms": round(ours, 4), "ours_tflops": round(fl / ours / 1e9, 1),
            "classic_tflops": round(fl / classic / 1e9, 1),
            "torch_ms": round(theirs, 4), "torch_tflops": round(fl / theirs / 1e9, 1), "max_abs_err": err}


def main():
    cases = [(4096, 4096, 4096), (8192, 8192, 8192), (8192, 4096, 4096), (16384, 1024, 1024)]
    dtypes = ((torch.bfloat16, 20),) if "--bf16" in sys.argv else ((torch.bfloat16, 20), (torch.float32, 5))
    for dtype, its in dtypes:
        for (M, N, K) in cases:
            if dtype == torch.float32 and M * N * K > 4096 ** 3:
                continue
            for ta, tb in ((False, False), (False, True), (True, True)):
                print(json.dumps(case(M, N, K, ta, tb, dtype, its)), flush=True)


if __name__ == "__main__":
    main()
