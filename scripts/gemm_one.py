"""Run one GEMM shape through csrc/gemm.hip repeatedly (profiling target).

usage: python scripts/gemm_one.py M N K LAYOUT [iters] [fast|classic|torch]
LAYOUT in NN, NT, TT (trans_a, trans_b as in ops/gemm.py); bf16 operands, uniform [-1, 1).
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd.ops.gemm import gemm  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    ta, tb = sys.argv[4][0] == "T", sys.argv[4][1] == "T"
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 50
    which = sys.argv[6] if len(sys.argv) > 6 else "fast"
    dev = torch.device("cuda", 0)
    a = (torch.rand(*((K, M) if ta else (M, K)), device=dev) * 2 - 1).bfloat16()
    b = (torch.rand(*((K, N) if tb else (N, K)), device=dev) * 2 - 1).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    if which == "torch":
        A, Bt = (a.t() if ta else a), (b if tb else b.t())
        fn = lambda: torch.matmul(A, Bt, out=out)  # noqa: E731
    else:
        fast = which == "fast" or (2 + int(which[3:]) if which.startswith("var") else False)
        fn = lambda: gemm(a, b, trans_a=ta, trans_b=tb, out=out, fast=fast)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    print(f"{which} {M}x{N}x{K} {sys.argv[4]}: {dt * 1e3:.4f} ms  {2.0 * M * N * K / dt / 1e12:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
