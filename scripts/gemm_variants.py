"""A/B the fast GEMM's schedule variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24). usage: python scripts/gemm_variants.py [rounds]

VARIANTS=var2,var32,var34,torch  selects variants (fast = 2 + N): var2 the two-buffer
kernel, var32 / var34 the 8-phase kernel with balanced / unbalanced reads, var35 the
balanced 8-phase kernel as a persistent tile walk.
SHAPES=wide  times the wide-MLP GEMMs (W=4096, batch 8192) instead of the squares;
SHAPES=nn the NN per-tile scan."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd.ops.gemm import gemm  # noqa: E402

DEV = torch.device("cuda", 0)


def t_ms(fn, iters=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    variants = os.environ.get("VARIANTS", "var2,var32,var34,torch").split(",")
    shapes = [(4096, 4096, 4096, "NN"), (8192, 8192, 8192, "NN"), (8192, 8192, 8192, "TT"), (8192, 8192, 8192, "NT")]
    if os.environ.get("SHAPES") == "wide":  # forward, input gradient, weight gradient of a 4096-wide layer
        shapes = [(8192, 4096, 4096, "NN"), (8192, 4096, 4096, "NT"), (4096, 4096, 8192, "TT")]
    if os.environ.get("SHAPES") == "nn":  # the per-tile cost scan of profiles/r4_gemm (NN, 2-8 tiles per CU)
        shapes = [(8192, 4096, 2048, "NN"), (8192, 4096, 4096, "NN"), (8192, 4096, 8192, "NN"),
                  (8192, 8192, 4096, "NN"), (16384, 8192, 4096, "NN"), (8192, 8192, 8192, "NN")]
    for (M, N, K, lay) in shapes:
        ta, tb = lay[0] == "T", lay[1] == "T"
        a = (torch.rand(*((K, M) if ta else (M, K)), device=DEV) * 2 - 1).bfloat16()
        b = (torch.rand(*((K, N) if tb else (N, K)), device=DEV) * 2 - 1).bfloat16()
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        A, Bt = (a.t() if ta else a), (b if tb else b.t())
        ref = torch.matmul(A, Bt)
        fns = {}
        for v in variants:
            if v == "torch":
                fns[v] = lambda: torch.matmul(A, Bt, out=out)
            else:
                k = 2 + int(v[3:])
                fns[v] = (lambda k=k: gemm(a, b, trans_a=ta, trans_b=tb, out=out, fast=k))
                fns[v]()
                err = (out.float() - ref.float()).abs().max().item()
                assert err < 1.0, (v, err)
        res = {v: [] for v in variants}
        for _ in range(rounds):
            for v in variants:
                res[v].append(t_ms(fns[v]))
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": [M, N, K], "layout": lay,
                          **{v: round(fl / sorted(ts)[len(ts) // 2] / 1e9, 1) for v, ts in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
