"""CPU plumbing of the GEMM op and the wide-MLP autograd function (reference path)."""
import pytest
import torch

from distributed_training_pytorch_amd.models.wide import WideMLP
from distributed_training_pytorch_amd.ops.gemm import colsum, gemm


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_gemm_reference_layouts(ta, tb):
    a = torch.randn(7, 5) if not ta else torch.randn(5, 7)
    b = torch.randn(3, 5) if not tb else torch.randn(5, 3)
    A = a.t() if ta else a
    B = b.t() if tb else b
    torch.testing.assert_close(gemm(a, b, trans_a=ta, trans_b=tb), A @ B.t())


def test_gemm_shape_errors():
    with pytest.raises(ValueError):
        gemm(torch.randn(4, 5), torch.randn(3, 6))
    with pytest.raises(ValueError):
        gemm(torch.randn(4, 5), torch.randn(3, 5, dtype=torch.float64))


def test_wide_mlp_matches_autograd_cpu():
    torch.manual_seed(0)
    m = WideMLP((2, 16, 12, 1))
    x = torch.randn(33, 2, requires_grad=True)
    y = torch.randn(33, 1)
    out = m(x)
    torch.nn.functional.mse_loss(out, y).backward()
    got = [p.grad.clone() for p in m.parameters()] + [x.grad.clone()]
    m.zero_grad()
    x.grad = None
    ref = m.reference_forward(x)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-6)
    torch.nn.functional.mse_loss(ref, y).backward()
    for g, r in zip(got, [p.grad for p in m.parameters()] + [x.grad]):
        torch.testing.assert_close(g, r, rtol=1e-5, atol=1e-6)
    assert m.flat_params.numel() == sum(p.numel() for p in m.parameters())
    torch.testing.assert_close(colsum(torch.ones(4, 3)), torch.full((3,), 4.0))


def test_wide_mlp_fused_grad_accumulates_in_place():
    """Parameters marked with ``mark_fused_grad`` get dz^T h added straight into
    their (flat-view) .grad by the backward; autograd returns nothing for them, the
    grad-ready hooks fire once per parameter per backward, and two backwards
    accumulate exactly like AccumulateGrad."""
    from distributed_training_pytorch_amd.ops.gemm import add_grad_ready_hook, mark_fused_grad

    torch.manual_seed(0)
    m = WideMLP((2, 16, 12, 1))
    ps = list(m.parameters())
    flat_grad = torch.zeros(sum(p.numel() for p in ps))
    o, fired = 0, []
    for p in ps:
        p.grad = flat_grad[o:o + p.numel()].view_as(p)
        o += p.numel()
        mark_fused_grad(p)
        add_grad_ready_hook(p, lambda q: fired.append(q))
    x, y = torch.randn(33, 2), torch.randn(33, 1)
    for _ in range(2):
        torch.nn.functional.mse_loss(m(x), y).backward()
    assert len(fired) == 2 * len(ps) and all(any(q is p for q in fired) for p in ps)
    assert all(p.grad.data_ptr() == flat_grad[0:1].data_ptr() + 4 * sum(q.numel() for q in ps[:i])
               for i, p in enumerate(ps)), "grads must stay views of the flat buffer"
    got = flat_grad.clone()
    ref = WideMLP((2, 16, 12, 1))
    ref.load_state_dict(m.state_dict())
    for _ in range(2):
        torch.nn.functional.mse_loss(ref.reference_forward(x), y).backward()
    torch.testing.assert_close(got, torch.cat([p.grad.reshape(-1) for p in ref.parameters()]), rtol=1e-5, atol=1e-6)


def test_gemm_single_backend():
    """ops/gemm.py has one backend (the HIP kernels; hipBLASLt is an A/B reference in
    scripts/blaslt_ref.py); on CPU tensors it runs the PyTorch reference of the same math."""
    from distributed_training_pytorch_amd.ops import gemm as g

    assert not any(hasattr(g, n) for n in ("set_backend", "get_backend", "tuned_choices", "_gemm_blaslt"))
    a, b = torch.randn(64, 32).bfloat16(), torch.randn(48, 32).bfloat16()
    torch.testing.assert_close(g.gemm(a, b, out_dtype=torch.float32), a.float() @ b.float().t())


@pytest.mark.parametrize("M,N,K,ta,tb,splits", [
    (2048, 2048, 8192, True, True, 4),     # dW of a 2048-wide layer, batch 8192: 64 tiles x 4 slices
    (1024, 1024, 16384, True, True, 16),   # dW of a 1024-wide layer, batch 16384: 16 tiles x 16
    (520, 264, 2048, True, True, 4),       # ragged: 6 tiles, 32 K-tiles -> 4 slices of 8
    (4096, 4096, 8192, True, True, 0),     # 256 tiles fill the chip: no split
    (2048, 2048, 8192 + 64, True, True, 0),  # odd K-tile count: no even slices
    (2048, 2048, 512, True, True, 0),      # 8 K-tiles: slices would drop below 8
])
def test_ph8_split_k_plan(M, N, K, ta, tb, splits):
    """The 8-phase GEMM's split-K plan (host code in libdtp.so, no GPU needed): slices
    only for problems with < 128 256x256 tiles, tiles x slices <= 256, every slice an
    even number (>= 8) of 64-deep K-tiles; the workspace holds one f32 plane per slice."""
    from distributed_training_pytorch_amd import _native as nat

    try:
        lib = nat.load()
    except nat.NativeUnavailable as e:
        pytest.skip(f"native library not built: {e}")
    a = nat.GemmArgs()
    a.A, a.B = 256, 256  # 16-byte aligned addresses; nothing is dereferenced
    a.M, a.N, a.K = M, N, K
    a.lda = M if ta else K
    a.ldb = N if tb else K
    a.dtype, a.out_dtype, a.trans_a, a.trans_b = nat.DT_BF16, nat.DT_F32, int(ta), int(tb)
    a.splitk = 0
    assert lib.dtp_gemm_workspace(a) == 4 * splits * M * N
    a.out_dtype = nat.DT_BF16  # a bf16 output (or an activation epilogue) never splits
    assert lib.dtp_gemm_workspace(a) == 0


def test_compute_shadow_tracks_the_masters():
    """ComputeShadow: the bf16 operands equal w.to(bf16) after every optimizer step
    (the optimizer writes them in its own pass and marks them fresh), and any torch
    in-place write to the masters (an edit, load_state_dict) is detected by the
    version counters and re-cast before the next use."""
    from distributed_training_pytorch_amd.models.bank import ModelBank
    from distributed_training_pytorch_amd.ops.gemm import _compute_weight
    from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig

    torch.manual_seed(0)
    bank = ModelBank(2, hidden=32, depth=2, compute_dtype=torch.bfloat16)
    sh = bank.compute_shadow()
    opt = FlatOptimizer(bank.flat, bank.flat_grad, OptimConfig(lr=1e-2), shadow=sh)
    weights = [p for m in bank.models for n, p in m.layers.named_parameters() if n.endswith("weight")]

    def check():
        for w in weights:
            v = _compute_weight(w, torch.bfloat16)
            assert v.dtype == torch.bfloat16 and torch.equal(v, w.detach().to(torch.bfloat16))

    check()
    for _ in range(3):
        bank.flat_grad.normal_()
        opt.step()
        assert sh._token == sh._current()  # written by the step itself, no re-cast pending
        check()
    with torch.no_grad():
        weights[3].mul_(2.0)
    assert sh._token != sh._current()
    check()
    bank[0].load_state_dict({k: torch.ones_like(t) for k, t in bank[0].state_dict().items()})
    check()
    assert float(_compute_weight(weights[0], torch.bfloat16).float().mean()) == 1.0
    # a rebuilt bank (``.to()`` re-packs the buffers) drops the old shadow's views
    bank = bank.to(torch.float32)
    assert getattr(bank, "_shadow", None) is None
    assert not hasattr(bank[0].layers[0].weight, "_dtp_shadow")
    # fp32 compute never uses it
    w = bank[0].layers[0].weight
    assert _compute_weight(w, torch.float32).dtype == torch.float32
