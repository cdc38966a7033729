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
