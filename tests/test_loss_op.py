"""Fused MSE loss (``ops/loss.py``, ``csrc/loss.hip``) against torch's fp32 mse_loss."""
import pytest
import torch

from distributed_training_pytorch_amd.ops.loss import MSELoss, mse_loss


def test_mse_loss_cpu_falls_back_to_torch():
    a = torch.randn(37, 3, requires_grad=True)
    b = torch.randn(37, 3)
    out = MSELoss()(a, b)
    ref = torch.nn.functional.mse_loss(a, b)
    assert torch.equal(out, ref)
    assert torch.equal(mse_loss(a, b, "sum"), torch.nn.functional.mse_loss(a, b, reduction="sum"))


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(128, 1), (256, 4), (1000,), (21000, 3)])
def test_mse_loss_fused_matches_torch(shape):
    from distributed_training_pytorch_amd import _native as nat

    nat.require(torch.device("cuda", 0))
    torch.manual_seed(0)
    a = torch.randn(*shape, device="cuda", requires_grad=True)
    b = torch.randn(*shape, device="cuda", requires_grad=True)
    a2 = a.detach().clone().requires_grad_()
    b2 = b.detach().clone().requires_grad_()
    out = mse_loss(a, b)
    assert out.grad_fn is not None and "FusedMSE" in type(out.grad_fn).__name__  # the HIP path ran
    ref = torch.nn.functional.mse_loss(a2, b2)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-7)
    (3.0 * out).backward()
    (3.0 * ref).backward()
    torch.testing.assert_close(a.grad, a2.grad, rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(b.grad, b2.grad, rtol=1e-5, atol=1e-8)


@pytest.mark.gpu
def test_mse_loss_large_inputs_take_torchs_reduction():
    """Above 64 Ki elements the one-workgroup forward would stream everything through one
    CU: torch's multi-block reduction runs instead (same values)."""
    a = torch.randn(70000, 3, device="cuda", requires_grad=True)
    b = torch.randn(70000, 3, device="cuda")
    out = mse_loss(a, b)
    assert "FusedMSE" not in type(out.grad_fn).__name__
    torch.testing.assert_close(out, torch.nn.functional.mse_loss(a, b))


@pytest.mark.gpu
def test_mse_loss_fused_in_a_captured_graph():
    """The loss reads the incoming gradient on the device: it replays inside a hipGraph."""
    from distributed_training_pytorch_amd import _native as nat

    nat.require(torch.device("cuda", 0))
    w = torch.randn(8, 1, device="cuda", requires_grad=True)
    x = torch.randn(64, 8, device="cuda")
    y = torch.randn(64, 1, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up outside the capture
        mse_loss(x @ w, y).backward()
    torch.cuda.current_stream().wait_stream(s)
    w.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss = mse_loss(x @ w, y)
        loss.backward()
    for _ in range(3):
        w.grad.zero_()
        x.copy_(torch.randn_like(x))
        g.replay()
        torch.cuda.synchronize()
        w2 = w.detach().clone().requires_grad_()
        ref = torch.nn.functional.mse_loss(x @ w2, y)
        ref.backward()
        torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(w.grad, w2.grad, rtol=1e-5, atol=1e-7)


@pytest.mark.gpu
def test_trainer_batch_gather_matches_index_select():
    """The Trainer's replayed-step gather of (X, Y) rows: one launch, same rows as two
    index_selects (out-of-range indices clamp instead of faulting)."""
    from distributed_training_pytorch_amd import _native as nat
    from distributed_training_pytorch_amd.trainer.trainer import _DevBatch

    nat.require(torch.device("cuda", 0))
    X = torch.randn(512, 2, device="cuda")
    Y = torch.randn(512, 1, device="cuda")
    idx = torch.randperm(512, device="cuda")[:128]
    out = [torch.empty(128, 2, device="cuda"), torch.empty(128, 1, device="cuda")]
    _DevBatch(X, Y, idx).gather_into(idx, out)
    assert torch.equal(out[0], X[idx]) and torch.equal(out[1], Y[idx])


def test_mse_loss_pair_cpu_is_torchs():
    from distributed_training_pytorch_amd.ops.loss import mse_loss_pair

    a1, a2, b = torch.randn(40, 1), torch.randn(40, 1), torch.randn(40, 1)
    l1, l2, ls = mse_loss_pair(a1, a2, b)
    assert torch.equal(l1, torch.nn.functional.mse_loss(a1, b)) and torch.equal(ls, l1 + l2)


@pytest.mark.gpu
@pytest.mark.parametrize("need2", [True, False])
def test_mse_loss_pair_fused_matches_two_calls_and_an_add(need2):
    """The two models' losses on one batch in one launch each way: the same values as two
    fused MSE calls and an add, and the same gradients (need2=False: the second prediction
    is frozen, as under the Trainer's optimizer toggling)."""
    from distributed_training_pytorch_amd.ops.loss import mse_loss_pair

    torch.manual_seed(1)
    a1 = torch.randn(128, 1, device="cuda", requires_grad=True)
    a2 = torch.randn(128, 1, device="cuda", requires_grad=need2)
    b = torch.randn(128, 1, device="cuda")
    r1 = a1.detach().clone().requires_grad_()
    r2 = a2.detach().clone().requires_grad_(need2)
    l1, l2, ls = mse_loss_pair(a1, a2, b)
    assert "FusedMSEPair" in type(ls.grad_fn).__name__
    q1, q2 = mse_loss(r1, b), mse_loss(r2, b)
    qs = q1 + q2
    assert torch.equal(l1, q1) and torch.equal(l2, q2) and torch.equal(ls, qs)
    ls.backward()
    qs.backward()
    assert torch.equal(a1.grad, r1.grad)
    if need2:
        assert torch.equal(a2.grad, r2.grad)
    # a logged loss used on its own (and the sum) also back-propagates
    a1.grad = None
    r1.grad = None
    l1, _, ls = mse_loss_pair(a1, a2, b)
    (2.0 * l1 + ls).backward()
    q1 = mse_loss(r1, b)
    (2.0 * q1 + (q1 + mse_loss(r2, b))).backward()
    torch.testing.assert_close(a1.grad, r1.grad, rtol=1e-6, atol=1e-8)
