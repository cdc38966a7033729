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
    _DevBatch(X, Y, idx, None).gather_into(idx, out)
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


def _ring_loader(device, shuffle, world=1, rank=0):
    from distributed_training_pytorch_amd.trainer.trainer import _DeviceBatches

    g = torch.Generator().manual_seed(3)
    X = torch.randn(500, 2, generator=g).to(device)  # 500 = 3 full batches of 128 + a short one
    Y = torch.randn(500, 1, generator=g).to(device)
    loader = _DeviceBatches(X, Y, 128, world, rank, shuffle=shuffle)
    if device == "cpu":  # the ring's bookkeeping on the host (the one-launch form is GPU only)
        loader.ring = torch.zeros(1 + len(loader) * 128, dtype=torch.int64)
    else:
        assert loader.use_ring()
    return loader, X, Y


def _check_ring_epochs(device, shuffle, world=1):
    from distributed_training_pytorch_amd.data.sampler import torch_distributed_indices

    loader, X, Y = _ring_loader(device, shuffle, world)
    uploads = []
    real_copy = loader.ring.copy_
    for epoch, skip in ((0, 0), (1, 0), (2, 2), (3, 0)):
        loader.set_epoch(epoch)
        loader.skip = skip
        before = loader._ring_idx
        ref = torch_distributed_indices(500, world, 0, epoch, 0, shuffle)
        for b, dev in enumerate(loader):
            if b < skip:
                continue
            n = dev.sel.shape[0]
            out = [torch.empty(n, 2, device=device), torch.empty(n, 1, device=device)]
            dev.gather_into(None, out)
            rows = torch.tensor(ref[b * 128:(b + 1) * 128], device=device)
            assert torch.equal(out[0], X[rows]) and torch.equal(out[1], Y[rows]), (epoch, b)
        uploads.append(loader._ring_idx is not before)
    del real_copy
    return uploads


def test_trainer_epoch_ring_bookkeeping_cpu():
    """The epoch ring's cursor: every gathered batch advances it, a resumed epoch starts at
    its skip, and an unchanged order is not uploaded again (host form of the ring gather)."""
    uploads = _check_ring_epochs("cpu", shuffle=False)
    # epoch 2 resumes after 2 batches (uploaded with the cursor there); it then runs to its end,
    # so epoch 3 finds the cursor at a multiple of the epoch and the same order: no upload
    assert uploads == [True, False, True, False]
    assert all(_check_ring_epochs("cpu", shuffle=True, world=2))  # a new order every epoch


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle", [False, True])
def test_trainer_epoch_ring_gather_on_device(shuffle):
    """The one-launch ring gather (the cursor read and advanced on the device) gives every
    epoch's batches in DistributedSampler order, short last batch and resume skips included,
    and a captured gather replays batch after batch with nothing refreshed in between."""
    from distributed_training_pytorch_amd import _native as nat
    from distributed_training_pytorch_amd.data.sampler import torch_distributed_indices

    nat.require(torch.device("cuda", 0))
    _check_ring_epochs("cuda", shuffle, world=2 if shuffle else 1)
    loader, X, Y = _ring_loader("cuda", False)
    it = iter(loader)
    dev = next(it)
    out = [torch.empty(128, 2, device="cuda"), torch.empty(128, 1, device="cuda")]
    dev.gather_into(None, out)  # batch 0, eagerly
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s):
        dev.gather_into(None, out)
    ref = torch_distributed_indices(500, 1, 0, 0, 0, False)
    for k in range(1, 9):  # batches 1, 2, 3, 0, 1, ...: the cursor wraps modulo the 4 steps
        g.replay()
        b = k % 4
        if b == 3:  # the short batch (the Trainer replays its own graph for it)
            continue
        rows = torch.tensor(ref[b * 128:(b + 1) * 128], device="cuda")
        assert torch.equal(out[0], X[rows]) and torch.equal(out[1], Y[rows]), k
    assert int(loader.ring[0]) == 9


@pytest.mark.gpu
def test_mse_loss_pair_writes_the_loss_log_row_in_its_launch():
    """``mse_loss_pair(log=(rows, slot))``: the two losses also land in row ``slot`` of the
    engine's device loss log and the slot advances -- in the loss's own launch, replayed
    by a captured graph row after row."""
    from distributed_training_pytorch_amd.ops.loss import mse_loss_pair

    torch.manual_seed(4)
    rows = torch.full((5, 2), -1.0, device="cuda")
    slot = torch.zeros(1, dtype=torch.int64, device="cuda")
    a1, a2, b = (torch.randn(64, 1, device="cuda") for _ in range(3))
    l1, l2, _ = mse_loss_pair(a1, a2, b, log=(rows, slot))
    torch.cuda.synchronize()
    assert int(slot) == 1 and rows[0, 0] == l1 and rows[0, 1] == l2 and (rows[1:] == -1).all()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s):
        o1, o2, _ = mse_loss_pair(a1, a2, b, log=(rows, slot))
    for k in range(1, 4):
        a1.add_(0.5)
        g.replay()
        torch.cuda.synchronize()
        assert int(slot) == k + 1
        assert rows[k, 0] == o1 and rows[k, 1] == o2
        torch.testing.assert_close(o1, torch.nn.functional.mse_loss(a1, b), rtol=1e-5, atol=1e-7)
    assert (rows[4] == -1).all()


def test_mse_loss_pair_log_cpu_form():
    from distributed_training_pytorch_amd.ops.loss import mse_loss_pair

    rows = torch.zeros(3, 2)
    slot = torch.ones(1, dtype=torch.int64)
    a1, a2, b = torch.randn(8, 1), torch.randn(8, 1), torch.randn(8, 1)
    l1, l2, _ = mse_loss_pair(a1, a2, b, log=(rows, slot))
    assert int(slot) == 2 and rows[1, 0] == l1 and rows[1, 1] == l2 and not rows[0].any() and not rows[2].any()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["torch_shuffle", "device_shuffle", "noshuffle", "sequential"])
def test_sampler_gather_follows_the_batch_indexer(mode):
    """gather_rows2_sampler: the step's indices computed on the device by the engine's
    sampler (torch's exact DistributedSampler order from the device permutation ring, the
    keyed shuffle, the unshuffled orders), the cursor advanced by the kernel -- the same
    rows as the host-side BatchIndexer, step after step across epochs and short batches,
    also when replayed from a captured graph."""
    from distributed_training_pytorch_amd import _native as nat
    from distributed_training_pytorch_amd.data.sampler import BatchIndexer, SamplerGeometry
    from distributed_training_pytorch_amd.ops.gather import gather_rows2_sampler

    nat.require(torch.device("cuda", 0))
    g = torch.Generator().manual_seed(5)
    X = torch.randn(500, 2, generator=g).cuda()
    Y = torch.randn(500, 1, generator=g).cuda()
    geom = SamplerGeometry(n=500, world=2, rank=1, batch=96, seed=4, shuffle=mode.endswith("shuffle") and
                           mode != "noshuffle", distributed=mode != "sequential")
    exact = mode != "device_shuffle"
    ref = BatchIndexer(geom, torch.device("cuda", 0), exact_torch=exact)
    dev_ix = BatchIndexer(geom, torch.device("cuda", 0), exact_torch=exact)
    cfg = geom.to_native()
    ring = dev_ix.permutation_ring()
    assert (ring is not None) == dev_ix.needs_ring()
    if ring is not None:
        ring.native(cfg)
    cursor = torch.full((1,), 3, dtype=torch.int64, device="cuda")
    steps = 3 * geom.steps_per_epoch + 2
    for t in range(3, steps):
        if ring is not None:
            e = geom.batch_pos(t)[0]
            ring.ensure(e, e)
        size = geom.batch_size_at(t)
        ox, oy = torch.empty(size, 2, device="cuda"), torch.empty(size, 1, device="cuda")
        gather_rows2_sampler(X, Y, cfg, cursor, ox, oy)
        idx = ref(t).long()
        assert torch.equal(ox, X[idx]) and torch.equal(oy, Y[idx]), t
    assert int(cursor) == steps
    # replayed: a captured gather draws the next step's batch every replay
    t = steps
    while geom.batch_size_at(t) != geom.batch:
        t += 1
    cursor.fill_(t)
    ox, oy = torch.empty(geom.batch, 2, device="cuda"), torch.empty(geom.batch, 1, device="cuda")
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    if ring is not None:
        ring.ensure(geom.batch_pos(t)[0], geom.batch_pos(t)[0] + 1)
    with torch.cuda.graph(gr, stream=s):
        gather_rows2_sampler(X, Y, cfg, cursor, ox, oy)
    gr.replay()
    torch.cuda.synchronize()
    idx = ref(t).long()
    assert torch.equal(ox, X[idx]) and int(cursor) == t + 1
