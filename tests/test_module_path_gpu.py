"""The Trainer demo's module-path helpers: several ToyModels on one input forward in ONE
launch (``ToyModel.forward_many`` -> ``ops.mlp.fused_mlp_multi``), against the models'
own fused forwards / backwards (bitwise), including a frozen model (the Trainer's
optimizer toggling) and the CPU fallback."""
import pytest
import torch

from distributed_training_pytorch_amd.models.toy import ToyModel


def test_forward_many_cpu_is_the_models_own():
    torch.manual_seed(0)
    ms = [ToyModel(), ToyModel()]
    x = torch.randn(16, 2)
    outs = ToyModel.forward_many(ms, x)
    for m, o in zip(ms, outs):
        assert torch.equal(o, m(x))


@pytest.mark.gpu
@pytest.mark.parametrize("freeze_second", [False, True])
def test_forward_many_matches_separate_fused_calls(freeze_second):
    torch.manual_seed(3)
    ms = [ToyModel().cuda(), ToyModel().cuda()]
    refs = [ToyModel().cuda(), ToyModel().cuda()]
    for r, m in zip(refs, ms):
        r.load_state_dict(m.state_dict())
    if freeze_second:
        for p in list(ms[1].parameters()) + list(refs[1].parameters()):
            p.requires_grad_(False)
    x = torch.randn(300, 2, device="cuda")  # two blocks of 256 per model
    y = torch.randn(300, 1, device="cuda")
    outs = ToyModel.forward_many(ms, x)
    assert "FusedMLPMulti" in type(outs[0].grad_fn).__name__
    routs = [r(x) for r in refs]
    for o, r in zip(outs, routs):
        assert torch.equal(o, r)
    loss = ((outs[0] - y) ** 2).mean() + ((outs[1] - y) ** 2).mean()
    rloss = ((routs[0] - y) ** 2).mean() + ((routs[1] - y) ** 2).mean()
    loss.backward()
    rloss.backward()
    for m, r in zip(ms, refs):
        for p, q in zip(m.parameters(), r.parameters()):
            if q.grad is None:
                assert p.grad is None
            else:
                assert torch.equal(p.grad, q.grad)


def _train_flat(fuse: bool, opt_name: str, steps: int = 6, batch: int = 200):
    import contextlib

    from distributed_training_pytorch_amd.ops.loss import mse_loss
    from distributed_training_pytorch_amd.ops.mlp import ParamBackwardFusion
    from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    torch.manual_seed(5)
    m = ToyModel().cuda()
    ddp = FlatDDP(m)
    cfg = OptimConfig(name=opt_name, lr=1e-2, momentum=0.9 if opt_name == "sgd" else 0.0)
    opt = FlatOptimizer(ddp.flat_params, ddp.flat_grad, cfg)
    g = torch.Generator(device="cuda").manual_seed(1)
    taken = 0
    for _ in range(steps):
        x = torch.randn(batch, 2, device="cuda", generator=g)
        y = torch.randn(batch, 1, device="cuda", generator=g)
        ddp.zero_grad()
        with (ParamBackwardFusion() if fuse else contextlib.nullcontext()) as fus:
            mse_loss(ddp(x), y).backward()
            pend = fus.take() if fus is not None else None
            taken += pend is not None
            opt.step(zero_grad=True, fused=pend)
    torch.cuda.synchronize()
    return [t.detach().clone() for t in (ddp.flat_params, opt.m, opt.v, opt.step_ctr, ddp.flat_grad)], taken


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name", ["adam", "sgd"])
def test_stage_backward_fused_with_flat_optimizer_is_bitwise_the_pair(opt_name):
    """ParamBackwardFusion: the model's stage backward (adding into its persistent flat
    gradient) and the flat optimizer step over that span in ONE launch
    (``mlp_stage_bwd_opt_kernel``) leave parameters, moments, step counter and the
    (zeroed) gradient bitwise where the two separate launches leave them."""
    from distributed_training_pytorch_amd import _native as nat

    nat.require(torch.device("cuda", 0))
    ref, n0 = _train_flat(False, opt_name)
    got, n1 = _train_flat(True, opt_name)
    assert n0 == 0 and n1 == 6  # every step fused
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    assert int(got[3][0]) == 6 and not got[4].any()


def _fit_lit(root, copies, graphs=True, steps=23, batch=96):
    import csv
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from demo_pytorch_lightning import LitToyModel
    from distributed_training_pytorch_amd.data.toy_data import ToyData
    from distributed_training_pytorch_amd.trainer import Trainer

    torch.manual_seed(0)
    dl = torch.utils.data.DataLoader(ToyData(seed=0), batch_size=batch)
    model = LitToyModel()
    tr = Trainer(gpus=1, max_steps=steps, accelerator="gpu", log_every_n_steps=1, default_root_dir=str(root),
                 enable_progress_bar=False, use_graphs=graphs, enable_checkpointing=False, engine="module",
                 graph_copies=copies)
    tr.fit(model, dl)
    with open(os.path.join(tr._log_dir, "metrics.csv")) as f:
        rows = list(csv.DictReader(f))
    return {k: v.cpu() for k, v in model.state_dict().items()}, rows, tr.graph_replays, tr.callback_metrics


@pytest.mark.gpu
def test_trainer_graph_copies_log_every_step_like_eager(tmp_path):
    """Several graph copies per batch shape (the metric rows stacked once per copies
    batches, each copy's logged outputs kept until its next replay): the same weights and
    the same metrics.csv, row for row, as one copy and as eager batches -- batch 96 of
    512 samples gives a short last batch (a second batch shape) every epoch."""
    from distributed_training_pytorch_amd import _native as nat

    nat.require(torch.device("cuda", 0))
    s4, r4, n4, c4 = _fit_lit(tmp_path / "c4", 4)
    s1, r1, n1, c1 = _fit_lit(tmp_path / "c1", 1)
    se, re_, ne, ce = _fit_lit(tmp_path / "e", 1, graphs=False)
    assert ne == 0 and n1 >= 15 and n4 >= 10, (n1, n4)
    assert len(r4) == len(r1) == len(re_) == 23
    assert r4 == r1 == re_
    assert c4 == c1 == ce
    for k in s1:
        assert torch.equal(s4[k], s1[k]) and torch.equal(s1[k], se[k]), k


def _train_bank(fuse: bool, steps: int = 6, batch: int = 256):
    import contextlib

    from distributed_training_pytorch_amd.models.bank import ModelBank
    from distributed_training_pytorch_amd.ops.loss import MSELoss
    from distributed_training_pytorch_amd.ops.mlp import ParamBackwardFusion
    from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    torch.manual_seed(7)
    bank = ModelBank(2).cuda()
    ddp = FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad)
    opt = FlatOptimizer(bank.flat, bank.flat_grad, OptimConfig(name="adam", lr=1e-2))
    lossf = MSELoss()
    g = torch.Generator(device="cuda").manual_seed(2)
    taken = []
    for _ in range(steps):
        x = torch.randn(batch, 2, device="cuda", generator=g)
        y = torch.randn(batch, 1, device="cuda", generator=g)
        bank.zero_grad()
        with (ParamBackwardFusion() if fuse else contextlib.nullcontext()) as fus:
            ox, oy = ddp(x)
            _, _, lsum = lossf.pair(ox, oy, y)
            lsum.backward()
            pend = fus.take() if fus is not None else None
            taken.append(0 if pend is None else len(pend))
            opt.step(zero_grad=True, fused=pend)
    torch.cuda.synchronize()
    return [t.detach().clone() for t in (bank.flat, opt.m, opt.v, opt.step_ctr, bank.flat_grad)], taken


@pytest.mark.gpu
def test_bank_backwards_fused_with_the_two_model_optimizer_is_bitwise():
    """The module engine's ModelBank under ParamBackwardFusion: both models' stage
    backwards and the one flat Adam over both rows as ONE launch (one block per model),
    bitwise the three separate launches."""
    from distributed_training_pytorch_amd import _native as nat

    nat.require(torch.device("cuda", 0))
    ref, t0 = _train_bank(False)
    got, t1 = _train_bank(True)
    assert t0 == [0] * 6 and t1 == [2] * 6
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    assert not got[4].any()


@pytest.mark.gpu
def test_loss_ring_flush_without_sync_returns_every_row_in_order():
    """LossRing.flush(wait=False): the chunk's copy is queued, its rows come back from a
    later flush (or the final wait=True one) -- every row once, in step order, with the
    values the device wrote."""
    from distributed_training_pytorch_amd.utils.logging import LossRing

    ring = LossRing(4, 2, torch.device("cuda", 0))
    got = []
    for step in range(10):
        v = torch.tensor([float(step), -float(step)], device="cuda")
        ring.put(step, v[0], v[1])
        if ring.full():
            got += ring.flush(wait=False)
    got += ring.flush(wait=True)
    assert [s for s, _ in got] == list(range(10))
    assert all(vals == [float(s), -float(s)] for s, vals in got)


def test_param_backward_fusion_window_cpu():
    """The deferral window's bookkeeping (no GPU): backwards queue in model order, a
    different shape or device flushes what waits, leftovers launch when the window closes,
    an exception drops them, and windows nest."""
    from distributed_training_pytorch_amd.ops import mlp

    launched = []

    class Fake:
        def __init__(self, name, key=(2, 10, 5, 1, 0), device="cuda:0"):
            self.name, self.key, self.device = name, key, device

        def compatible(self, other):
            return other.key == self.key and other.device == self.device

        def launch(self):
            launched.append(self.name)

    with mlp.ParamBackwardFusion() as f:
        assert mlp._FUSION is f
        f.defer(Fake("a"))
        f.defer(Fake("b"))
        assert [p.name for p in f.take()] == ["a", "b"] and f.take() is None
        f.defer(Fake("c"))
        f.defer(Fake("d", key=(2, 15, 5, 1, 0)))  # another shape: "c" goes out first
        assert launched == ["c"]
        with mlp.ParamBackwardFusion() as inner:
            assert mlp._FUSION is inner
        assert mlp._FUSION is f
    assert mlp._FUSION is None and launched == ["c", "d"]  # the leftover launched at exit
    try:
        with mlp.ParamBackwardFusion() as f:
            f.defer(Fake("e"))
            raise RuntimeError("backward failed")
    except RuntimeError:
        pass
    assert launched == ["c", "d"] and mlp._FUSION is None  # dropped
