"""Data-parallel semantics on CPU with gloo (world_size 2): init broadcast,
gradient averaging == single-process average of the per-rank batch gradients,
replica consistency, global mean loss."""
import torch

from distributed_training_pytorch_amd.data.sampler import EpochIndexStream, SamplerGeometry, torch_distributed_indices
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC, mlp_forward_ref
from distributed_training_pytorch_amd.ops.optim import OptimConfig, adam_update_ref

from .dist_utils import run_ranks

STEPS = 5


def _init(seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(TOY_SPEC.P, generator=g) * 0.3 for _ in range(2)]


def _rank_fn(rank, world, steps):
    ds = ToyData(n=512, seed=1)
    geom = SamplerGeometry(n=512, world=world, rank=rank, batch=128, seed=3)
    tr = FusedTrainer(TOY_SPEC, 2, ds.X, ds.Y, geom, OptimConfig(lr=1e-2), EngineConfig(),
                      init_params=_init(100 + rank))  # different local init: broadcast must win
    tr.train(steps)
    return tr.params.clone(), tr.losses(0, steps)


def _reference(world, steps):
    ds = ToyData(n=512, seed=1)
    # the engine's default sampler is the reference's exact DistributedSampler order
    geoms = [EpochIndexStream(SamplerGeometry(n=512, world=world, rank=r, batch=128, seed=3)) for r in range(world)]
    params = torch.stack(_init(100))
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    cfg = OptimConfig(lr=1e-2)
    losses = []
    for t in range(steps):
        row = []
        for i in range(2):
            gs, ls = [], []
            for g in geoms:
                idx = torch.tensor(g.indices(t))
                p = params[i].clone().requires_grad_(True)
                loss = torch.nn.functional.mse_loss(mlp_forward_ref(p, TOY_SPEC, ds.X[idx]), ds.Y[idx])
                (gr,) = torch.autograd.grad(loss, p)
                gs.append(gr)
                ls.append(loss.item())
            with torch.no_grad():
                adam_update_ref(params[i], m[i], v[i], torch.stack(gs).mean(0), t + 1, cfg)
            row.append(sum(ls) / world)
        losses.append(row)
    return params, torch.tensor(losses)


def test_fused_trainer_gloo_dp_matches_single_process_average():
    res = run_ranks(_rank_fn, 2, (STEPS,))
    ref_p, ref_l = _reference(2, STEPS)
    p0, l0 = res[0]
    p1, l1 = res[1]
    assert torch.equal(p0, p1), "replicas diverged"
    torch.testing.assert_close(p0, ref_p, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(l0, ref_l, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(l1, ref_l, rtol=1e-5, atol=1e-6)


def test_device_sampler_partitions_each_epoch():
    for n, W in [(512, 2), (512, 8), (1000, 3)]:
        seen = []
        for r in range(W):
            g = SamplerGeometry(n=n, world=W, rank=r, batch=64, seed=9)
            for t in range(g.steps_per_epoch):
                seen += g.indices(t)
        total = -(-n // W) * W
        assert len(seen) == total
        assert set(seen) == set(range(n))


def test_torch_order_matches_distributed_sampler():
    from torch.utils.data import DistributedSampler

    ds = list(range(100))
    for W, r, e in [(1, 0, 0), (3, 1, 2), (8, 7, 5)]:
        s = DistributedSampler(ds, num_replicas=W, rank=r, shuffle=True, seed=4)
        s.set_epoch(e)
        assert list(iter(s)) == torch_distributed_indices(100, W, r, e, seed=4)


def _barrier_fn(rank, world):
    import time

    import torch

    from distributed_training_pytorch_amd.parallel.xgmi import DeviceBarrier

    bar = DeviceBarrier(torch.device("cpu"))
    if rank == 1:
        time.sleep(0.3)  # the late rank: rank 0's barrier must wait for it
    t0 = time.perf_counter()
    bar()
    waited = time.perf_counter() - t0
    native = bar.native
    bar.close()
    return waited, native


def test_device_barrier_falls_back_to_the_process_group():
    """Without xGMI buffers (CPU ranks) every rank agrees on the process-group
    barrier; it still synchronises the ranks."""
    res = run_ranks(_barrier_fn, 2, ())
    assert res[0][1] is False and res[1][1] is False
    assert res[0][0] > 0.2  # rank 0 waited for the late rank


def _loss_optim_rank(rank, world, loss, ocfg, steps):
    from distributed_training_pytorch_amd.ops.mlp import MlpSpec

    spec = MlpSpec(2, 10, 5, 4) if loss == "ce" else TOY_SPEC
    ds = ToyData(n=512, seed=3, classes=4 if loss == "ce" else 0)
    geom = SamplerGeometry(n=512, world=world, rank=rank, batch=128, seed=11)
    g = torch.Generator().manual_seed(100)
    init = [torch.randn(spec.P, generator=g) * 0.4 for _ in range(2)]
    tr = FusedTrainer(spec, 2, ds.X, ds.Y, geom, ocfg, EngineConfig(loss=loss), init_params=init)
    tr.train(steps)
    return tr.params.clone(), tr.losses(0, steps)


import pytest  # noqa: E402


@pytest.mark.parametrize("loss,ocfg", [("ce", OptimConfig(lr=1e-2)),
                                       ("mse", OptimConfig("sgd", 5e-2, momentum=0.9, weight_decay=1e-4)),
                                       ("ce", OptimConfig("sgd", 5e-2, momentum=0.9))])
def test_loss_and_optimizer_options_gloo_dp(loss, ocfg):
    """--loss ce / --optimizer sgd on the CPU (gloo, 2 ranks) path against autograd +
    torch.optim (F.cross_entropy, torch.optim.SGD with momentum / weight decay)."""
    from distributed_training_pytorch_amd.ops.mlp import MlpSpec

    from .ref_train import torch_train

    steps = 8
    res = run_ranks(_loss_optim_rank, 2, (loss, ocfg, steps))
    spec = MlpSpec(2, 10, 5, 4) if loss == "ce" else TOY_SPEC
    ds = ToyData(n=512, seed=3, classes=4 if loss == "ce" else 0)
    geoms = [EpochIndexStream(SamplerGeometry(n=512, world=2, rank=r, batch=128, seed=11)) for r in range(2)]
    g = torch.Generator().manual_seed(100)
    init = [torch.randn(spec.P, generator=g) * 0.4 for _ in range(2)]
    rp, rl = torch_train(spec, init, ds.X, ds.Y, geoms, steps, ocfg, loss)
    assert torch.equal(res[0][0], res[1][0])
    torch.testing.assert_close(res[0][0], rp, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(res[0][1], rl, rtol=1e-5, atol=1e-6)


def test_toy_flat_params_follow_a_repack():
    """FlatDDP re-packs a module's parameters into its own flat buffer; ToyModel's
    flat_params / load_flat_ must then read and write the live parameters, not the
    abandoned packing."""
    from distributed_training_pytorch_amd.models.toy import ToyModel
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    torch.manual_seed(0)
    m = ToyModel()
    FlatDDP(m)  # one process: no broadcast; re-packs the parameters
    with torch.no_grad():
        for p in m.parameters():
            p.add_(1.0)
    live = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert torch.equal(m.flat_params, live)
    m.load_flat_(torch.zeros_like(live))
    assert all(bool((p == 0).all()) for p in m.parameters())
