"""Every loss and optimizer the fused kernels claim, against autograd + torch.optim
(tests/ref_train.py): cross-entropy (Stage<2,10,5,4>, F.cross_entropy) and SGD
(momentum, weight decay: torch.optim.SGD) through the persistent, hipGraph and eager
launches, the RCCL grad -> all-reduce -> flat-optimizer path, the stand-alone flat
optimizer kernel, and the in-kernel xGMI exchange (MODE_XGMI_SGD, 2 ranks on one GPU)."""
import pytest
import torch

from distributed_training_pytorch_amd.data.sampler import EpochIndexStream, SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC, MlpSpec
from distributed_training_pytorch_amd.ops.optim import OptimConfig, flat_optimizer_step

from .dist_utils import run_ranks
from .ref_train import torch_train

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
CE_SPEC = MlpSpec(2, 10, 5, 4)
SGD_CFGS = [OptimConfig("sgd", 5e-2), OptimConfig("sgd", 5e-2, momentum=0.9),
            OptimConfig("sgd", 5e-2, momentum=0.9, weight_decay=1e-4), OptimConfig("sgd", 5e-2, weight_decay=1e-4)]


def _init(spec, seed, n=2):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(spec.P, generator=g) * 0.4 for _ in range(n)]


def _data(loss, n=512, seed=3):
    return ToyData(n=n, seed=seed, classes=4 if loss == "ce" else 0)


def _fused(spec, loss, ocfg, launch, steps, spl=4, comm="auto", batch=256, world=1, rank=0, init_seed=100):
    ds = _data(loss)
    X, Y = ds.device_tensors(DEV)
    geom = SamplerGeometry(n=512, world=world, rank=rank, batch=batch, seed=11)
    init = [p.to(DEV) for p in _init(spec, init_seed)]
    tr = FusedTrainer(spec, 2, X, Y, geom, ocfg, EngineConfig(comm=comm, launch=launch, steps_per_launch=spl,
                                                              loss=loss), init_params=init)
    tr.train(steps)
    tr.synchronize()
    out = tr.params.cpu(), tr.losses(0, steps), tr.comm
    tr.close()
    return out


def _expect(spec, loss, ocfg, steps, batch=256, world=1, init_seed=100):
    ds = _data(loss)
    geoms = [EpochIndexStream(SamplerGeometry(n=512, world=world, rank=r, batch=batch, seed=11)) for r in range(world)]
    return torch_train(spec, _init(spec, init_seed), ds.X, ds.Y, geoms, steps, ocfg, loss)


@pytest.mark.parametrize("launch", ["persistent", "graph", "eager"])
def test_fused_cross_entropy_adam(launch):
    steps = 10
    p, l, _ = _fused(CE_SPEC, "ce", OptimConfig(lr=1e-2), launch, steps)
    rp, rl = _expect(CE_SPEC, "ce", OptimConfig(lr=1e-2), steps)
    torch.testing.assert_close(l, rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(p, rp, rtol=1e-3, atol=3e-5)


@pytest.mark.parametrize("launch", ["persistent", "graph", "eager"])
@pytest.mark.parametrize("ci", range(len(SGD_CFGS)))
def test_fused_sgd(launch, ci):
    ocfg = SGD_CFGS[ci]
    steps = 10
    p, l, _ = _fused(TOY_SPEC, "mse", ocfg, launch, steps)
    rp, rl = _expect(TOY_SPEC, "mse", ocfg, steps)
    torch.testing.assert_close(l, rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(p, rp, rtol=1e-4, atol=1e-5)


def test_fused_cross_entropy_sgd_momentum():
    ocfg = OptimConfig("sgd", 5e-2, momentum=0.9, weight_decay=1e-4)
    p, l, _ = _fused(CE_SPEC, "ce", ocfg, "persistent", 12, spl=5)
    rp, rl = _expect(CE_SPEC, "ce", ocfg, 12)
    torch.testing.assert_close(l, rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(p, rp, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("momentum,wd", [(0.0, 0.0), (0.9, 0.0), (0.9, 1e-4), (0.0, 1e-4)])
def test_flat_optimizer_sgd_matches_torch(momentum, wd):
    P = 371
    p0 = torch.randn(2, P, device=DEV)
    ps = [torch.nn.Parameter(p0[i].clone()) for i in range(2)]
    opt = torch.optim.SGD(ps, lr=1e-2, momentum=momentum, weight_decay=wd)
    params = p0.clone()
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    step = torch.zeros(2, dtype=torch.int32, device=DEV)
    cfg = OptimConfig("sgd", 1e-2, momentum=momentum, weight_decay=wd)
    for _ in range(5):
        g = torch.randn(2, P, device=DEV)
        for i in range(2):
            ps[i].grad = g[i].clone()
        opt.step()
        flat_optimizer_step(params, m, v, step, torch.cat([g.reshape(-1), torch.zeros(2, device=DEV)]), cfg)
    torch.testing.assert_close(params, torch.stack([p.detach() for p in ps]), rtol=1e-6, atol=1e-7)
    assert step.tolist() == [5, 5]


def _rank_job(rank, world, comm, spec, loss, ocfg, steps, batch):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    p, l, used = _fused(spec, loss, ocfg, "persistent", steps, spl=4, comm=comm, batch=batch, world=world,
                        rank=rank, init_seed=100)
    return p, l, used


@pytest.mark.parametrize("comm", ["xgmi", "host"])
@pytest.mark.parametrize("loss,optim", [("mse", "sgd"), ("ce", "adam"), ("ce", "sgd")])
def test_two_ranks_loss_optim(comm, loss, optim):
    """MODE_XGMI_SGD / CE through the in-kernel exchange (and the host all-reduce path)
    with two ranks sharing the GPU, against the 2-rank data-parallel torch.optim run."""
    spec = CE_SPEC if loss == "ce" else TOY_SPEC
    ocfg = OptimConfig("sgd", 5e-2, momentum=0.9, weight_decay=1e-4) if optim == "sgd" else OptimConfig(lr=1e-2)
    steps = 9
    res = run_ranks(_rank_job, 2, (comm, spec, loss, ocfg, steps, 128), timeout=300)
    rp, rl = _expect(spec, loss, ocfg, steps, batch=128, world=2)
    for r in range(2):
        p, l, used = res[r]
        assert used == comm
        torch.testing.assert_close(l, rl, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(p, rp, rtol=1e-4, atol=2e-5)
    assert torch.equal(res[0][0], res[1][0]), "replicas diverged"


def test_rccl_path_sgd_single_rank():
    ocfg = OptimConfig("sgd", 5e-2, momentum=0.9)
    res = run_ranks(_rank_job, 1, ("rccl", TOY_SPEC, "mse", ocfg, 9, 128), timeout=300, backend="nccl")
    rp, rl = _expect(TOY_SPEC, "mse", ocfg, 9, batch=128, world=1)
    p, l, used = res[0]
    assert used == "rccl"
    torch.testing.assert_close(l, rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(p, rp, rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("batch,groups", [(64, 1), (128, 2), (256, 4)])
@pytest.mark.parametrize("loss,optim", [("mse", "sgd"), ("ce", "adam"), ("ce", "sgd")])
def test_lanes_and_split_batch_loss_optim(batch, groups, loss, optim):
    """SGD (momentum, weight decay) and cross-entropy on the fast steps: the 4-lanes step
    at per-rank batch 64 and the split-batch step (64 samples per workgroup, batch / 64
    workgroups per model) above it, against autograd + torch.optim."""
    spec = CE_SPEC if loss == "ce" else TOY_SPEC
    ocfg = OptimConfig("sgd", 5e-2, momentum=0.9, weight_decay=1e-4) if optim == "sgd" else OptimConfig(lr=1e-2)
    ds = _data(loss)
    X, Y = ds.device_tensors(DEV)
    geom = SamplerGeometry(n=512, batch=batch, seed=11)
    tr = FusedTrainer(spec, 2, X, Y, geom, ocfg, EngineConfig(steps_per_launch=4, loss=loss, groups="on"),
                      init_params=[p.to(DEV) for p in _init(spec, 100)])
    assert (tr.lanes, tr.groups) == (4, groups)
    steps = 11
    tr.train(steps)
    tr.synchronize()
    p, l = tr.params.cpu(), tr.losses(0, steps)
    tr.close()
    rp, rl = _expect(spec, loss, ocfg, steps, batch=batch)
    torch.testing.assert_close(l, rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(p, rp, rtol=1e-3, atol=3e-5)
