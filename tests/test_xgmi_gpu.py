"""Multi-rank GPU paths on a single MI355X: two processes share cuda:0, so the
xGMI exchange runs through IPC-mapped uncached buffers (same-device mapping) and
the in-kernel granule protocol; results must equal the host all-reduce path and
the single-process reference.  Also the RCCL step path (1-rank NCCL group,
hipGraph-captured all-reduce)."""
import pytest
import torch

from distributed_training_pytorch_amd.data.sampler import EpochIndexStream, SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC, MlpSpec, mlp_forward_ref
from distributed_training_pytorch_amd.ops.optim import OptimConfig, adam_update_ref

from .dist_utils import run_ranks
from .test_dp_cpu import _init, _reference

pytestmark = pytest.mark.gpu
STEPS = 9


def _gpu_rank(rank, world, comm, steps, launch, sampler="torch", groups="auto"):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ds = ToyData(n=512, seed=1)
    X, Y = ds.device_tensors(dev)
    geom = SamplerGeometry(n=512, world=world, rank=rank, batch=128, seed=3)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, OptimConfig(lr=1e-2),
                      EngineConfig(comm=comm, launch=launch, steps_per_launch=4, sampler=sampler, groups=groups),
                      init_params=_init(100 + rank))
    tr.train(steps)
    tr.synchronize()
    out = (tr.params.cpu(), tr.losses(0, steps), tr.comm)
    tr.close()
    return out


@pytest.mark.parametrize("comm,launch", [("xgmi", "persistent"), ("xgmi", "graph"), ("host", "persistent")])
def test_two_ranks_one_gpu(comm, launch):
    res = run_ranks(_gpu_rank, 2, (comm, STEPS, launch), timeout=300)
    ref_p, ref_l = _reference(2, STEPS)
    for r in range(2):
        p, l, used = res[r]
        assert used == comm, f"rank {r} fell back to {used}"
        torch.testing.assert_close(p, ref_p, rtol=1e-4, atol=2e-5)
        torch.testing.assert_close(l, ref_l, rtol=1e-4, atol=1e-5)
    assert torch.equal(res[0][0], res[1][0]), "replicas diverged"


@pytest.mark.parametrize("launch", ["persistent", "graph"])
def test_two_ranks_split_batch_flat_exchange(launch):
    """groups="on" at per-rank batch 128: each rank runs the step on 2 workgroups per model
    and the 2 x 2 members all-reduce in ONE flat xGMI exchange (4 virtual members)."""
    res = run_ranks(_gpu_rank, 2, ("xgmi", STEPS, launch, "torch", "on"), timeout=300)
    ref_p, ref_l = _reference(2, STEPS)
    for r in range(2):
        p, l, used = res[r]
        assert used == "xgmi", f"rank {r} fell back to {used}"
        torch.testing.assert_close(p, ref_p, rtol=1e-4, atol=2e-5)
        torch.testing.assert_close(l, ref_l, rtol=1e-4, atol=1e-5)
    assert torch.equal(res[0][0], res[1][0]), "replicas diverged"


def test_rccl_step_path_single_rank():
    res = run_ranks(_gpu_rank, 1, ("rccl", STEPS, "persistent"), timeout=300, backend="nccl")
    ref_p, ref_l = _reference(1, STEPS)
    p, l, used = res[0]
    assert used == "rccl"
    torch.testing.assert_close(p, ref_p, rtol=1e-4, atol=2e-5)
    torch.testing.assert_close(l, ref_l, rtol=1e-4, atol=1e-5)


def test_rccl_step_path_torch_sampler_matches_fused():
    """RCCL path with the exact DistributedSampler order (host-built indices per
    step) equals the fused single-rank path fed the same explicit indices; 9 steps
    over a 512-sample / batch-128 epoch cross an epoch boundary."""
    a = run_ranks(_gpu_rank, 1, ("rccl", STEPS, "persistent", "torch"), timeout=300, backend="nccl")
    b = run_ranks(_gpu_rank, 1, ("auto", STEPS, "persistent", "torch"), timeout=300, backend="nccl")
    assert a[0][2] == "rccl"
    torch.testing.assert_close(a[0][0], b[0][0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a[0][1], b[0][1], rtol=1e-5, atol=1e-6)


def _ar_rank(rank, world, n, calls):
    from distributed_training_pytorch_amd.parallel.xgmi import XgmiAllReduce

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ar = XgmiAllReduce(1 << 14, dev)
    outs = []
    for c in range(calls):
        g = torch.Generator().manual_seed(100 * c + rank)
        t = torch.randn(n, generator=g).to(dev)
        if rank == 1 and c % 2 == 0:
            torch.cuda._sleep(2_000_000)  # uneven arrival: rank 1 late on every other call
        ar.all_reduce_(t, scale=0.5)
        outs.append(t.cpu())
    torch.cuda.synchronize()
    ar.check()
    ar.close()
    return outs


def test_xgmi_allreduce_standalone_uneven():
    n, calls = 5000, 6
    res = run_ranks(_ar_rank, 2, (n, calls), timeout=300)
    for c in range(calls):
        ref = sum(torch.randn(n, generator=torch.Generator().manual_seed(100 * c + r)) for r in range(2)) * 0.5
        torch.testing.assert_close(res[0][c], ref, rtol=1e-6, atol=1e-6)
        assert torch.equal(res[0][c], res[1][c]), "ranks disagree"


def _ddp_rank(rank, world, comm):
    from distributed_training_pytorch_amd.models.bank import ModelBank
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    bank = ModelBank(2).to(dev)
    ddp = FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad, first_bucket_mb=0.0005, comm=comm)
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(64, 2, generator=g).to(dev)
    y = torch.randn(64, 1, generator=g).to(dev)
    grads = []
    for _ in range(3):
        bank.zero_grad()
        ox, oy = ddp(x)
        (torch.nn.functional.mse_loss(ox, y) + torch.nn.functional.mse_loss(oy, y)).backward()
        grads.append(bank.flat_grad.cpu().clone())
    ddp.check_comm()
    return grads, ddp.comm, len(ddp._buckets)


def test_flat_ddp_xgmi_matches_host_path():
    a = run_ranks(_ddp_rank, 2, ("xgmi",), timeout=300)
    b = run_ranks(_ddp_rank, 2, ("rccl",), timeout=300)
    assert a[0][1] == "xgmi" and b[0][1] == "rccl" and a[0][2] > 1
    for r in range(2):
        for ga, gb in zip(a[r][0], b[r][0]):
            torch.testing.assert_close(ga, gb, rtol=1e-6, atol=1e-7)
    assert all(torch.equal(x, y) for x, y in zip(a[0][0], a[1][0]))


def _forced_selftest_failure(rank, world):
    import os

    os.environ["DTP_XGMI_SELFTEST_FAIL_RANK"] = "1"  # only rank 1 reports a failed self-test
    return _gpu_rank(rank, world, "xgmi", STEPS, "persistent")


def test_xgmi_selftest_failure_on_one_rank_falls_back_consistently():
    """A self-test failure on ONE rank moves every rank to the RCCL path, with the
    trial step undone everywhere: the replicas stay identical and equal the
    single-process reference."""
    res = run_ranks(_forced_selftest_failure, 2, (), timeout=300)
    ref_p, ref_l = _reference(2, STEPS)
    for r in range(2):
        p, l, used = res[r]
        assert used == "rccl", f"rank {r} kept {used}"
        torch.testing.assert_close(p, ref_p, rtol=1e-4, atol=2e-5)
        torch.testing.assert_close(l, ref_l, rtol=1e-4, atol=1e-5)
    assert torch.equal(res[0][0], res[1][0]), "replicas diverged after the fallback"


H15 = MlpSpec(2, 15, 5, 1)


def _h15_init(seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(H15.P, generator=g) * 0.3 for _ in range(2)]


def _h15_rank(rank, world, steps):
    """MlpSpec(2, 15, 5, 1) (P = 781) at per-rank batch 64: the 4-lanes step owns 4
    parameters per thread, the layout with the most granules per slot -- the receive
    buffer must be sized for it (the buffer rsrc does no bounds check)."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    X, Y = ToyData(n=512, seed=1).device_tensors(dev)
    geom = SamplerGeometry(n=512, world=world, rank=rank, batch=64, seed=3)
    tr = FusedTrainer(H15, 2, X, Y, geom, OptimConfig(lr=1e-2), EngineConfig(comm="xgmi", steps_per_launch=4),
                      init_params=_h15_init(7))
    assert tr.lanes == 4, tr.lanes
    tr.train(steps)
    tr.synchronize()
    out = (tr.params.cpu(), tr.losses(0, steps), tr.comm)
    tr.close()
    return out


def _h15_reference(world, steps):
    ds = ToyData(n=512, seed=1)
    geoms = [EpochIndexStream(SamplerGeometry(n=512, world=world, rank=r, batch=64, seed=3)) for r in range(world)]
    params = torch.stack(_h15_init(7)).double()
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    cfg = OptimConfig(lr=1e-2)
    losses = []
    for t in range(steps):
        row = []
        for i in range(2):
            gs, ls = [], []
            for g in geoms:
                idx = torch.tensor(g.indices(t))
                p = params[i].clone().requires_grad_(True)
                loss = torch.nn.functional.mse_loss(mlp_forward_ref(p, H15, ds.X[idx].double()), ds.Y[idx].double())
                (gr,) = torch.autograd.grad(loss, p)
                gs.append(gr)
                ls.append(loss.item())
            with torch.no_grad():
                adam_update_ref(params[i], m[i], v[i], torch.stack(gs).mean(0), t + 1, cfg)
            row.append(sum(ls) / world)
        losses.append(row)
    return params.float(), torch.tensor(losses, dtype=torch.float32)


def test_two_ranks_h15_lanes_exchange_buffer():
    steps = 8
    res = run_ranks(_h15_rank, 2, (steps,), timeout=300)
    ref_p, ref_l = _h15_reference(2, steps)
    for r in range(2):
        p, l, used = res[r]
        assert used == "xgmi", f"rank {r} fell back to {used}"
        torch.testing.assert_close(p, ref_p, rtol=1e-4, atol=5e-5)
        torch.testing.assert_close(l, ref_l, rtol=1e-4, atol=1e-5)
    assert torch.equal(res[0][0], res[1][0]), "replicas diverged"
