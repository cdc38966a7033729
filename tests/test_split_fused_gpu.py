"""The persistent layer-split engine (csrc/split_train.hip, parallel/layer_split.py:
FusedLayerSplit): every stage one resident workgroup, activations / gradients handed
over as epoch-tagged granules through the neighbour's receive buffer, weight
gradients reduced over DP ranks in-kernel, Adam / SGD fused.  Stages share the one
GPU here (distinct streams), so the same peer-store protocol runs through local
uncached memory.  Ground truth: the UNSPLIT model trained with autograd +
torch.optim (tests/ref_train.py)."""
import time

import pytest
import torch

from distributed_training_pytorch_amd.data.sampler import EpochIndexStream, SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC
from distributed_training_pytorch_amd.ops.optim import OptimConfig
from distributed_training_pytorch_amd.parallel.layer_split import FusedLayerSplit

from .dist_utils import run_ranks
from .ref_train import torch_train

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _init(seed=5):
    return torch.randn(TOY_SPEC.P, generator=torch.Generator().manual_seed(seed)) * 0.4


def _engine(K, ocfg, bounds=None, batch=256, world=1, rank=0, seed=11, n=512, members=0, **kw):
    """members=0: the one-workgroup stages (split_train.hip); the split-batch stage
    tests below pass members explicitly."""
    ds = ToyData(n=n, seed=2)
    geom = SamplerGeometry(n=n, world=world, rank=rank, batch=batch, seed=seed)
    return FusedLayerSplit(TOY_SPEC, [DEV] * K, ds.X, ds.Y, geom, ocfg, _init(), boundaries=bounds, members=members,
                           **kw), ds


def _reference(ocfg, steps, batch=256, world=1, seed=11, n=512):
    ds = ToyData(n=n, seed=2)
    # the engine's default order: the reference's DistributedSampler (randperm per epoch)
    geoms = [EpochIndexStream(SamplerGeometry(n=n, world=world, rank=r, batch=batch, seed=seed))
             for r in range(world)]
    p, l = torch_train(TOY_SPEC, [_init()], ds.X, ds.Y, geoms, steps, ocfg, "mse")
    return p[0], l[:, 0]


@pytest.mark.parametrize("K,bounds", [(2, None), (3, None), (2, [(0, 2), (3, 4)]), (5, None)])
@pytest.mark.parametrize("ocfg", [OptimConfig(lr=1e-2), OptimConfig("sgd", 5e-2, momentum=0.9)],
                         ids=["adam", "sgd"])
def test_fused_split_matches_unsplit_reference(K, bounds, ocfg):
    steps = 12
    eng, _ = _engine(K, ocfg, bounds)
    eng.train(5)
    eng.train(steps - 5)  # two launches: the stage state and the link epochs carry over
    eng.synchronize()
    rp, rl = _reference(ocfg, steps)
    torch.testing.assert_close(eng.losses(0, steps), rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(eng.flat_params_cpu(), rp, rtol=1e-4, atol=2e-5)
    assert [int(s.item()) for s in eng.step] == [steps] * K
    eng.close()


def test_fused_split_partial_batches_and_epochs():
    """batch 100 over a 512-sample epoch: 5 full batches and a 12-sample tail per epoch."""
    ocfg = OptimConfig(lr=1e-2)
    steps = 14
    eng, _ = _engine(2, ocfg, batch=100)
    eng.train(steps)
    eng.synchronize()
    rp, rl = _reference(ocfg, steps, batch=100)
    torch.testing.assert_close(eng.losses(0, steps), rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(eng.flat_params_cpu(), rp, rtol=1e-4, atol=2e-5)
    eng.close()


@pytest.mark.parametrize("K", [1, 2])
def test_fused_split_dataset_past_lds_cache(K):
    """4096 samples x (2 inputs + 1 target) floats exceed the stage's LDS data cache
    (8192 floats) on the whole-model stage: that stage gathers from global memory
    through the round-3 body, the cached stages through the pipelined one."""
    ocfg = OptimConfig(lr=1e-2)
    steps = 10
    eng, _ = _engine(K, ocfg, n=4096)
    eng.train(steps)
    eng.synchronize()
    rp, rl = _reference(ocfg, steps, n=4096)
    torch.testing.assert_close(eng.losses(0, steps), rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(eng.flat_params_cpu(), rp, rtol=1e-4, atol=2e-5)
    eng.close()


def test_fused_split_loss_readback_across_a_small_log_ring():
    """A 16-slot loss ring and 8-step launches: launch k+2 rewrites the slots read-back k
    reads, so it must wait for that copy (and only for that one)."""
    ocfg = OptimConfig(lr=1e-2)
    eng, _ = _engine(2, ocfg, log_cap=16)
    handles = []
    for _ in range(5):
        t0 = eng.t
        eng.train(8)
        handles.append(eng.losses_async(t0, t0 + 8))
    got = torch.tensor([r[0] for h in handles for r in h.wait()])
    eng.synchronize()
    _, rl = _reference(ocfg, 40)
    torch.testing.assert_close(got, rl, rtol=1e-4, atol=1e-5)
    eng.close()


def test_fused_split_step_time():
    """The reference's 2-GPU split at batch 256, both stages on one GPU: the whole
    iteration (2 hand-offs + both stages' fwd/bwd/Adam) in microseconds, not the
    ~0.44 ms of the host-driven autograd path."""
    eng, _ = _engine(2, OptimConfig(lr=1e-3))
    eng.train(50)
    eng.synchronize()
    n = 1000
    t0 = time.perf_counter()
    eng.train(n)
    eng.synchronize()
    us = (time.perf_counter() - t0) / n * 1e6
    print(f"fused layer split (2 stages, one GPU): {us:.2f} us/step")
    assert us < 40.0, us
    eng.close()


def _dp_rank(rank, world, steps):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng, _ = _engine(2, OptimConfig(lr=1e-2), batch=128, world=world, rank=rank)
    eng.train(steps)
    eng.synchronize()
    out = eng.flat_params_cpu(), eng.losses(0, steps)
    eng.close()
    return out


def test_fused_split_with_data_parallel_two_ranks():
    """Hybrid: 2 stages x 2 DP ranks, all four stage kernels on the one GPU; each
    stage's gradient is reduced over the ranks inside its kernel."""
    steps = 9
    res = run_ranks(_dp_rank, 2, (steps,), timeout=300)
    rp, rl = _reference(OptimConfig(lr=1e-2), steps, batch=128, world=2)
    for r in range(2):
        torch.testing.assert_close(res[r][1], rl, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(res[r][0], rp, rtol=1e-4, atol=2e-5)
    assert torch.equal(res[0][0], res[1][0]), "replicas diverged"


@pytest.mark.parametrize("K", [2, 3])
def test_fused_split_per_stage_launches(K):
    """The launch path of a node with one GPU per stage: every stage its own persistent
    launch on its own stream (here: streams of distinct priority levels on the one GPU,
    so no two stages share an in-order hardware queue).  Same numbers as the unsplit
    reference, no link timeout."""
    from distributed_training_pytorch_amd import _native as nat

    if K > len(nat.stream_priority_levels(DEV)):
        with pytest.raises(ValueError, match="priority levels"):
            _engine(K, OptimConfig(lr=1e-2), launch="per_stage")
        return
    ocfg = OptimConfig(lr=1e-2)
    steps = 12
    eng, _ = _engine(K, ocfg, launch="per_stage", timeout_us=500_000)
    assert len(eng._launch) == K and eng.launch_mode == "per_stage"
    eng.train(5)
    eng.train(steps - 5)
    eng.synchronize()  # raises on a link / exchange timeout
    rp, rl = _reference(ocfg, steps)
    torch.testing.assert_close(eng.losses(0, steps), rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(eng.flat_params_cpu(), rp, rtol=1e-4, atol=2e-5)
    eng.close()


# ---- split-batch stages (csrc/split_lanes.hip): M member workgroups per stage, member k of
# every stage one micro-batch of batch / M samples on its own links, the members' gradients
# summed on chip before each stage's optimizer step


@pytest.mark.parametrize("K,bounds", [(2, None), (3, None), (2, [(0, 2), (3, 4)]), (5, None), (1, None)])
@pytest.mark.parametrize("ocfg", [OptimConfig(lr=1e-2), OptimConfig("sgd", 5e-2, momentum=0.9)],
                         ids=["adam", "sgd"])
def test_split_members_match_unsplit_reference(K, bounds, ocfg):
    steps = 12
    eng, _ = _engine(K, ocfg, bounds, members="auto")
    assert eng.members == 4  # batch 256: four 64-sample micro-batches per stage
    eng.train(5)
    eng.train(steps - 5)  # two launches: state, link epochs and member exchange epochs carry over
    eng.synchronize()
    rp, rl = _reference(ocfg, steps)
    torch.testing.assert_close(eng.losses(0, steps), rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(eng.flat_params_cpu(), rp, rtol=1e-4, atol=2e-5)
    assert [int(s.item()) for s in eng.step] == [steps] * K
    eng.close()


@pytest.mark.parametrize("batch,members", [(100, "auto"), (200, "auto"), (256, 8), (64, "auto"), (50, 2)])
def test_split_members_slices_and_short_batches(batch, members):
    """Member slices of batch / M samples, including the epoch's short last batch (512 =
    5 x 100 + 12, 2 x 200 + 112: some members have no sample), 8 members of 32 samples and
    one member."""
    ocfg = OptimConfig(lr=1e-2)
    steps = 14
    eng, _ = _engine(2, ocfg, batch=batch, members=members)
    assert eng.members == (-(-batch // 64) if members == "auto" else members)
    eng.train(steps)
    eng.synchronize()
    rp, rl = _reference(ocfg, steps, batch=batch)
    torch.testing.assert_close(eng.losses(0, steps), rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(eng.flat_params_cpu(), rp, rtol=1e-4, atol=2e-5)
    eng.close()


def test_split_members_per_stage_launches():
    """One launch per stage (the multi-GPU launch path), members co-resident across the
    two launches through distinct stream priorities."""
    from distributed_training_pytorch_amd import _native as nat

    if len(nat.stream_priority_levels(DEV)) < 2:
        pytest.skip("one stream priority level")
    ocfg = OptimConfig(lr=1e-2)
    steps = 12
    eng, _ = _engine(2, ocfg, launch="per_stage", timeout_us=500_000, members="auto")
    eng.train(steps)
    eng.synchronize()
    rp, rl = _reference(ocfg, steps)
    torch.testing.assert_close(eng.losses(0, steps), rl, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(eng.flat_params_cpu(), rp, rtol=1e-4, atol=2e-5)
    eng.close()


def test_split_members_step_time():
    """The reference's 2-stage split at batch 256 on split-batch stages: well under the
    one-workgroup stages' ~10 us per iteration."""
    eng, _ = _engine(2, OptimConfig(lr=1e-3), members="auto")
    eng.train(50)
    eng.synchronize()
    n = 2000
    t0 = time.perf_counter()
    eng.train(n)
    eng.synchronize()
    us = (time.perf_counter() - t0) / n * 1e6
    print(f"fused layer split, split-batch stages (2 stages x 4 members, one GPU): {us:.2f} us/step")
    assert us < 8.0, us
    eng.close()


def _dp_members_rank(rank, world, steps):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng, _ = _engine(2, OptimConfig(lr=1e-2), batch=128, world=world, rank=rank, members="auto")
    assert eng.members == 2
    eng.train(steps)
    eng.synchronize()
    out = eng.flat_params_cpu(), eng.losses(0, steps)
    eng.close()
    return out


def test_split_members_with_data_parallel_two_ranks():
    """Hybrid: 2 stages x 2 members x 2 DP ranks; each stage's gradient in ONE cross-rank
    exchange over ranks x members (xgmi_allreduce_g3)."""
    steps = 9
    res = run_ranks(_dp_members_rank, 2, (steps,), timeout=300)
    rp, rl = _reference(OptimConfig(lr=1e-2), steps, batch=128, world=2)
    for r in range(2):
        torch.testing.assert_close(res[r][1], rl, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(res[r][0], rp, rtol=1e-4, atol=2e-5)
    assert torch.equal(res[0][0], res[1][0]), "replicas diverged"
