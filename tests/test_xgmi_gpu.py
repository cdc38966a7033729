"""Multi-rank GPU paths on a single MI355X: two processes share cuda:0, so the
xGMI exchange runs through IPC-mapped uncached buffers (same-device mapping) and
the in-kernel granule protocol; results must equal the host all-reduce path and
the single-process reference.  Also the RCCL step path (1-rank NCCL group,
hipGraph-captured all-reduce)."""
import pytest
import torch

from distributed_training_pytorch_amd.data.sampler import SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC
from distributed_training_pytorch_amd.ops.optim import OptimConfig

from .dist_utils import run_ranks
from .test_dp_cpu import _init, _reference

pytestmark = pytest.mark.gpu
STEPS = 9


def _gpu_rank(rank, world, comm, steps, launch):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ds = ToyData(n=512, seed=1)
    X, Y = ds.device_tensors(dev)
    geom = SamplerGeometry(n=512, world=world, rank=rank, batch=128, seed=3)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, OptimConfig(lr=1e-2),
                      EngineConfig(comm=comm, launch=launch, steps_per_launch=4), init_params=_init(100 + rank))
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


def test_rccl_step_path_single_rank():
    res = run_ranks(_gpu_rank, 1, ("rccl", STEPS, "persistent"), timeout=300, backend="nccl")
    ref_p, ref_l = _reference(1, STEPS)
    p, l, used = res[0]
    assert used == "rccl"
    torch.testing.assert_close(p, ref_p, rtol=1e-4, atol=2e-5)
    torch.testing.assert_close(l, ref_l, rtol=1e-4, atol=1e-5)
