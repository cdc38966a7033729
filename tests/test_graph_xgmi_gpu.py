"""hipGraph capture of steps that all-reduce through the in-kernel xGMI exchange, and
the stand-alone xGMI all-reduce at full capacity: two ranks share the one GPU (the
exchange runs through IPC-mapped uncached buffers exactly as across xGMI)."""
import os
import sys

import pytest
import torch

from .dist_utils import run_ranks

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _module_steps(rank, world, graphs, steps):
    from distributed_training_pytorch_amd.engine.graph_step import CapturedStep
    from distributed_training_pytorch_amd.models.bank import ModelBank
    from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    bank = ModelBank(2).to(dev)
    # small buckets: several xGMI calls per backward (different sizes -> different
    # workgroup counts, each workgroup with its own device epoch counter)
    ddp = FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad, first_bucket_mb=0.0005,
                  bucket_cap_mb=0.001, comm="xgmi")
    opt = FlatOptimizer(bank.flat, bank.flat_grad, OptimConfig(lr=1e-2))
    g = torch.Generator().manual_seed(rank)
    xs = torch.randn(steps, 64, 2, generator=g).to(dev)
    ys = torch.randn(steps, 64, 1, generator=g).to(dev)
    x_st, y_st = xs[0].clone(), ys[0].clone()

    def body(_):
        bank.zero_grad()
        ox, oy = ddp(x_st)
        (torch.nn.functional.mse_loss(ox, y_st) + torch.nn.functional.mse_loss(oy, y_st)).backward()
        opt.step()

    stepper = CapturedStep(body, dev, enabled=graphs, on_abort=ddp.reset_hooks)
    for t in range(steps):
        x_st.copy_(xs[t])
        y_st.copy_(ys[t])
        stepper.run(0)
    torch.cuda.synchronize()
    ddp.check_comm()
    return bank.flat.cpu().clone(), ddp.comm, ddp.graph_safe(), stepper.replays, len(ddp._buckets), \
        stepper.fallback_reason


def test_module_step_graph_equals_eager_on_xgmi():
    steps = 8
    g = run_ranks(_module_steps, 2, (True, steps), timeout=300)
    e = run_ranks(_module_steps, 2, (False, steps), timeout=300)
    for r in range(2):
        p, comm, safe, replays, nb, why = g[r]
        assert comm == "xgmi" and safe and nb > 1
        assert replays >= steps - 2, (replays, why)  # warmup steps run eagerly, the rest replay
        assert torch.equal(p, e[r][0]), "graph replay differs from eager"
    assert torch.equal(g[0][0], g[1][0]), "replicas diverged"


def _trainer_rank(rank, world, graphs, root, engine="module", seed_per_rank=False):
    os.environ["LOCAL_RANK"] = "0"  # both ranks on the one GPU (the process group is already up)
    sys.path.insert(0, ROOT)
    from demo_pytorch_lightning import LitToyModel
    from distributed_training_pytorch_amd.data.toy_data import ToyData
    from distributed_training_pytorch_amd.trainer import Trainer

    torch.manual_seed(0)
    dl = torch.utils.data.DataLoader(ToyData(seed=0), batch_size=128)
    if seed_per_rank:  # the reference demo never seeds its models: every rank builds different weights
        torch.manual_seed(1000 + rank)
    model = LitToyModel()
    tr = Trainer(gpus=2, max_steps=12, accelerator="gpu", strategy="ddp", log_every_n_steps=4,
                 default_root_dir=os.path.join(root, f"g{int(graphs)}"), enable_progress_bar=False,
                 use_graphs=graphs, enable_checkpointing=False, engine=engine)
    tr.fit(model, dl)
    return {k: v.cpu() for k, v in model.state_dict().items()}, tr.graph_replays, \
        getattr(getattr(tr, "_stepper", None), "fallback_reason", None), tr.engine_used


def test_trainer_graph_equals_eager_on_xgmi(tmp_path):
    """The Lightning-style Trainer (two optimizers, DDP strategy) on two ranks replays
    each batch as a hipGraph over the xGMI buckets, bitwise equal to eager batches."""
    g = run_ranks(_trainer_rank, 2, (True, str(tmp_path)), timeout=300)
    e = run_ranks(_trainer_rank, 2, (False, str(tmp_path)), timeout=300)
    for r in range(2):
        sd, replays, why, _ = g[r]
        assert replays > 0, why
        for k in sd:
            assert torch.equal(sd[k], e[r][0][k]), k
    for k in g[0][0]:
        assert torch.equal(g[0][0][k], g[1][0][k]), k


def test_trainer_fused_engine_on_two_ranks(tmp_path):
    """Trainer(engine='auto') with DDP on two ranks runs LitToyModel on the fused
    train-step engine (in-kernel xGMI gradient exchange, DistributedSampler order) and
    ends where the per-batch module path ends, to fp32 summation-order tolerance, with
    identical replicas."""
    f = run_ranks(_trainer_rank, 2, (False, str(tmp_path / "f"), "auto"), timeout=300)
    e = run_ranks(_trainer_rank, 2, (False, str(tmp_path / "e"), "module"), timeout=300)
    for r in range(2):
        assert f[r][3] == "fused" and e[r][3] == "module", (f[r][3], e[r][3])
        for k, v in e[r][0].items():
            torch.testing.assert_close(f[r][0][k], v, rtol=0, atol=1e-4)
    for k in f[0][0]:
        assert torch.equal(f[0][0][k], f[1][0][k]), k


def test_trainer_fused_engine_ranks_built_from_different_seeds(tmp_path):
    """Ranks whose models start from different weights: the engine broadcasts rank 0's,
    the modules take them before fused_spec() is checked, so the check passes on every
    rank (it compared rank r's own weights with rank 0's before) and training ends where
    the module path ends."""
    f = run_ranks(_trainer_rank, 2, (False, str(tmp_path / "f"), "fused", True), timeout=300)
    e = run_ranks(_trainer_rank, 2, (False, str(tmp_path / "e"), "module", True), timeout=300)
    for r in range(2):
        assert f[r][3] == "fused" and e[r][3] == "module", (f[r][3], e[r][3])
        for k, v in e[r][0].items():
            torch.testing.assert_close(f[r][0][k], v, rtol=0, atol=1e-4)
    for k in f[0][0]:
        assert torch.equal(f[0][0][k], f[1][0][k]), k


def _full_cap_rank(rank, world, calls, graph_reps):
    from distributed_training_pytorch_amd.parallel.xgmi import XgmiAllReduce

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cap = XgmiAllReduce.MAX_CAP
    ar = XgmiAllReduce(cap, dev)
    outs = []
    for c, n in enumerate(calls):
        gen = torch.Generator().manual_seed(1000 * c + rank)
        t = torch.randn(n, generator=gen).to(dev)
        if rank == 1 and c % 3 == 1:
            torch.cuda._sleep(3_000_000)  # one rank arrives late: every block's spin must wait it out
        ar.all_reduce_(t)
        outs.append(t.cpu())
    # the same exchange captured once and replayed: each replay is a fresh exchange
    gen = torch.Generator().manual_seed(77 + rank)
    src = torch.randn(cap, generator=gen).to(dev)
    buf = torch.empty_like(src)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        buf.copy_(src)
        ar.all_reduce_(buf, scale=0.5)
    torch.cuda.current_stream().wait_stream(s)
    reps = []
    for k in range(graph_reps):
        src.mul_(2.0)  # new inputs per replay
        graph.replay()
        reps.append(buf.cpu().clone())
    torch.cuda.synchronize()
    ar.check()
    ar.close()
    return outs, reps


def test_xgmi_allreduce_full_capacity_uneven_and_graph_replays():
    """64 Ki floats = 64 workgroups, each polling its own granules with its own device
    epoch; call sizes vary (full, tiny, full), rank 1 is late on some calls, and the
    captured call is replayed with fresh inputs."""
    from distributed_training_pytorch_amd.parallel.xgmi import XgmiAllReduce

    cap = XgmiAllReduce.MAX_CAP
    calls = [cap, 100, cap, 5000, cap - 1, cap]
    reps = 3
    res = run_ranks(_full_cap_rank, 2, (calls, reps), timeout=300)
    for c, n in enumerate(calls):
        ref = sum(torch.randn(n, generator=torch.Generator().manual_seed(1000 * c + r)) for r in range(2))
        torch.testing.assert_close(res[0][0][c], ref, rtol=1e-6, atol=1e-6)
        assert torch.equal(res[0][0][c], res[1][0][c]), f"ranks disagree on call {c}"
    base = [torch.randn(cap, generator=torch.Generator().manual_seed(77 + r)) for r in range(2)]
    for k in range(reps):
        ref = (base[0] * 2 ** (k + 1) + base[1] * 2 ** (k + 1)) * 0.5
        torch.testing.assert_close(res[0][1][k], ref, rtol=1e-6, atol=1e-5)
        assert torch.equal(res[0][1][k], res[1][1][k])
