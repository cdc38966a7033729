"""The several-lanes-per-sample fused step (csrc/mlp_lanes.h) against plain autograd +
torch.optim.Adam, its selection by the per-rank batch, and its self-consistency across
launch modes (GPU only)."""
import os
import subprocess
import sys

import pytest
import torch

from distributed_training_pytorch_amd.data.sampler import EpochIndexStream, SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC, MlpSpec
from distributed_training_pytorch_amd.ops.optim import OptimConfig

from .ref_train import torch_train

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _init(spec, seed, n=2, scale=0.4):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(spec.P, generator=g) * scale).to(DEV) for _ in range(n)]


@pytest.mark.parametrize("batch,lanes,groups", [(64, 4, 1), (50, 4, 1), (128, 4, 2), (100, 4, 2), (256, 4, 4),
                                                (200, 4, 4)])
def test_lanes_selected_by_batch_and_match_torch(batch, lanes, groups):
    """batch 50 / 100 / 200: the epoch's last batch is short (512 = 10 x 50 + 12,
    5 x 100 + 12, 2 x 200 + 112), so the lanes past it must drop out of the loss, the dW
    tiles and the mean; at 200 the last batch leaves split-batch members 2 and 3 without
    a sample.  Batches above 64 run the split-batch step: batch / 64 workgroups per model
    (csrc/grp_core.h)."""
    X, Y = ToyData(n=512, seed=21).device_tensors(DEV)
    geom = SamplerGeometry(n=512, batch=batch, seed=3)
    init = _init(TOY_SPEC, batch)
    ocfg = OptimConfig(lr=1e-2)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, ocfg, EngineConfig(steps_per_launch=7, groups="on"), init_params=init)
    assert (tr.lanes, tr.groups) == (lanes, groups)
    steps = 2 * geom.steps_per_epoch + 3
    tr.train(steps)
    tr.synchronize()
    ref_p, ref_l = torch_train(TOY_SPEC, init, X, Y, [EpochIndexStream(geom)], steps, ocfg)
    torch.testing.assert_close(tr.losses(0, steps), ref_l, rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(tr.params.cpu(), ref_p, rtol=1e-4, atol=2e-5)
    assert tr.step_ctr.tolist() == [steps, steps]
    tr.close()


@pytest.mark.parametrize("spec", [MlpSpec(2, 10, 3, 1), MlpSpec(2, 15, 5, 1), MlpSpec(2, 10, 5, 4)],
                         ids=["nl3", "h15", "out4"])
@pytest.mark.parametrize("batch", [64, 128])
def test_lanes_other_shapes_match_torch(spec, batch):
    """H = 15 leaves a padding slot in the last part (L = 4: 4 x 4 = 16 units; L = 2:
    2 x 8) that must never reach the tiles; OUT = 4 is a whole last layer of 4 rows."""
    X, Y = ToyData(n=512, seed=5).device_tensors(DEV)
    if spec.out_features > 1:
        Y = torch.randn(512, spec.out_features, device=DEV)
    geom = SamplerGeometry(n=512, batch=batch, seed=9)
    init = _init(spec, 7 + batch, scale=0.3)
    ocfg = OptimConfig(lr=5e-3)
    tr = FusedTrainer(spec, 2, X, Y, geom, ocfg, EngineConfig(steps_per_launch=5), init_params=init)
    assert tr.lanes == (4 if batch == 64 else 2) and tr.groups == 1  # split-batch step: the toy shape only
    steps = 12
    tr.train(steps)
    tr.synchronize()
    ref_p, ref_l = torch_train(spec, init, X, Y, [EpochIndexStream(geom)], steps, ocfg)
    torch.testing.assert_close(tr.losses(0, steps), ref_l, rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(tr.params.cpu(), ref_p, rtol=1e-4, atol=2e-5)
    tr.close()


@pytest.mark.parametrize("batch", [64, 128, 256])
def test_lanes_bitwise_across_launch_modes(batch):
    """The lanes instance is deterministic: one persistent launch, short persistent
    launches, per-step eager launches and hipGraph replays give bitwise the same run,
    including a launch longer than the kernel's Adam-scalar table (1024 steps).  At 128
    and 256 that is the split-batch step (2 / 4 workgroups per model): its on-chip sums
    run in member order, whatever order the members finish in."""
    X, Y = ToyData(n=512, seed=2).device_tensors(DEV)
    geom = SamplerGeometry(n=512, batch=batch, seed=1)
    init = _init(TOY_SPEC, 40)
    res = {}
    for name, ecfg, steps in [("long", EngineConfig(steps_per_launch=1100, groups="on"), 1100),
                              ("short", EngineConfig(steps_per_launch=100, groups="on"), 1100),
                              ("one", EngineConfig(steps_per_launch=1100, groups="on"), 30),
                              ("eager", EngineConfig(launch="eager", groups="on"), 30),
                              ("graph", EngineConfig(launch="graph", steps_per_launch=8, groups="on"), 30)]:
        tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, OptimConfig(lr=1e-3), ecfg, init_params=init)
        assert (tr.lanes, tr.groups) == (4, batch // 64)
        tr.train(steps)
        tr.synchronize()
        res[name] = (tr.params.clone(), tr.losses(0, steps))
        tr.close()
    assert torch.equal(res["long"][0], res["short"][0]) and torch.equal(res["long"][1], res["short"][1])
    for k in ("eager", "graph"):
        assert torch.equal(res["one"][0], res[k][0]), k
        assert torch.equal(res["one"][1], res[k][1]), k


_FORCE_SCRIPT = r"""
import sys, torch
sys.path.insert(0, {root!r})
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC
from distributed_training_pytorch_amd.ops.optim import OptimConfig
dev = torch.device("cuda", 0)
X, Y = ToyData(n=512, seed=8).device_tensors(dev)
g = torch.Generator().manual_seed(0)
init = [(torch.randn(TOY_SPEC.P, generator=g) * 0.4).to(dev) for _ in range(2)]
tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch={batch}, seed=4), OptimConfig(lr=1e-2),
                  EngineConfig(steps_per_launch=9, groups={groups!r}), init_params=init)
lanes = tr.lanes
tr.train(40)
tr.synchronize()
torch.save({{"p": tr.params.cpu(), "l": tr.losses(0, 40), "lanes": lanes}}, {out!r})
"""


def test_lanes_agree_with_one_lane_kernel(tmp_path):
    """DTP_LANES forces the instance: at batch 64 the L = 1, 2, 4 kernels run the same
    training (forward / input-gradient chains are the same fmaf sequence; the batch sums
    are grouped differently, so agreement is to float reassociation)."""
    outs = {}
    for flag in ("1", "2", "4"):
        out = str(tmp_path / f"l{flag}.pt")
        env = dict(os.environ, DTP_LANES=flag)
        r = subprocess.run([sys.executable, "-c", _FORCE_SCRIPT.format(root=ROOT, batch=64, out=out, groups="auto")], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[flag] = torch.load(out, weights_only=True)
        assert outs[flag]["lanes"] == int(flag)
    for flag in ("2", "4"):
        torch.testing.assert_close(outs[flag]["l"], outs["1"]["l"], rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(outs[flag]["p"], outs["1"]["p"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("batch", [256, 128])
def test_split_batch_step_agrees_with_single_workgroup(batch, tmp_path):
    """The split-batch step (groups="on") and the one-workgroup step (groups="off": the
    one-lane step at 256, the 2-lanes step at 128) run the same training to float
    reassociation; the default policy is the split-batch step at 256 (4 members), the
    2-lanes step at 128."""
    outs = {}
    for flag in ("off", "on", "auto"):
        out = str(tmp_path / f"g{flag}.pt")
        env = {k: v for k, v in os.environ.items() if k not in ("DTP_LANES", "DTP_GROUPS")}
        r = subprocess.run([sys.executable, "-c", _FORCE_SCRIPT.format(root=ROOT, batch=batch, out=out, groups=flag)],
                           env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[flag] = torch.load(out, weights_only=True)
    assert outs["off"]["lanes"] == (1 if batch == 256 else 2) and outs["on"]["lanes"] == 4
    assert torch.equal(outs["auto"]["p"], outs["on" if batch == 256 else "off"]["p"])
    torch.testing.assert_close(outs["on"]["l"], outs["off"]["l"], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(outs["on"]["p"], outs["off"]["p"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("batch", [256, 64])
def test_host_adam_table_bitwise_equals_kernel_fill(batch):
    """The persistent launch reads Adam's per-step scalars from the host-built table
    (ops/optim.py:adam_bias_table) with its prologue loads; without the table the kernel
    forms them itself in f64.  Same bits, across a table refill (1100 steps > 1024) and
    past the table's saturated end (t0 near 37k)."""
    X, Y = ToyData(n=512, seed=12).device_tensors(DEV)
    geom = SamplerGeometry(n=512, batch=batch, seed=6)
    init = _init(TOY_SPEC, 77)
    res = []
    for host in (True, False):
        tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, OptimConfig(lr=1e-3), EngineConfig(steps_per_launch=1100),
                          init_params=init)
        assert (tr._adam_tab is not None) and tr._adam_tab.shape[0] > 30000
        if not host:
            tr._adam_tab = None
        tr.train(1100)
        # jump the step counter near / past the table's end (37413 rows for the default betas)
        tr.t = 37400
        tr.step_ctr.fill_(37400)
        tr.train(40)
        tr.synchronize()
        res.append((tr.params.clone(), tr.losses(0, 1100), tr.losses(37400, 37440)))
        tr.close()
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


_W8_SCRIPT = r"""
import sys, torch
sys.path.insert(0, {root!r})
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC
from distributed_training_pytorch_amd.ops.optim import OptimConfig
dev = torch.device("cuda", 0)
X, Y = ToyData(n=512, seed=31).device_tensors(dev)
g = torch.Generator().manual_seed(3)
init = [(torch.randn(TOY_SPEC.P, generator=g) * 0.4).to(dev) for _ in range(2)]
tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch={batch}, seed=2), OptimConfig(lr=1e-2),
                  EngineConfig(steps_per_launch=6), init_params=init)
pick = (tr.lanes, tr.kernel_waves)
tr.train({steps})
tr.synchronize()
torch.save({{"p": tr.params.cpu(), "l": tr.losses(0, {steps}), "pick": pick, "init": [p.cpu() for p in init]}},
           {out!r})
"""


@pytest.mark.parametrize("force,batch", [("2x8", 256), ("2x8", 200), ("4x8", 128)])
def test_two_waves_per_simd_instances_match_torch(force, batch, tmp_path):
    """The 8-wave lanes step (two waves per SIMD, 512 / L samples per step; DTP_LANES=<L>x8)
    against autograd + torch.optim.Adam, including a short last batch (200)."""
    steps = 11
    out = str(tmp_path / "w8.pt")
    env = dict(os.environ, DTP_LANES=force)
    r = subprocess.run([sys.executable, "-c", _W8_SCRIPT.format(root=ROOT, batch=batch, steps=steps, out=out)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = torch.load(out, weights_only=True)
    assert res["pick"] == (int(force[0]), 8)
    X, Y = ToyData(n=512, seed=31).device_tensors(DEV)
    geom = SamplerGeometry(n=512, batch=batch, seed=2)
    ref_p, ref_l = torch_train(TOY_SPEC, res["init"], X, Y, [EpochIndexStream(geom)], steps, OptimConfig(lr=1e-2))
    torch.testing.assert_close(res["l"], ref_l, rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(res["p"], ref_p, rtol=1e-4, atol=2e-5)


def test_split_batch_dead_launch_keeps_the_state():
    """A launch whose member exchange timed out (sticky status word) sums incomplete
    gradients: it must write nothing back -- parameters, moments and step counters stay
    those before it -- and check_comm must raise."""
    import ctypes

    from distributed_training_pytorch_amd import _native as nat

    X, Y = ToyData(n=512, seed=21).device_tensors(DEV)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=256, seed=3), OptimConfig(lr=1e-2),
                      EngineConfig(groups="on"), init_params=_init(TOY_SPEC, 4))
    assert tr.groups == 4
    tr.train(5)
    tr.synchronize()
    before = [t.clone() for t in (tr.params, tr.m, tr.v, tr.step_ctr)]
    nat.check(nat.load().dtp_train_engine_poison(ctypes.c_void_p(tr._engine), 6), "poison")
    tr.train(3)
    torch.cuda.synchronize()
    for a, b in zip(before, (tr.params, tr.m, tr.v, tr.step_ctr)):
        assert torch.equal(a, b)
    with pytest.raises(RuntimeError, match="timed out"):
        tr.check_comm()
    tr.close()


@pytest.mark.parametrize("distributed", [True, False], ids=["dist_noshuffle", "sequential"])
def test_unshuffled_orders_take_the_fast_step_and_match_torch(distributed):
    """DistributedSampler(shuffle=False) and one rank reading the dataset in order (the
    Lightning demo at one GPU) go through an identity permutation table, so the fast step
    instances serve them (they read a SAMPLER_TABLE ring): the same order and results as
    autograd + torch.optim on those indices."""
    X, Y = ToyData(n=512, seed=21).device_tensors(DEV)
    geom = SamplerGeometry(n=512, batch=128, seed=3, shuffle=False, distributed=distributed)
    init = _init(TOY_SPEC, 77)
    ocfg = OptimConfig(lr=1e-2)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, ocfg, EngineConfig(steps_per_launch=7), init_params=init)
    assert tr._ring is not None and tr._ring.kind == "identity"
    assert tr.lanes > 1  # a several-lanes / split-batch instance, not the generic one-lane step
    steps = 3 * geom.steps_per_epoch + 1
    tr.train(steps)
    tr.synchronize()
    ref_p, ref_l = torch_train(TOY_SPEC, init, X, Y, [EpochIndexStream(geom)], steps, ocfg)
    torch.testing.assert_close(tr.losses(0, steps), ref_l, rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(tr.params.cpu(), ref_p, rtol=1e-4, atol=2e-5)
    tr.close()
