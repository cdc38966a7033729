"""Numerics of the HIP kernels against plain PyTorch fp32 references (GPU only)."""
import ctypes

import pytest
import torch

from distributed_training_pytorch_amd import _native as nat
from distributed_training_pytorch_amd.data.sampler import EpochIndexStream, SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC, MlpSpec, mlp_forward_ref, stage_backward, stage_forward
from distributed_training_pytorch_amd.ops.optim import OptimConfig, adam_update_ref, flat_optimizer_step

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _params(spec, seed=0, scale=0.5):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(spec.P, generator=g) * scale).to(DEV)


def test_native_library_loads():
    lib = nat.require(DEV)
    assert lib.dtp_version() == 1
    assert TOY_SPEC.native_supported()


@pytest.mark.parametrize("B", [1, 7, 64, 200, 256, 1000, 3000])
def test_stage_forward_backward_full_model(B):
    spec = TOY_SPEC
    flat = _params(spec, B)
    x = torch.randn(B, spec.in_features, device=DEV)
    out, saved = stage_forward(x, flat, spec)
    fr = flat.clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    ref = mlp_forward_ref(fr, spec, xr)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    go = torch.randn_like(ref)
    ref.backward(go)
    gin, gp = stage_backward(x, flat, spec, out, saved, go)
    torch.testing.assert_close(gin, xr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gp, fr.grad, rtol=1e-4, atol=1e-4 * max(1.0, B / 256))


@pytest.mark.parametrize("a,b", [(0, 1), (2, 4), (0, 3), (1, 4), (2, 2), (4, 4), (0, 0)])
def test_stage_substages(a, b):
    spec = TOY_SPEC.substage(a, b)
    flat = _params(spec, a * 10 + b)
    B = 129
    x = torch.randn(B, spec.in_features, device=DEV)
    out, saved = stage_forward(x, flat, spec)
    fr = flat.clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    ref = mlp_forward_ref(fr, spec, xr)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    go = torch.randn_like(ref)
    ref.backward(go)
    gin, gp = stage_backward(x, flat, spec, out, saved, go)
    torch.testing.assert_close(gin, xr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gp, fr.grad, rtol=1e-4, atol=1e-4)


def test_batch_indexer_device_matches_host():
    from distributed_training_pytorch_amd.data.sampler import BatchIndexer

    for n, W, r, B in [(512, 1, 0, 256), (1000, 3, 2, 100)]:
        g = SamplerGeometry(n=n, world=W, rank=r, batch=B, seed=77)
        ix = BatchIndexer(g, DEV, block=5)  # block refills inside and across epochs
        assert ix._native is not None  # the native sampler kernel, not a host fallback
        for t in range(3 * g.steps_per_epoch + 4):
            assert ix(t).cpu().tolist() == g.indices(t), (n, W, r, t)


def test_batch_indexer_exact_order_from_the_device_ring():
    """The exact DistributedSampler order (module engine, split module path) gathered on
    the device from the permutation ring equals torch's order, across epochs and with
    the padded last positions of an uneven split."""
    from distributed_training_pytorch_amd.data.sampler import BatchIndexer, EpochIndexStream

    for n, W, r, B in [(512, 1, 0, 256), (1000, 3, 2, 100), (37, 4, 3, 5)]:
        g = SamplerGeometry(n=n, world=W, rank=r, batch=B, seed=5)
        ix = BatchIndexer(g, DEV, exact_torch=True)
        assert ix._ring is not None
        stream = EpochIndexStream(g)
        for t in range(3 * g.steps_per_epoch + 2):
            assert ix(t).cpu().tolist() == stream.indices(t), (n, W, r, t)


def test_sampler_device_matches_python():
    lib = nat.require(DEV)
    for n, W, r, B in [(512, 1, 0, 256), (512, 8, 3, 256), (1000, 3, 2, 100), (4096, 8, 7, 256)]:
        g = SamplerGeometry(n=n, world=W, rank=r, batch=B, seed=1234)
        T = 2 * g.steps_per_epoch + 1
        out = torch.full((T, B), -7, dtype=torch.int32, device=DEV)
        cfg = g.to_native()
        nat.check(lib.dtp_sampler_indices(ctypes.byref(cfg), 0, T, nat.ptr(out), nat.stream_ptr()), "probe")
        got = out.cpu()
        for t in range(T):
            ref = g.indices(t)
            assert got[t, :len(ref)].tolist() == ref
            assert (got[t, len(ref):] == -1).all()
        # epoch 0 is a permutation of this rank's share
        ep = sorted(sum((g.indices(t) for t in range(g.steps_per_epoch)), []))
        assert len(ep) == g.num_samples


def _ref_train(spec, params, X, Y, geom, steps, cfg: OptimConfig):
    params = params.clone()
    nm, P = params.shape
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    losses = []
    for t in range(steps):
        idx = torch.tensor(geom.indices(t), device=X.device)
        x, y = X[idx], Y[idx]
        row = []
        for i in range(nm):
            p = params[i].clone().requires_grad_(True)
            loss = torch.nn.functional.mse_loss(mlp_forward_ref(p, spec, x), y)
            (g,) = torch.autograd.grad(loss, p)
            with torch.no_grad():
                if cfg.name == "adam":
                    adam_update_ref(params[i], m[i], v[i], g, t + 1, cfg)
                else:
                    params[i].add_(g, alpha=-cfg.lr)
            row.append(loss.item())
        losses.append(row)
    return params, torch.tensor(losses)


@pytest.mark.parametrize("launch", ["persistent", "graph", "eager"])
def test_fused_trainer_matches_reference(launch):
    ds = ToyData(seed=3)
    X, Y = ds.device_tensors(DEV)
    geom = SamplerGeometry(n=512, batch=256, seed=11)
    init = [_params(TOY_SPEC, 100 + i, 0.4) for i in range(2)]
    cfg = OptimConfig(lr=1e-2)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, cfg,
                      EngineConfig(launch=launch, steps_per_launch=4), init_params=init)
    steps = 14  # graph: three 4-step graphs, then a 2-step tail of one-step launches
    tr.train(steps)
    tr.synchronize()
    ref_p, ref_l = _ref_train(TOY_SPEC, torch.stack(init), X, Y, EpochIndexStream(geom), steps, cfg)
    torch.testing.assert_close(tr.losses(0, steps), ref_l, rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(tr.params, ref_p, rtol=1e-3, atol=2e-5)
    assert tr.step_ctr.tolist() == [steps, steps]
    tr.close()


@pytest.mark.parametrize("n,cache", [(4096, True), (4096, False), (8192, True)])
def test_fused_trainer_large_dataset(n, cache):
    """The 8-GPU weak-scaling dataset (n = 4096) stays in LDS; beyond it the kernel
    gathers from global memory -- same numbers either way."""
    ds = ToyData(n=n, seed=4)
    X, Y = ds.device_tensors(DEV)
    geom = SamplerGeometry(n=n, batch=256, seed=2)
    init = [_params(TOY_SPEC, 30 + i, 0.4) for i in range(2)]
    cfg = OptimConfig(lr=1e-2)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, cfg, EngineConfig(steps_per_launch=5, cache_data=cache),
                      init_params=init)
    steps = 10
    tr.train(steps)
    tr.synchronize()
    ref_p, ref_l = _ref_train(TOY_SPEC, torch.stack(init), X, Y, EpochIndexStream(geom), steps, cfg)
    torch.testing.assert_close(tr.losses(0, steps), ref_l, rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(tr.params, ref_p, rtol=1e-3, atol=2e-5)
    tr.close()


_FAST_SCRIPT = r"""
import sys, torch
sys.path.insert(0, {root!r})
from distributed_training_pytorch_amd.data.sampler import EpochIndexStream, SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC
from distributed_training_pytorch_amd.ops.optim import OptimConfig
dev = torch.device("cuda", 0)
X, Y = ToyData(n={n}, seed=8).device_tensors(dev)
g = torch.Generator().manual_seed(0)
init = [(torch.randn(TOY_SPEC.P, generator=g) * 0.4).to(dev) for _ in range(2)]
tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n={n}, batch=256, seed=4), OptimConfig(lr=1e-2),
                  EngineConfig(steps_per_launch=7, groups="off"), init_params=init)  # the one-lane instances
tr.train(19)
tr.synchronize()
torch.save({{"p": tr.params.cpu(), "l": tr.losses(0, 19)}}, {out!r})
"""


@pytest.mark.parametrize("n", [512, 500])
def test_fast_instance_bitwise_equals_generic(n, tmp_path):
    """The FAST kernel instance (power-of-two cached dataset, shuffle sampler) and the
    generic one (DTP_FAST=0) give bitwise-identical weights and losses; n = 500 has no
    FAST instance (cycle-walking sampler) and must match itself either way."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for flag in ("1", "0"):
        out = str(tmp_path / f"fast{flag}.pt")
        env = dict(os.environ, DTP_FAST=flag)
        r = subprocess.run([sys.executable, "-c", _FAST_SCRIPT.format(root=root, n=n, out=out)], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[flag] = torch.load(out, weights_only=True)
    assert torch.equal(outs["1"]["p"], outs["0"]["p"])
    assert torch.equal(outs["1"]["l"], outs["0"]["l"])


def test_adam_table_refill_inside_one_launch():
    """A persistent launch longer than the kernel's Adam-scalar table (1024 steps)
    refills it at a step boundary: bitwise equal to short launches."""
    X, Y = ToyData(seed=6).device_tensors(DEV)
    init = [_params(TOY_SPEC, 50 + i, 0.4) for i in range(2)]
    res = []
    for spl in (1100, 100):
        tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=256, seed=1), OptimConfig(lr=1e-3),
                          EngineConfig(steps_per_launch=spl), init_params=init)
        tr.train(1100)
        tr.synchronize()
        res.append((tr.params.clone(), tr.losses(0, 1100)))
        tr.close()
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


def test_fused_trainer_torch_sampler_order():
    ds = ToyData(seed=3)
    X, Y = ds.device_tensors(DEV)
    geom = SamplerGeometry(n=512, batch=256, seed=5)
    init = [_params(TOY_SPEC, 7 + i, 0.4) for i in range(2)]
    cfg = OptimConfig(lr=1e-3)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, cfg, EngineConfig(sampler="torch", steps_per_launch=3),
                      init_params=init)
    tr.train(6)
    tr.synchronize()
    # reference with the torch DistributedSampler order
    from distributed_training_pytorch_amd.data.sampler import EpochIndexStream

    es = EpochIndexStream(geom)

    class G:
        def indices(self, t):
            return es.indices(t)

    ref_p, ref_l = _ref_train(TOY_SPEC, torch.stack(init), X, Y, G(), 6, cfg)
    torch.testing.assert_close(tr.params, ref_p, rtol=1e-3, atol=2e-5)


@pytest.mark.parametrize("n,P,shadow", [(2, 371, False), (4, 371, False), (4, 370, False), (3, 3, False),
                                         (4, 20001, False), (3, 20002, False), (2, 20000, True), (2, 371, True),
                                         (3, 20001, True)])
def test_flat_optimizer_matches_torch_adam(n, P, shadow):
    """Every row phase of the float4 body (P % 4 = 0..3 over n rows: head peels of 0-3
    elements), rows shorter than a head (P = 3), the multi-block launch (P > 4096), and
    the bf16 shadow write (float4 path when P % 4 == 0, bf16-pair path otherwise)."""
    p0 = torch.randn(n, P, device=DEV)
    ps = [torch.nn.Parameter(p0[i].clone()) for i in range(n)]
    opt = torch.optim.Adam(ps, lr=1e-3)
    params = p0.clone()
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    step = torch.zeros(n, dtype=torch.int32, device=DEV)
    sh = torch.full((n, -(-P // 256) * 256), float("nan"), dtype=torch.bfloat16, device=DEV) if shadow else None
    for t in range(5):
        g = torch.randn(n, P, device=DEV)
        for i in range(n):
            ps[i].grad = g[i].clone()
        opt.step()
        buf = torch.cat([g.reshape(-1), torch.zeros(n, device=DEV)])
        flat_optimizer_step(params, m, v, step, buf, OptimConfig(), shadow=sh)
        if shadow:
            assert torch.equal(sh[:, :P], params.to(torch.bfloat16))
            assert torch.isnan(sh[:, P:].float()).all()  # the row padding is never written
    torch.testing.assert_close(params, torch.stack([p.detach() for p in ps]), rtol=1e-5, atol=1e-6)
    assert step.tolist() == [5] * n


def test_toy_model_autograd_path_matches_cpu():
    from distributed_training_pytorch_amd.models.toy import ToyModel

    torch.manual_seed(0)
    m_cpu = ToyModel()
    m_gpu = ToyModel()
    m_gpu.load_state_dict(m_cpu.state_dict())
    m_gpu = m_gpu.to(DEV)
    x = torch.randn(256, 2)
    y = torch.randn(256, 1)
    l_cpu = torch.nn.functional.mse_loss(m_cpu(x), y)
    l_cpu.backward()
    l_gpu = torch.nn.functional.mse_loss(m_gpu(x.to(DEV)), y.to(DEV))
    l_gpu.backward()
    torch.testing.assert_close(l_gpu.cpu(), l_cpu, rtol=1e-5, atol=1e-6)
    for pc, pg in zip(m_cpu.parameters(), m_gpu.parameters()):
        torch.testing.assert_close(pg.grad.cpu(), pc.grad, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("B", [256, 3000])  # one block (plain add) and the multi-block atomic path
def test_model_bank_grads_accumulate_in_place(B):
    """ModelBank's .grad views are fused-grad targets: the stage backward adds straight
    into the flat gradient buffer (no AccumulateGrad adds), and a second backward
    accumulates like autograd would."""
    from distributed_training_pytorch_amd.models.bank import ModelBank

    torch.manual_seed(1)
    bank = ModelBank(2)
    ref = [p.detach().clone().requires_grad_(True) for p in bank.flat]  # fp32 CPU reference params
    bank = bank.to(DEV)
    x = torch.randn(B, 2)
    y = torch.randn(B, 1)
    grad_buf = bank.flat_grad
    for _ in range(2):
        outs = bank(x.to(DEV))
        sum(torch.nn.functional.mse_loss(o, y.to(DEV)) for o in outs).backward()
        lr = sum(torch.nn.functional.mse_loss(mlp_forward_ref(r, TOY_SPEC, x), y) for r in ref)
        lr.backward()
    assert bank.flat_grad.data_ptr() == grad_buf.data_ptr()  # still the same buffer, written in place
    for i in range(2):
        torch.testing.assert_close(bank.flat_grad[i].cpu(), ref[i].grad, rtol=1e-4, atol=1e-5)
