"""bf16 compute (BASELINE config 2): the bf16 instances of the fused kernels --
bf16 matmul operands (weights, activations, backward gradients), fp32 accumulation,
fp32 master weights, weight gradients and Adam.  Checked against (a) a PyTorch model
of exactly that rounding recipe (ops.mlp.mlp_forward_ref_bf16) and (b) the fp32
reference with bf16 tolerances."""
import json
import os
import subprocess
import sys

import pytest
import torch

from distributed_training_pytorch_amd.data.sampler import EpochIndexStream, SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC, fused_mlp, mlp_forward_ref_bf16, unflatten
from distributed_training_pytorch_amd.ops.optim import OptimConfig

from .ref_train import torch_train

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fused_mlp_bf16_matches_rounding_model():
    torch.manual_seed(0)
    flat = torch.randn(TOY_SPEC.P) * 0.5
    x = torch.randn(300, 2)
    go = torch.randn(300, 1)
    params = [p.clone().to(DEV).requires_grad_(True) for p in unflatten(flat, TOY_SPEC)]
    xd = x.to(DEV).requires_grad_(True)
    out = fused_mlp(xd, TOY_SPEC, params, bf16=True)
    out.backward(go.to(DEV))
    fr = flat.clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    ref = mlp_forward_ref_bf16(fr, TOY_SPEC, xr)
    ref.backward(go)
    # same rounding points; accumulation order may move a bf16 output by one ulp (2^-8)
    torch.testing.assert_close(out.detach().cpu(), ref.detach(), rtol=1e-2, atol=1e-2)
    g = torch.cat([p.grad.reshape(-1).cpu() for p in params])
    torch.testing.assert_close(g, fr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(xd.grad.cpu(), xr.grad, rtol=3e-2, atol=3e-2)
    # and it really is bf16 compute: the output values are bf16-representable
    assert torch.equal(out.detach().bfloat16().float(), out.detach())


def test_toy_model_under_autocast_runs_bf16_kernels():
    from distributed_training_pytorch_amd.models.toy import ToyModel

    torch.manual_seed(0)
    m = ToyModel().to(DEV)
    x = torch.randn(256, 2, device=DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    assert torch.equal(y.detach().bfloat16().float(), y.detach().float())
    y32 = m(x)
    assert not torch.equal(y.float(), y32) and torch.allclose(y.float(), y32, rtol=5e-2, atol=5e-2)


@pytest.mark.parametrize("launch", ["persistent", "graph", "eager"])
def test_fused_trainer_bf16_tracks_fp32_reference(launch):
    ds = ToyData(seed=3)
    X, Y = ds.device_tensors(DEV)
    geom = SamplerGeometry(n=512, batch=256, seed=11)
    g = torch.Generator().manual_seed(100)
    init = [torch.randn(TOY_SPEC.P, generator=g) * 0.4 for _ in range(2)]
    steps = 40
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, OptimConfig(lr=1e-2),
                      EngineConfig(launch=launch, steps_per_launch=8, precision="bf16"),
                      init_params=[p.to(DEV) for p in init])
    tr.train(steps)
    tr.synchronize()
    got = tr.losses(0, steps)
    _, ref = torch_train(TOY_SPEC, init, ds.X, ds.Y, [EpochIndexStream(geom)], steps, OptimConfig(lr=1e-2), "mse")
    rel = ((got - ref).abs() / ref.abs().clamp_min(1e-3)).max().item()
    assert rel < 5e-2, rel  # bf16 tolerance against the fp32 run
    assert not torch.equal(got, ref)  # and not silently the fp32 kernel
    tr.close()


def test_bench_bf16_json():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "200", "--warmup", "20", "--precision", "bf16"],
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert rec["dtype"] == "bf16" and rec["value"] > 1e6
    assert all(0.0 < v < 10.0 for v in rec["final_loss"])


def test_demo_bf16_end_to_end(tmp_path):
    r = subprocess.run([sys.executable, "demo.py", "--precision", "bf16", "--iters", "300", "--seed", "0",
                        "--no_progress", "--dry_run", "--log_dir", str(tmp_path)], cwd=ROOT, capture_output=True,
                       text=True, timeout=120, env=dict(os.environ, WANDB_MODE="disabled"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "engine: fused" in r.stdout, r.stdout[-2000:]
    line = [l for l in r.stdout.splitlines() if "summary:" in l][-1]
    s = eval(line.split("summary:", 1)[1])
    assert all(0.0 < v < 4.0 for v in s["final_loss"]), s


@pytest.mark.parametrize("engine", ["auto", "module"])
def test_trainer_precision_bf16(tmp_path, engine):
    r = subprocess.run([sys.executable, "demo_pytorch_lightning.py", "--gpus", "1", "--steps", "40", "--seed", "0",
                        "--no_progress", "--precision", "bf16", "--root_dir", str(tmp_path), "--engine", engine],
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "'global_step': 40" in r.stdout
    assert f"'engine': '{'fused' if engine == 'auto' else 'module'}'" in r.stdout, r.stdout[-1500:]


@pytest.mark.parametrize("batch,lanes,groups", [(64, 4, 1), (128, 4, 2), (256, 4, 4)])
def test_bf16_lanes_and_split_batch_steps_match_rounding_model(batch, lanes, groups):
    """The bf16 instances of the several-lanes step (per-rank batch <= 64) and of the
    split-batch step (4-lanes members, 64 samples each) against autograd through the bf16
    rounding model + torch.optim.Adam.  Accumulation order may move a bf16 value by an ulp
    (2^-8), hence the bf16 tolerances."""
    X, Y = ToyData(n=512, seed=4).device_tensors(DEV)
    geom = SamplerGeometry(n=512, batch=batch, seed=5)
    g = torch.Generator().manual_seed(9)
    init = [torch.randn(TOY_SPEC.P, generator=g) * 0.4 for _ in range(2)]
    ocfg = OptimConfig(lr=1e-2)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, geom, ocfg, EngineConfig(steps_per_launch=5, precision="bf16", groups="on"),
                      init_params=[p.to(DEV) for p in init])
    assert (tr.lanes, tr.groups) == (lanes, groups)
    steps = 10
    tr.train(steps)
    tr.synchronize()
    got_l, got_p = tr.losses(0, steps), tr.params.cpu()
    tr.close()
    ref_p, ref_l = torch_train(TOY_SPEC, init, X, Y, [EpochIndexStream(geom)], steps, ocfg, forward=mlp_forward_ref_bf16)
    torch.testing.assert_close(got_l, ref_l, rtol=2e-2, atol=1e-3)
    torch.testing.assert_close(got_p, ref_p, rtol=2e-2, atol=2e-3)
    fp_p, fp_l = torch_train(TOY_SPEC, init, X, Y, [EpochIndexStream(geom)], steps, ocfg)
    assert not torch.allclose(got_l, fp_l, rtol=1e-6, atol=0)  # bf16 compute for real, not the fp32 kernel
