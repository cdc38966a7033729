"""FlatDDP vs torch DDP, ModelBank packing, and the Lightning-style Trainer (CPU, gloo, 2 ranks)."""
import os
import subprocess
import sys
from pathlib import Path

import torch

from distributed_training_pytorch_amd.models.bank import ModelBank
from distributed_training_pytorch_amd.runtime import bootstrap

from .dist_utils import run_ranks

ROOT = Path(__file__).resolve().parents[1]


def _flatddp_vs_ddp(rank, world):
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP

    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    torch.manual_seed(100 + rank)  # different local init: the broadcast must equalise
    bank = ModelBank(2)
    ddp = FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad, first_bucket_mb=0.0005,
                  bucket_cap_mb=0.001)  # several buckets
    torch.manual_seed(100 + rank)
    ref = [torch.nn.Sequential(*[m for m in ModelBank(2)[i].layers]) for i in range(2)]
    # same start point as the broadcast bank (rank 0's init)
    for i in range(2):
        for p, q in zip(ref[i].parameters(), bank[i].parameters()):
            p.data.copy_(q.data)
    refd = [DDP(r) for r in ref]
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(64, 2, generator=g)
    y = torch.randn(64, 1, generator=g)
    bank.zero_grad()
    ox, oy = ddp(x)
    (torch.nn.functional.mse_loss(ox, y) + torch.nn.functional.mse_loss(oy, y)).backward()
    for r in refd:
        torch.nn.functional.mse_loss(r(x), y).backward()
    gref = torch.cat([p.grad.reshape(-1) for r in ref for p in r.parameters()])
    return bank.flat_grad.reshape(-1).clone(), gref, len(ddp._buckets)


def test_flatddp_matches_torch_ddp():
    res = run_ranks(_flatddp_vs_ddp, 2)
    for r in range(2):
        g, gref, nb = res[r]
        assert nb > 1
        torch.testing.assert_close(g, gref, rtol=1e-5, atol=1e-7)
    assert torch.equal(res[0][0], res[1][0])


def test_model_bank_views_and_state_dict():
    torch.manual_seed(0)
    bank = ModelBank(2)
    assert bank.flat.shape == (2, 371)
    w = bank[1].layers[2].weight
    w.data.fill_(3.0)
    assert (bank.flat[1, 30:130] == 3.0).all()
    keys = set(bank[0].state_dict().keys())
    assert keys == {f"layers.{i}.{k}" for i in (0, 2, 4, 6, 8) for k in ("weight", "bias")}


def test_lightning_style_trainer_two_ranks(tmp_path):
    env = dict(os.environ, PYTHONPATH=str(ROOT), PL_TORCH_DISTRIBUTED_BACKEND="gloo", OMP_NUM_THREADS="1")
    env.pop("RANK", None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(bootstrap.free_port()),
                        "demo_pytorch_lightning.py", "--steps", "12", "--accelerator", "cpu", "--root_dir",
                        str(tmp_path), "--no_progress", "--gpus", "2"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "'global_step': 12" in r.stdout
    ck = list((tmp_path / "lightning_logs" / "version_0" / "checkpoints").glob("*.ckpt"))
    assert len(ck) == 1 and "step=12" in ck[0].name
    sd = torch.load(ck[0], weights_only=True)
    assert "model_X.layers.0.weight" in sd["state_dict"]


def _flatddp_bucket_views(rank, world):
    """Every bucket must reduce exactly its own slice of the flat grad (regression:
    a 2-D flat buffer sliced by rows reduced the whole buffer in one bucket)."""
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    torch.manual_seed(0)
    bank = ModelBank(2)
    ddp = FlatDDP(bank, flat_params=bank.flat, flat_grad=bank.flat_grad, first_bucket_mb=0.0005,
                  bucket_cap_mb=0.001)
    sizes = [ddp._grad1d[lo:hi].numel() for lo, hi in ddp._spans]
    return sizes, sum(hi - lo for lo, hi in ddp._spans)


def test_flatddp_bucket_views_cover_the_buffer():
    res = run_ranks(_flatddp_bucket_views, 2)
    sizes, total = res[0]
    assert len(sizes) > 2 and all(s > 0 for s in sizes) and sum(sizes) == total == 742


def _flatddp_wide(rank, world):
    from torch.nn.parallel import DistributedDataParallel as DDP

    from distributed_training_pytorch_amd.models.wide import WideMLP
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    torch.manual_seed(0)
    m = WideMLP((2, 24, 24, 1))
    ref = WideMLP((2, 24, 24, 1))
    ref.load_state_dict(m.state_dict())
    ddp = FlatDDP(m, first_bucket_mb=0.0005, bucket_cap_mb=0.001)
    refd = DDP(ref.layers)
    g = torch.Generator().manual_seed(rank)
    x, y = torch.randn(32, 2, generator=g), torch.randn(32, 1, generator=g)
    ddp.zero_grad()
    torch.nn.functional.mse_loss(ddp(x), y).backward()  # GEMM backward: grads accumulated in place
    torch.nn.functional.mse_loss(refd(x), y).backward()
    return ddp.flat_grad.clone(), torch.cat([p.grad.reshape(-1) for p in ref.parameters()]), len(ddp._buckets)


def test_flatddp_in_place_gemm_grads_match_torch_ddp():
    res = run_ranks(_flatddp_wide, 2)
    for r in range(2):
        g, gref, nb = res[r]
        assert nb > 1
        torch.testing.assert_close(g, gref, rtol=1e-5, atol=1e-6)
    assert torch.equal(res[0][0], res[1][0])


def _flatddp_auto_buckets(rank, world):
    from distributed_training_pytorch_amd.models.wide import WideMLP
    from distributed_training_pytorch_amd.parallel import bucket_tuning
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    # small probes on the CPU ranks (the node's defaults go to 64 MB)
    bucket_tuning.DEFAULT_SIZES = (16 << 10, 64 << 10, 256 << 10, 1 << 20)
    torch.manual_seed(0)
    m = WideMLP((2, 256, 256, 256, 1))  # ~133 K parameters: larger than the smallest probe
    ddp = FlatDDP(m)
    plan = ddp.bucket_plan
    toy = FlatDDP(ModelBank(2))  # 3 KB of gradients: nothing to choose, no measurement
    g = torch.Generator().manual_seed(rank)
    x, y = torch.randn(16, 2, generator=g), torch.randn(16, 1, generator=g)
    ddp.zero_grad()
    torch.nn.functional.mse_loss(ddp(x), y).backward()
    return plan, toy.bucket_plan, len(ddp._buckets), ddp.flat_grad.clone()


def test_flatddp_auto_buckets_measured_on_the_group():
    """bucket_cap_mb / first_bucket_mb = "auto": every rank measures the group's all-reduce
    at a few sizes, fits t = alpha + n / beta and takes the same plan (the slowest rank's
    medians); a model that fits the smallest probe keeps torch's defaults unmeasured."""
    res = run_ranks(_flatddp_auto_buckets, 2)
    plan0, toy0, nb0, g0 = res[0]
    plan1, _, nb1, g1 = res[1]
    assert plan0["source"] == "measured" and plan0 == plan1 and nb0 == nb1
    assert plan0["alpha_us"] >= 0 and plan0["bandwidth_GBps"] > 0 and len(plan0["measured"]) == 4
    assert 1.0 <= plan0["bucket_cap_mb"] <= 256.0
    assert 64 / 1024 <= plan0["first_bucket_mb"] <= plan0["bucket_cap_mb"]
    assert toy0["source"] == "default" and toy0["bucket_cap_mb"] == 25.0
    assert torch.equal(g0, g1)  # the averaged gradient is the same on both ranks


def test_bucket_choice_from_a_latency_bandwidth_fit():
    from distributed_training_pytorch_amd.parallel import bucket_tuning

    alpha, beta = 20e-6, 50e9  # 20 us fixed, 50 GB/s
    meas = [(n, alpha + n / beta) for n in (1 << 20, 4 << 20, 16 << 20, 64 << 20)]
    a, b = bucket_tuning.fit_latency_bandwidth(meas)
    assert abs(a - alpha) < 1e-9 and abs(b - beta) / beta < 1e-6
    p = bucket_tuning.choose_buckets(meas)
    assert abs(p["bucket_cap_mb"] - 9 * alpha * beta / 2 ** 20) < 1e-3  # 8.6 MB: 10 % fixed cost
    assert abs(p["first_bucket_mb"] - alpha * beta / 2 ** 20) < 1e-3  # 0.95 MB: half bytes, half latency


def _lit_run(tmp_path, steps, ckpt_path=None, every=0, precision=32):
    sys.path.insert(0, str(ROOT))
    from demo_pytorch_lightning import LitToyModel
    from distributed_training_pytorch_amd.data.toy_data import ToyData
    from distributed_training_pytorch_amd.trainer import Trainer

    torch.manual_seed(0)
    ds = ToyData(seed=0)
    dl = torch.utils.data.DataLoader(ds, batch_size=128)
    model = LitToyModel()
    tr = Trainer(gpus=0, max_steps=steps, accelerator="cpu", log_every_n_steps=1, default_root_dir=str(tmp_path),
                 enable_progress_bar=False, every_n_train_steps=every, precision=precision)
    tr.fit(model, dl, ckpt_path=ckpt_path)
    return tr, model


def test_trainer_resume_is_bit_exact(tmp_path):
    """fit(ckpt_path="last") continues a run from its periodic last.ckpt (weights, both
    Adams, global_step, epoch and the position inside the epoch: 512 samples / batch
    128 = 4 batches per epoch, so step 6 is mid-epoch) and ends bitwise where an
    uninterrupted run ends."""
    ref_tr, ref = _lit_run(tmp_path / "ref", 10)
    a_tr, _ = _lit_run(tmp_path / "run", 6, every=3)
    assert (tmp_path / "run" / "lightning_logs" / "version_0" / "checkpoints" / "last.ckpt").exists()
    b_tr, b = _lit_run(tmp_path / "run", 10, ckpt_path="last")
    assert b_tr.resumed_from.endswith(".ckpt")
    assert b_tr.global_step == 10 == ref_tr.global_step
    assert b_tr.current_epoch == ref_tr.current_epoch
    for (k, v), (k2, v2) in zip(ref.state_dict().items(), b.state_dict().items()):
        assert k == k2 and torch.equal(v, v2), k


def test_post_accumulate_hooks_fire_for_none_grads_and_flatddp_counts_once():
    """torch runs post-accumulate-grad hooks even for a None gradient, so a fused-grad
    parameter (grad-ready hook + post-accumulate hook) notifies FlatDDP twice per
    backward; a bucket must still wait for every parameter (regression: buckets were
    released after half of them, before the last backward kernel ran)."""
    from distributed_training_pytorch_amd.ops.gemm import _grad_ready, mark_fused_grad
    from distributed_training_pytorch_amd.parallel.ddp import FlatDDP

    class F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            ctx.w = w
            return x * w

        @staticmethod
        def backward(ctx, g):
            _grad_ready(ctx.w)  # a fused kernel "wrote" w.grad in place
            return g, None

    ws = [torch.nn.Parameter(torch.ones(3)) for _ in range(2)]
    m = torch.nn.ParameterList(ws)
    ddp = FlatDDP(m)
    for w in ws:
        mark_fused_grad(w)
    reduced = []
    orig = ddp._reduce_bucket
    ddp._reduce_bucket = lambda b: (reduced.append((b, sum(len(ddp._ready) for _ in [0]))), orig(b))
    x = torch.ones(3, requires_grad=True)
    (F.apply(x, ws[0]).sum() + F.apply(x, ws[1]).sum()).backward()
    assert reduced and reduced[0][1] == 2, reduced  # released only once both parameters reported


def test_trainer_metric_rows_cover_every_logged_step(tmp_path):
    """Logged metrics are reduced and written in blocks (one sync per 64 logged
    steps), but metrics.csv still holds one row per logged step with that step's
    values, and callback_metrics is the last step's after fit."""
    import csv

    steps = 70
    tr, _ = _lit_run(tmp_path, steps)
    rows = list(csv.DictReader(open(tmp_path / "lightning_logs" / "version_0" / "metrics.csv")))
    assert [int(r["step"]) for r in rows] == list(range(1, steps + 1))
    keys = [k for k in rows[0] if k != "step"]
    assert keys and set(keys) == set(tr.callback_metrics)
    assert all(float(rows[-1][k]) == tr.callback_metrics[k] for k in keys)
    assert len({rows[i][keys[0]] for i in range(steps)}) > steps // 2  # per-step values, not one repeated


def test_csv_logger_block_rows_match_single_rows(tmp_path):
    """CSVLogger.log_rows (the fused engine's one call per launch) writes the same
    file as one log() per step: header order, step column, per-name values, sum."""
    from distributed_training_pytorch_amd.trainer.trainer import CSVLogger

    names = ["loss/lossX", "loss/lossY"]
    rows = [[0.5 + k, 0.25 * k] for k in range(5)]
    steps = [4, 8, 12, 16, 20]
    a = CSVLogger(str(tmp_path / "a"), 0)
    for s, r in zip(steps, rows):
        a.log(s, {**dict(zip(names, r)), "train_loss": sum(r)})
    a.close()
    b = CSVLogger(str(tmp_path / "b"), 0)
    b.log_rows(steps[:2], names, rows[:2])
    b.log_rows([], names, [])
    b.log_rows(steps[2:], names, rows[2:])
    b.close()
    assert (a.dir / "metrics.csv").read_text() == (b.dir / "metrics.csv").read_text()


def test_trainer_stops_at_the_first_of_max_steps_and_max_epochs(tmp_path):
    """max_epochs bounds the fit when it comes before max_steps (4 batches per epoch), and
    max_steps=0 runs no batch; the fused engine computes its step total by the same rule
    (trainer.py:_fit_fused)."""
    sys.path.insert(0, str(ROOT))
    from demo_pytorch_lightning import LitToyModel
    from distributed_training_pytorch_amd.data.toy_data import ToyData
    from distributed_training_pytorch_amd.trainer import Trainer

    for kw, want in [(dict(max_steps=100, max_epochs=2), 8), (dict(max_steps=3, max_epochs=2), 3),
                     (dict(max_steps=0), 0), (dict(max_steps=None, max_epochs=1), 4)]:
        torch.manual_seed(0)
        dl = torch.utils.data.DataLoader(ToyData(seed=0), batch_size=128)
        tr = Trainer(gpus=0, accelerator="cpu", log_every_n_steps=1, default_root_dir=str(tmp_path / str(want)),
                     enable_progress_bar=False, **kw)
        tr.fit(LitToyModel(), dl)
        assert tr.global_step == want, (kw, tr.global_step)
