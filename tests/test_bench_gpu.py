"""The bench.py contract on a GPU: the 1-rank JSON line, and the multi-rank path the
driver's 2/4/8-GPU scaling runs take (torch.distributed.run, one rank per process,
in-kernel xGMI exchange, max-over-ranks timing), rehearsed with every rank on the
one visible GPU (--share-gpu)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_line(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_one_gpu_json_contract():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "200", "--warmup", "20"], cwd=ROOT,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _json_line(r.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == 200 and rec["value"] > 1e6
    assert rec["config"]["parallelism"] == "dp1" and rec["scaling"] == "strong"
    assert rec["config"]["global_batch"] == 256 and rec["config"]["dataset_samples"] == 512


def _single_process_full_batch_losses(steps: int) -> list[float]:
    """The strong-scaling reference: at W >= 2 the 512-sample set is split over the W
    ranks with per-rank batch 512/W, so one step of the job sees every sample once --
    the same update as ONE process training on batch 512 (summation order aside)."""
    import torch

    sys.path.insert(0, ROOT)
    from distributed_training_pytorch_amd.data.sampler import SamplerGeometry
    from distributed_training_pytorch_amd.data.toy_data import ToyData
    from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
    from distributed_training_pytorch_amd.models.toy import ToyModel
    from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC
    from distributed_training_pytorch_amd.ops.optim import OptimConfig

    dev = torch.device("cuda", 0)
    X, Y = ToyData(n=512, seed=0).device_tensors(dev)
    torch.manual_seed(0)
    init = [ToyModel().flat_params.detach().clone() for _ in range(2)]
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=512, seed=0), OptimConfig(lr=1e-3),
                      EngineConfig(steps_per_launch=64), init_params=init)
    tr.train(steps)
    tr.synchronize()
    out = tr.losses(steps - 1, steps)[0].tolist()
    tr.close()
    return out


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_strong_scaling_share_gpu(world):
    """The driver's N-GPU bench config, rehearsed with W ranks on the one GPU: the
    reference's strong-scaling workload (512 samples total, per-rank batch 512/W),
    in-kernel xGMI exchange, and the final global loss of the job equal to one
    process training the full 512-sample batch."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    steps, warmup = 60, 20
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(world),
           "--share-gpu", "--steps", str(steps), "--warmup", str(warmup)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["scaling"] == "strong"
    assert rec["n_gpus"] == world and rec["config"]["parallelism"] == f"dp{world}"
    assert rec["config"]["comm"] == "xgmi", rec["config"]
    assert rec["config"]["dataset_samples"] == 512
    assert rec["config"]["global_batch"] == 512
    assert rec["config"]["per_rank_batch"] == 512 // world
    # per-rank batch 256 / 128 / 64: the 4-lanes step on 4 workgroups per model (the
    # split-batch members join the xGMI exchange as world x groups virtual members), the
    # 2-lanes step, the 4-lanes step
    assert (rec["config"]["lanes_per_sample"], rec["config"]["workgroups_per_model"]) == \
        {2: (4, 4), 4: (2, 1), 8: (4, 1)}[world], rec["config"]
    # the multi-GPU diagnostics of the line: no fallback, exchange wait and compute split
    assert rec["comm_fallback_reason"] is None
    assert len(rec["exchange_wait_us_per_step_by_rank"]) == world
    assert 0 <= rec["exchange_wait_us_per_step"] <= 1e3 * rec["ms_per_step"]
    assert rec["compute_us_per_step"] > 0
    # the step three ways: publish, wait, rest
    assert 0 <= rec["publish_us_per_step"] <= 1e3 * rec["ms_per_step"]
    assert abs(rec["publish_us_per_step"] + rec["exchange_wait_us_per_step"] + rec["step_rest_us_per_step"]
               - 1e3 * rec["ms_per_step"]) < 1e-6
    ref = _single_process_full_batch_losses(steps + warmup)
    for got, want in zip(rec["final_loss"], ref):
        assert abs(got - want) <= 1e-3 * abs(want) + 1e-5, (rec["final_loss"], ref)


def test_bench_self_launch_share_gpu():
    """No torchrun around bench.py: --gpus 2 starts its own two ranks (the driver's N-GPU
    call shape), here both on the one GPU -- from an environment WITHOUT
    HSA_ENABLE_IPC_MODE_LEGACY, as the driver may call it: bench.py must set it itself
    before any GPU touch, or the IPC mapping fails and the run falls back to RCCL."""
    drop = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE",
            "HSA_ENABLE_IPC_MODE_LEGACY", "DTP_BENCH_CHILD")
    env = {k: v for k, v in os.environ.items() if k not in drop}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--share-gpu", "--steps", "20", "--warmup", "5"],
                       cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["value"] > 0
    assert rec["config"]["comm"] == "xgmi", (rec["config"], rec.get("comm_fallback_reason"))
    assert rec["comm_fallback_reason"] is None
    assert rec["config"]["ipc_env_at_start"] == "0"


def test_bench_weak_scaling_flag_share_gpu():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--share-gpu",
           "--scaling", "weak", "--steps", "100", "--warmup", "10"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["scaling"] == "weak" and rec["config"]["global_batch"] == 512
    assert rec["config"]["per_rank_batch"] == 256 and rec["config"]["dataset_samples"] == 1024


def test_bench_cu_mask_keeps_split_batch_resident():
    """--cu-mask on pins the step to 2 CUs: the split-batch step (8 x 4 co-resident
    workgroups spinning on each other) cannot run there, so the engine refuses it and
    runs the one-workgroup-per-model step instead of timing out."""
    r = subprocess.run([sys.executable, "bench.py", "--cu-mask", "on", "--steps", "50", "--warmup", "5"],
                       cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _json_line(r.stdout)
    assert rec["config"]["cu_mask"] == "on" and rec["config"]["workgroups_per_model"] == 1, rec["config"]
    assert "groups_refused" in rec["config"]
