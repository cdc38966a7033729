"""bench.py's launch contract on the CPU (gloo): ``--gpus N`` with no launcher around it
starts its own N ranks (torch.distributed.run on 127.0.0.1, the reference's
torchrun_launcher.sh:9-20 pattern), forwards rank 0's one JSON line, and fails when a
rank fails."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "DTP_BENCH_CHILD", "HSA_ENABLE_IPC_MODE_LEGACY")}
    env["HIP_VISIBLE_DEVICES"] = ""  # CPU ranks even on a GPU box
    env["CUDA_VISIBLE_DEVICES"] = ""
    env.update(kw)
    return env


def _run(args, **kw):
    return subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, capture_output=True, text=True,
                          timeout=240, env=_env(**kw))


def test_bench_self_launches_ranks():
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout  # exactly rank 0's JSON line on stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 512
    assert rec["value"] > 0 and len(rec["final_loss"]) == 2


def test_bench_self_launch_fails_with_a_rank():
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "1"], DTP_BENCH_FAIL_RANK="1")
    assert r.returncode != 0
    assert "forced failure" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_children_inherit_ipc_env():
    """The parent sets the collective environment before it launches the ranks: a rank
    finds HSA_ENABLE_IPC_MODE_LEGACY=0 at its own start, although the caller's
    environment (like the driver's) never set it.  HSA reads it once, at the first GPU
    touch, so a rank that set it itself later would be too late."""
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.strip()][0])
    assert rec["config"]["ipc_env_at_start"] == "0", rec["config"]
