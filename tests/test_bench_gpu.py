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
    assert rec["config"]["parallelism"] == "dp1"


def test_bench_two_ranks_share_gpu():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--share-gpu",
           "--steps", "200", "--warmup", "20"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["comm"] == "xgmi", rec["config"]
    assert rec["config"]["global_batch"] == 512
    assert all(abs(v) < 10 for v in rec["final_loss"])
