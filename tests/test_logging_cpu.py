"""MetricLogger.log_rows (one block per fused-engine launch) writes exactly the JSONL
lines that one log() per step writes, NaN / inf included."""
import json

from distributed_training_pytorch_amd.utils.logging import MetricLogger


def test_log_rows_matches_per_step_log(tmp_path):
    names = ["loss/lossX", "loss/lossY"]
    steps = [3, 4, 5]
    rows = [[0.5, 1e-7], [2.0, float("nan")], [float("inf"), -0.0]]
    a = MetricLogger(log_dir=str(tmp_path / "a"), use_wandb=False)
    a.log_rows(steps, names, rows)
    a.log_rows([], names, [])
    a.finish()
    b = MetricLogger(log_dir=str(tmp_path / "b"), use_wandb=False)
    for st, row in zip(steps, rows):
        b.log(dict(zip(names, row)), step=st)
    b.finish()

    def body(d):
        return [l for l in open(tmp_path / d / "metrics.jsonl") if '"event"' not in l]

    assert body("a") == body("b")
    assert [json.loads(l)["step"] for l in body("a")] == steps
    assert a.step == b.step == 6
