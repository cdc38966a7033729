"""MetricLogger.log_rows (one block per fused-engine launch) writes exactly the JSONL
lines that one log() per step writes, NaN / inf included."""
import json

import pytest

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


def _host_log_lib():
    import ctypes

    from distributed_training_pytorch_amd import _native as nat

    if not nat.LIB_PATH.exists():
        pytest.skip("libdtp.so not built")
    lib = ctypes.CDLL(str(nat.LIB_PATH))
    ll, vp = ctypes.c_longlong, ctypes.c_void_p
    lib.dtp_format_loss_rows.restype = ll
    lib.dtp_format_loss_rows.argtypes = [vp, ctypes.c_int, ll, ll, ll, ll, ll, ctypes.c_int, vp, ll]
    lib.dtp_format_loss_rows_jsonl.restype = ll
    lib.dtp_format_loss_rows_jsonl.argtypes = [vp, ctypes.c_int, ll, ll, ll, ll, ll, ctypes.c_char_p, vp, ll]
    return lib


def _edge_rows(ncols):
    import numpy as np

    rng = np.random.default_rng(3)
    v = np.concatenate([
        rng.random(3000).astype(np.float32),
        (rng.standard_normal(3000) * 10.0 ** rng.integers(-44, 38, 3000)).astype(np.float32),
        np.array([0.0, -0.0, 1.0, 1e16, 1e17, 1e-4, 1e-5, 123456789.0, 0.5, np.nan, np.inf, -np.inf, 3.4e38,
                  1e-45, 2.0 ** 24, 1e15, 9.999e15, 0.1, -2.5], dtype=np.float32)])
    return v[:len(v) // ncols * ncols].reshape(-1, ncols)


def test_native_csv_rows_are_the_csv_modules_text():
    """csrc/host_log.hip: the fused engines' per-step loss rows as CSV -- the exact text
    Python's csv module writes for [step, *values, sum(values)] (repr of each double, the
    row sum in Python's order), every other row from a block, NaN / inf / subnormals."""
    import csv
    import ctypes
    import io

    lib = _host_log_lib()
    rows = _edge_rows(3)
    n = rows.shape[0] // 2
    buf = ctypes.create_string_buffer(n * 200)
    m = lib.dtp_format_loss_rows(rows.ctypes.data, 3, 1, n, 2, 11, 4, 1, buf, n * 200)
    assert m > 0
    ref = io.StringIO(newline="")
    w = csv.writer(ref)
    for k, r in enumerate(rows[1::2][:n].tolist()):
        w.writerow([11 + 4 * k, *r, sum(r)])
    assert buf.raw[:m].decode() == ref.getvalue()
    assert lib.dtp_format_loss_rows(rows.ctypes.data, 3, 0, n, 1, 0, 1, 1, buf, 10) == -1  # too small: refused


def test_native_jsonl_rows_are_json_dumps_text():
    import ctypes
    import json

    lib = _host_log_lib()
    rows = _edge_rows(2)
    names = ["loss/lossX", "loss/lossY"]
    keys = "".join(json.dumps(k) + "\n" for k in names).encode()
    n = rows.shape[0]
    buf = ctypes.create_string_buffer(n * 200)
    m = lib.dtp_format_loss_rows_jsonl(rows.ctypes.data, 2, 0, n, 1, 5, 1, keys, buf, n * 200)
    ref = "".join(json.dumps({"step": 5 + k, **{nm: float(v) for nm, v in zip(names, r)}}) + "\n"
                  for k, r in enumerate(rows.tolist()))
    assert buf.raw[:m].decode() == ref
