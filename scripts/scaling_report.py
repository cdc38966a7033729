"""Run bench.py at N = 1, 2, 4, 8 GPUs of one node (one rank per GPU through
torch.distributed.run on 127.0.0.1) and print the scaling table.

    python scripts/scaling_report.py [--gpus 1 2 4 8] [--steps 2000] [--warmup 200] [-- extra bench args]

Efficiency is (value_N / N) / value_1 (per-GPU throughput relative to one GPU);
with the default weak scaling every rank keeps 256 samples per step.
Writes the raw JSON lines and the table to --out (default gpurun_out/scaling.json).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(n, steps, warmup, port, extra):
    bench = os.path.join(ROOT, "bench.py")
    base = ["--gpus", str(n), "--steps", str(steps), "--warmup", str(warmup), *extra]
    if n == 1:
        cmd = [sys.executable, bench, *base]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), bench, *base]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=900)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not lines:
        raise RuntimeError(f"bench at N={n} failed (rc={r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
    return json.loads(lines[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--port", type=int, default=29611)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "scaling.json"))
    a, extra = ap.parse_known_args()
    extra = [e for e in extra if e != "--"]
    rows = []
    for i, n in enumerate(a.gpus):
        rows.append(run(n, a.steps, a.warmup, a.port + i, extra))
        print(json.dumps(rows[-1]), flush=True)
    base = next((r["value"] for r in rows if r["n_gpus"] == 1), None)
    print(f"{'N':>3} {'samples/s':>14} {'us/step':>9} {'per-GPU':>12} {'efficiency':>10}")
    for r in rows:
        n = r["n_gpus"]
        eff = (r["value"] / n) / base if base else float("nan")
        r["efficiency_vs_1"] = eff
        print(f"{n:>3} {r['value']:>14,.0f} {1e3 * r['ms_per_step']:>9.2f} {r['value'] / n:>12,.0f} {eff:>10.1%}")
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
