#!/usr/bin/env python3
"""A/B the fused step across library builds (``build.variant``), each in fresh processes.

Usage: python scripts/ab_libs.py NAME=PATH [NAME=PATH ...] [--reps 3] [--steps 2000 --warmup 200]
       (PATH "default" = the in-tree library).  Runs are interleaved over the variants so
       clock drift hits every variant alike; prints the median µs/step per variant.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(lib: str, steps: int, warmup: int, extra: list[str]) -> float | None:
    env = dict(os.environ)
    env.pop("DTP_LIB", None)
    if lib != "default":
        env["DTP_LIB"] = os.path.abspath(lib)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(steps), "--warmup",
                        str(warmup), *extra], env=env, capture_output=True, text=True, timeout=300)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not line:
        print(f"[{lib}] rc={r.returncode} {r.stderr[-600:]}", flush=True)
        return None
    return json.loads(line[-1])["ms_per_step"] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--extra", default="", help="extra bench.py args, space separated")
    a = ap.parse_args()
    libs = dict(x.split("=", 1) for x in a.libs)
    res = {n: [] for n in libs}
    for _ in range(a.reps):
        for n, p in libs.items():
            res[n].append(run(p, a.steps, a.warmup, a.extra.split()))
    out = {n: {"us_per_step": v, "median": statistics.median([x for x in v if x is not None] or [float("nan")])}
           for n, v in res.items()}
    for n, v in out.items():
        print(n, v, flush=True)
    print(json.dumps({"steps": a.steps, "warmup": a.warmup, "results": out}))


if __name__ == "__main__":
    main()
