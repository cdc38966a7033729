#!/usr/bin/env python3
"""A/B of the HIP runtime's host-side wait and launch modes on the bench sequence.

``bench.py --steps 20`` times ONE ``train(20)`` call plus ``torch.cuda.synchronize``;
how the host thread waits for the kernel's completion signal (spin vs. interrupt)
and where the kernel arguments live are runtime settings, not kernel work.  Each
variant runs ``bench.py`` in a fresh process (the settings are read at HIP init).

Usage: python scripts/latency_modes.py [--reps 3] [--steps 20] [--warmup 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

VARIANTS = {
    "default": {},
    "spin_flag": {"DTP_WAIT_MODE": "spin"},
    "active_wait_env": {"ROC_ACTIVE_WAIT_TIMEOUT": "100000"},
    "dev_kernarg": {"HIP_FORCE_DEV_KERNARG": "1"},
    "spin_flag+dev_kernarg": {"DTP_WAIT_MODE": "spin", "HIP_FORCE_DEV_KERNARG": "1"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    a = ap.parse_args()
    out = {}
    for name in a.variants.split(","):
        env = dict(os.environ)
        env.pop("DTP_WAIT_MODE", None)
        env.update(VARIANTS[name])
        vals = []
        for _ in range(a.reps):
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(a.steps),
                                "--warmup", str(a.warmup)], env=env, capture_output=True, text=True, timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not line:
                vals.append(None)
                print(f"[{name}] rc={r.returncode} {r.stderr[-400:]}", flush=True)
                continue
            rec = json.loads(line[-1])
            vals.append(rec["ms_per_step"] * 1e3)
        good = [v for v in vals if v is not None]
        out[name] = {"us_per_step": vals, "median": statistics.median(good) if good else None}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
