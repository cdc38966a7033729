#!/usr/bin/env python3
"""Per-wave, per-step SQ counters of the fused step from `scripts/pmc_step.sh` runs.

Usage: python scripts/pmc_summary.py [--waves N] TAG [TAG ...]   (reads gpurun_out/pmc_TAG/{A,B}/)
The last fused-step dispatch (mlp_train_kernel / mlp_train_lanes_kernel) of each pass is the
1000-step persistent launch of bench.py; its counters are divided by 1000 steps and the
waves of the launch (8: one workgroup per model; 32: the split-batch step, 8 workgroups).
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* are in quad-cycles.
"""
import collections
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def summary(tag: str, base: str = "gpurun_out", steps: int = 1000, waves: int = 8) -> dict:
    res = {}
    for p in "AB":
        path = os.path.join(ROOT, base, f"pmc_{tag}", p, f"{p}_counter_collection.csv")
        rows = [r for r in csv.DictReader(open(path)) if "mlp_train" in r["Kernel_Name"]]
        by = collections.defaultdict(dict)
        for r in rows:
            by[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        res.update(list(by.values())[-1])
    return {k.replace("SQ_", ""): round(v / steps / waves, 1) for k, v in sorted(res.items()) if k != "SQ_WAVES"}


if __name__ == "__main__":
    args = sys.argv[1:]
    w = 8
    if "--waves" in args:
        i = args.index("--waves")
        w = int(args[i + 1])
        args = args[:i] + args[i + 2:]
    for t in args:
        print(t, summary(t, waves=w))
