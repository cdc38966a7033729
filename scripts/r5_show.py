"""Summarise a split-batch GPU session directory: bench lines and exchange stamps."""
import json
import sys

d = sys.argv[1]
for f in ("bench_grp.json", "bench_nogrp.json"):
    try:
        for l in open(f"{d}/{f}"):
            if l.startswith("{"):
                r = json.loads(l)
                print(f, round(r["ms_per_step"] * 1e3, 3), "us/step", r["config"].get("lanes_per_sample"),
                      r["config"].get("workgroups_per_model"), r["final_loss"])
    except FileNotFoundError:
        pass
for fn in ("stamps_grp.log", "stamps_grp128.log"):
    try:
        t = open(f"{d}/{fn}").read()
    except FileNotFoundError:
        continue
    i = t.index("{")
    obj, end = json.JSONDecoder().raw_decode(t[i:])
    o = obj["2"]
    print(fn, {k: o[k] for k in ("x_loaded", "fwd+loss", "bwd_done(w0)", "tiles_reduced", "grads_summed", "adam_done",
                                 "step_end", "total_step")})
    print("   placement", obj.get("placement", [None])[-1])
    print("   realtime", obj.get("realtime_10ns", [None])[-2:])
    for x in obj["exchange_detail"][-1]:
        print("  ", x)
    print("  ", t[i + end:].strip()[:200])
