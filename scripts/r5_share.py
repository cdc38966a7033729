"""Summarise share-GPU rehearsal bench lines: us/step, exchange wait, pick."""
import glob
import json
import sys

for f in sorted(glob.glob(f"{sys.argv[1]}/share_*.json")):
    for l in open(f):
        if l.startswith("{"):
            r = json.loads(l)
            c = r["config"]
            print(f.split("/")[-1], round(r["ms_per_step"] * 1e3, 3), "us/step", "L", c.get("lanes_per_sample"),
                  "G", c.get("workgroups_per_model"), "wait", round(r.get("exchange_wait_us_per_step", 0), 3),
                  "loss", [round(x, 5) for x in r["final_loss"]])
