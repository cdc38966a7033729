"""Summarise the loss / optimizer / precision matrix (gpurun_out/r5h style): us/step and pick."""
import glob
import json
import sys

for f in sorted(glob.glob(f"{sys.argv[1]}/m_*.json")):
    for l in open(f):
        if l.startswith("{"):
            r = json.loads(l)
            c = r["config"]
            print(f.split("/")[-1][2:-5], round(r["ms_per_step"] * 1e3, 3), "us/step  L", c.get("lanes_per_sample"),
                  "G", c.get("workgroups_per_model"), "loss", [round(x, 4) for x in r["final_loss"]])
