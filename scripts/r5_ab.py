"""Summarise bench A/B JSON files of a session directory: us/step per file."""
import glob
import json
import sys

for f in sorted(glob.glob(f"{sys.argv[1]}/*.json")):
    vals = []
    for l in open(f):
        if l.startswith("{"):
            vals.append(round(json.loads(l)["ms_per_step"] * 1e3, 3))
    print(f.split("/")[-1], vals)
