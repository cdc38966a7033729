#!/bin/bash
# prologue stamps + kernel trace of repeated K=20 launches
export TMPDIR=/tmp
mkdir -p gpurun_out/r3h
bash scripts/gpu_steps.sh \
  "90|r3h/stamps|python scripts/prof_stamps.py" \
  "150|r3h/k20_rocprof|timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3h/prof -o k20 -- python3 scripts/k20_breakdown.py 20 30"
