#!/bin/bash
# round 4: spread of the driver's K=20 line over fresh processes on one box
export TMPDIR=/tmp
D=${1:-r4k20}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/k20|for r in \$(seq 12); do python bench.py --steps 20 --warmup 5 | grep -o '\"ms_per_step\": [0-9.e-]*'; done"
