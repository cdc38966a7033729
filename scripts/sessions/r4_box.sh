#!/bin/bash
# round 4: box diagnostics next to the bench -- host launch latency, steady state, K=20
export TMPDIR=/tmp
D=${1:-r4box}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "200|$D/box|python scripts/host_latency.py && python bench.py | grep -o '\"ms_per_step\": [0-9.e-]*' && for r in 1 2 3 4; do python bench.py --steps 20 --warmup 5 | grep -o '\"ms_per_step\": [0-9.e-]*'; done && python scripts/host_latency.py"
