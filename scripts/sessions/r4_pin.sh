#!/bin/bash
# round 4: K=20 line with the bench thread on the idlest local CPU vs the first local CPU,
# fresh processes interleaved, plus the box's host launch latency
export TMPDIR=/tmp
D=${1:-r4pin}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/k20|python scripts/host_latency.py && for r in 1 2 3 4 5 6; do for v in idle first; do echo pin=\$v; DTP_BENCH_PIN=\$v python bench.py --steps 20 --warmup 5 | grep -o '\"ms_per_step\": [0-9.e-]*\|\"host_cpu\": [0-9]*'; done; done"
