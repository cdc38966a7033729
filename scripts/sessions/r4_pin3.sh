#!/bin/bash
# round 4: K=20 line with the bench thread unpinned / on the 4 idlest local CPUs / on the idlest
# local CPU; fresh processes, interleaved
export TMPDIR=/tmp
D=${1:-r4pin5}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/k20|python scripts/host_latency.py && for r in 1 2 3 4 5; do for v in 0 set one; do echo pin=\$v; DTP_BENCH_PIN=\$v python bench.py --steps 20 --warmup 5 | grep -o '\"ms_per_step\": [0-9.e-]*'; done; done"
