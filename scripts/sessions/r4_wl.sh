#!/bin/bash
# round 4 (no pre-timing gc.collect): the K=20 line vs how the W=5 warm-up steps are
# launched (1 launch of 5 steps vs 5 one-step launches); fresh processes, interleaved
export TMPDIR=/tmp
D=${1:-r4wl}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/k20|for r in 1 2 3 4 5 6; do for l in 1 5; do echo launches=\$l; DTP_BENCH_WARMUP_LAUNCHES=\$l python bench.py --steps 20 --warmup 5 | grep -o '\"ms_per_step\": [0-9.e-]*'; done; done"
