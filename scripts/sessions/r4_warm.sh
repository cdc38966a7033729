#!/bin/bash
# round 4: do the first launches of a fresh process cost the K=20 line?  0 vs 64 tiny
# no-op launches (not training steps) before the timed call; fresh processes, interleaved
export TMPDIR=/tmp
D=${1:-r4warm}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/k20|for r in 1 2 3 4 5 6; do for v in 0 64; do echo warm=\$v; DTP_BENCH_RUNTIME_WARM=\$v python bench.py --steps 20 --warmup 5 | grep -o '\"ms_per_step\": [0-9.e-]*'; done; done"
