#!/bin/bash
# round 4: K=20 line vs the number of warm-up steps (each its own launch up to 16):
# does the timed call's cost depend on how many launches the process made before it?
export TMPDIR=/tmp
D=${1:-r4wu}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/k20|for r in 1 2 3 4; do for w in 5 16 64; do echo warmup=\$w; python bench.py --steps 20 --warmup \$w | grep -o '\"ms_per_step\": [0-9.e-]*'; done; done; for r in 1 2 3; do for w in 5 16; do echo launches=\$w; DTP_BENCH_WARMUP_LAUNCHES=\$w python bench.py --steps 20 --warmup 64 | grep -o '\"ms_per_step\": [0-9.e-]*'; done; done"
