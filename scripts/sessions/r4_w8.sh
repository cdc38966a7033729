#!/bin/bash
# round 4 (after the Adam change): the two-waves-per-SIMD lanes instances against the
# default pick at the batches where they compete, interleaved
export TMPDIR=/tmp
D=${1:-r4w8}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/ab|for r in 1 2 3; do for v in default:256 2x8:256 default:128 4x8:128; do l=\${v%%:*}; b=\${v##*:}; echo \"\$l batch=\$b\"; if [ \$l = default ]; then python bench.py --scaling weak --batch \$b; else DTP_LANES=\$l python bench.py --scaling weak --batch \$b; fi | grep -o '\"ms_per_step\": [0-9.e-]*'; done; done"
