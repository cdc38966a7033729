#!/bin/bash
# round 4: the K=20 line's first timed call vs the calls after it (DTP_BENCH_EXTRA) under
# three GC settings around the timed region; fresh processes, interleaved
export TMPDIR=/tmp
D=${1:-r4gc}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/k20|for r in 1 2 3 4; do for g in collect disable none; do echo gc=\$g; DTP_BENCH_GC=\$g DTP_BENCH_EXTRA=3 python bench.py --steps 20 --warmup 5 | grep -o '\"ms_per_step\": [0-9.e-]*\|\"extra_ms_per_step\": [^]]*]' | tr '\n' ' '; echo; done; done"
