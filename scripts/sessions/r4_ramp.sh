#!/bin/bash
# round 4: is the slow-box K=20 line GPU clock ramp or host latency?  K=20 with and without
# a 30 ms GPU busy-wait right before the timed call (fresh processes, interleaved), and a
# kernel trace of each
export TMPDIR=/tmp
D=${1:-r4ramp}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/k20|python scripts/host_latency.py && for r in 1 2 3 4 5; do for v in 0 30000; do echo busy=\$v; DTP_BENCH_DEVICE_BUSY_US=\$v python bench.py --steps 20 --warmup 5 | grep -o '\"ms_per_step\": [0-9.e-]*'; done; done" \
  "200|$D/trace0|timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$D/prof0 -o k20 -- python3 bench.py --steps 20 --warmup 5" \
  "200|$D/trace1|DTP_BENCH_DEVICE_BUSY_US=30000 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$D/prof1 -o k20 -- python3 bench.py --steps 20 --warmup 5"
