#!/bin/bash
# round 6 diagnostic: does the driver's first timed K=20 call of a fresh process pay a GPU
# clock ramp?  DTP_BENCH_CLOCK_WARM_MS untimed GEMMs before the timed region vs none,
# interleaved fresh processes; DTP_BENCH_EXTRA=3 times three more calls after the official one
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ab
mkdir -p $O
for i in 1 2 3 4 5 6; do
  DTP_BENCH_EXTRA=3 timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/k20_plain.json 2>> $O/err.log || exit $?
  DTP_BENCH_EXTRA=3 DTP_BENCH_CLOCK_WARM_MS=30 timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/k20_warm.json 2>> $O/err.log || exit $?
done
