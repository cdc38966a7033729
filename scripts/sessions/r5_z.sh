#!/bin/bash
# round 5: where the K=20 call's fixed cost goes with the split-batch step: kernel trace of
# the bench's K=20 calls (official + 3 extra), and K=1 / K=5 calls
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5z
mkdir -p $O
DTP_BENCH_EXTRA=3 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o k20 -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/k20_trace.json 2> $O/k20_trace.err || exit $?
for k in 1 5 20; do
  DTP_BENCH_EXTRA=5 timeout -k 10 150 python3 bench.py --gpus 1 --steps $k --warmup 5 >> $O/kscan.json 2>> $O/err.log || exit $?
done
