#!/bin/bash
# round 5: two waves per SIMD at batch 256 (DTP_LANES=2x8, one workgroup per model) against
# the split-batch default and the one-lane step, K=2000, interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/grp.json 2>> $O/err.log || exit $?
  DTP_LANES=2x8 timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --groups off >> $O/l2x8.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --groups off >> $O/onewg.json 2>> $O/err.log || exit $?
done
