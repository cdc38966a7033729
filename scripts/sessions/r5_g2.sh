#!/bin/bash
# round 5: two split-batch members (per-rank batch 128) on the 3-float exchange against the
# 2-lanes step, fp32 and bf16, K=2000
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5g2
mkdir -p $O
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --scaling weak --batch 128 --groups on >> $O/b128_grp.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --scaling weak --batch 128 >> $O/b128_auto.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --scaling weak --batch 128 --groups on --precision bf16 >> $O/b128_grp_bf16.json 2>> $O/err.log || exit $?
done
