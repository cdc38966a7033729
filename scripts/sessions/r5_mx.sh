#!/bin/bash
# round 5: the loss / optimizer matrix at per-rank batch 256 with the 3-float split-batch
# exchange (SGD + MSE, Adam + CE, SGD + CE), K=2000
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5mx
mkdir -p $O
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --optimizer sgd >> $O/sgd_mse.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --loss ce >> $O/adam_ce.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --optimizer sgd --loss ce >> $O/sgd_ce.json 2>> $O/err.log || exit $?
done
