#!/bin/bash
# round 6: the matrix of step options at batch 256 on the final kernels (K=2000): fp32
# Adam / SGD / CE, bf16; plus the driver-style K=20 line for bf16
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6v
mkdir -p $O
for r in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/adam.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --optimizer sgd >> $O/sgd.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --loss ce >> $O/ce.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --precision bf16 >> $O/bf16.json 2>> $O/err.log || exit $?
done
for r in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --precision bf16 >> $O/bf16_k20.json 2>> $O/err.log || exit $?
done
