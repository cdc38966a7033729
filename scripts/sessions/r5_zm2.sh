#!/bin/bash
# round 5: A/B of the timeout zeroing (DTP_GRP_ZERO_MISSING) on the normal path, interleaved,
# K=2000
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5zm2
L=distributed_training_pytorch_amd/_lib
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/zm.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_nozm/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/nozm.json 2>> $O/err.log || exit $?
done
