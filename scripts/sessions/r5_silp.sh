#!/bin/bash
# round 5: iterative-ilp scheduling of mlp_train.hip (var_silp) against the build's max-ilp,
# three interleaved rounds at batch 256 and the driver's K=20 line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5silp
L=distributed_training_pytorch_amd/_lib
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/main.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_silp/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/silp.json 2>> $O/err.log || exit $?
done
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/k20_main.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_silp/libdtp.so timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/k20_silp.json 2>> $O/err.log || exit $?
done
