#!/bin/bash
# round 5: 3-float granules -- single poll / no publisher-first barrier A/B, then the whole
# GPU suite on the new default
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5v
L=distributed_training_pytorch_amd/_lib
mkdir -p $O
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_g3.json 2>> $O/err.log || exit $?
  for v in nopipe3 nopf3; do
    DTP_LIB=$L/var_$v/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_$v.json 2>> $O/err.log || exit $?
  done
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
