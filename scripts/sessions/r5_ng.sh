#!/bin/bash
# round 5: the 3-float exchange drops the XCC id once plain (CE head: 128 granules, 2 poll
# items per lane) -- split-batch tests, then default and CE at 256, K=2000 and K=20
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ng
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lanes_gpu.py tests/test_loss_optim_gpu.py tests/test_bf16_gpu.py tests/test_xgmi_gpu.py > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/adam_mse.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --loss ce >> $O/adam_ce.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --optimizer sgd >> $O/sgd_mse.json 2>> $O/err.log || exit $?
done
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/k20.json 2>> $O/err.log || exit $?
done
