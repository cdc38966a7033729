#!/bin/bash
# round 5: the 3-float exchange without the XCC id once plain, two constexpr granule counts
# (DTP_GRP_SHORT) -- split-batch tests, A/B against var_noshort for Adam + MSE and Adam + CE
# at 256, K=2000
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ng2
L=distributed_training_pytorch_amd/_lib
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lanes_gpu.py tests/test_loss_optim_gpu.py tests/test_bf16_gpu.py > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/mse_short.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_noshort/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/mse_noshort.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --loss ce >> $O/ce_short.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_noshort/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --loss ce >> $O/ce_noshort.json 2>> $O/err.log || exit $?
done
