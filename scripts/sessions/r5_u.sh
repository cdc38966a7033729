#!/bin/bash
# round 5: 3-float granules in the split-batch exchange (DTP_GRP_G3) -- split-batch tests,
# stamps, A/B against the 2-float form (var_g2), K=2000 and K=20
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5u
L=distributed_training_pytorch_amd/_lib
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lanes_gpu.py tests/test_loss_optim_gpu.py tests/test_bf16_gpu.py -k "split or groups or lanes" > $O/tests.log 2>&1 || exit $?
timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/stamps.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_g3.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_g2/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_g2.json 2>> $O/err.log || exit $?
done
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/k20_g3.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_g2/libdtp.so timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/k20_g2.json 2>> $O/err.log || exit $?
done
