#!/bin/bash
# round 5: flat xGMI exchange with split-batch members, share-GPU rehearsal A/B (W = 2 / 4 / 8),
# xGMI + bench GPU tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
for W in 2 4 8; do
  for g in auto 1; do
    if [ $g = 1 ]; then export DTP_GROUPS=1; else unset DTP_GROUPS; fi
    timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 >> $O/share_w${W}_g${g}.json 2>> $O/share.err || exit $?
  done
done
unset DTP_GROUPS
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_xgmi_gpu.py tests/test_bench_gpu.py tests/test_loss_optim_gpu.py tests/test_bf16_gpu.py > $O/tests.log 2>&1
