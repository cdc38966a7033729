#!/bin/bash
# round 5: next-sample work inside the split-batch exchange's waits (DTP_GRP_OVERLAP) and one
# poll in flight with 3-float granules: split tests, A/B against var_noov, K=2000 and K=20
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5w
L=distributed_training_pytorch_amd/_lib
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lanes_gpu.py tests/test_loss_optim_gpu.py tests/test_bf16_gpu.py tests/test_graph_xgmi_gpu.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/stamps.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_main.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_noov/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_noov.json 2>> $O/err.log || exit $?
done
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/k20_main.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_noov/libdtp.so timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/k20_noov.json 2>> $O/err.log || exit $?
done
