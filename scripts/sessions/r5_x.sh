#!/bin/bash
# round 5: direct 3-float publish from the parked tiles (DTP_GRP_DIRECT3) -- split tests,
# stamps, A/B against the staged form (var_nod3), K=2000 and K=20; micro-batched split demo
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5x
L=distributed_training_pytorch_amd/_lib
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lanes_gpu.py tests/test_loss_optim_gpu.py tests/test_bf16_gpu.py tests/test_graph_xgmi_gpu.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/stamps.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_main.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_nod3/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_nod3.json 2>> $O/err.log || exit $?
done
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/k20_main.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_nod3/libdtp.so timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/k20_nod3.json 2>> $O/err.log || exit $?
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_entrypoints_gpu.py -k "layer_split" > $O/split_tests.log 2>&1
