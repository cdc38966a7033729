#!/bin/bash
# round 6: lanes-kernel parameter ownership in the forward blocks' LDS order (DTP_LANE_OWN=1,
# the default build) against torch order (var_own0) -- correctness (lanes / xGMI / split-batch
# tests) then K=2000 interleaved x4 and the driver's K=20 x6 per build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_lanes_gpu.py tests/test_xgmi_gpu.py tests/test_loss_optim_gpu.py tests/test_bf16_gpu.py tests/test_graph_xgmi_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
L=$PWD/distributed_training_pytorch_amd/_lib
for i in 1 2 3 4; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/k2000_own1.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_own0/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/k2000_own0.json 2>> $O/err.log || exit $?
done
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/k20_own1.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_own0/libdtp.so timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/k20_own0.json 2>> $O/err.log || exit $?
done
for W in 2 8; do
  timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 >> $O/share_w$W.json 2>> $O/err.log || exit $?
done
