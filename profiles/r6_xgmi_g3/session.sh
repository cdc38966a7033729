#!/bin/bash
# round 6, first box: bench contract + xGMI correctness (3-float exchange now the default of
# the 4-wave lanes instances), the driver's K=20 line in 6 fresh processes, K=2000, the
# share-GPU rehearsal A/B of the cross-GPU exchange forms, and the lanes tolerance probe
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_bench_gpu.py tests/test_xgmi_gpu.py tests/test_graph_xgmi_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_k20.json 2>> $O/err.log || exit $?
done
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_k2000.json 2>> $O/err.log || exit $?
done
L=distributed_training_pytorch_amd/_lib
for round in 1 2; do
  for v in default g2 pubw1 pubw2; do
    lib=$L/libdtp.so; [ $v != default ] && lib=$L/var_$v/libdtp.so
    for W in 2 4 8; do
      DTP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 \
        | sed "s/^{/{\"variant\": \"$v\", /" >> $O/share_w${W}.json 2>> $O/share.err || exit $?
    done
  done
done
timeout -k 10 300 python scripts/tol_probe.py > $O/tol_probe.json 2> $O/tol_probe.err || exit $?
