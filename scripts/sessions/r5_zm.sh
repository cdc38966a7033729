#!/bin/bash
# round 5: missing items add +0 after an exchange timeout -- split-batch tests, the bench
# (K=2000 and K=20) to check the normal path is unchanged
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5zm
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lanes_gpu.py tests/test_loss_optim_gpu.py tests/test_bf16_gpu.py > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_default.json 2>> $O/err.log || exit $?
done
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_k20.json 2>> $O/err.log || exit $?
done
