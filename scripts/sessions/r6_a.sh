#!/bin/bash
# round 6, first box: the bench's clean-env N-GPU call and the cu-mask residency guard
# (tests/test_bench_gpu.py), then the driver's K=20 line in 6 fresh processes and K=2000
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bench_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest_bench.log 2>&1 || exit $?
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_k20.json 2>> $O/err.log || exit $?
done
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_k2000.json 2>> $O/err.log || exit $?
done
