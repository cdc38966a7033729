#!/bin/bash
# round 6: LDS-DMA prologue fill -- stamps, K=20 default vs pool stream (interleaved x8),
# K=2000, the lanes / split / xGMI tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 120 python scripts/k20_prologue.py > $O/k20_prologue.json 2> $O/k20_prologue.err || exit $?
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --stream default >> $O/bench_k20.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --stream pool >> $O/bench_k20_pool.json 2>> $O/err.log || exit $?
done
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_k2000.json 2>> $O/err.log || exit $?
done
timeout -k 10 900 python -u -m pytest tests/test_lanes_gpu.py tests/test_split_fused_gpu.py tests/test_xgmi_gpu.py tests/test_loss_optim_gpu.py tests/test_bf16_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
