#!/bin/bash
# round 5: bf16 several-lanes / split-batch dW tiles on one bf16 MFMA (DTP_LANES_BFMMA) --
# bf16 tests, then bf16 at batch 64 / 128 / 256 against var_nobfmma and fp32, K=2000
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5bf
L=distributed_training_pytorch_amd/_lib
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bf16_gpu.py tests/test_lanes_gpu.py > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  for b in 64 128 256; do
    timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --scaling weak --batch $b --precision bf16 >> $O/bf16_b$b.json 2>> $O/err.log || exit $?
    DTP_LIB=$L/var_nobfmma/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --scaling weak --batch $b --precision bf16 >> $O/bf16_nobfmma_b$b.json 2>> $O/err.log || exit $?
    timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --scaling weak --batch $b >> $O/fp32_b$b.json 2>> $O/err.log || exit $?
  done
done
