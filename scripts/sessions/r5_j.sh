#!/bin/bash
# round 5: the multi-rank bench line three ways (publish / wait / rest), share-GPU W = 2 / 4 / 8,
# K = 2000 and the driver's K = 20; bench GPU tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
for W in 2 4 8; do
  timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 >> $O/share_w${W}.json 2>> $O/share.err || exit $?
  timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 20 --warmup 5 >> $O/share_w${W}_k20.json 2>> $O/share.err || exit $?
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_bench_gpu.py > $O/tests.log 2>&1
