#!/bin/bash
# round 6: the driver's scaling recipe rehearsed on one GPU (--share-gpu: every rank on the
# one device; the driver runs N = 1, 2, 4, 8 on a whole node) at its short K = 20 / W = 5,
# three fresh self-launches per N, plus K = 2000 once per N
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6af
mkdir -p $O
for W in 2 4 8; do
  for i in 1 2 3; do
    timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 20 --warmup 5 >> $O/share_k20_w$W.json 2>> $O/err.log || exit $?
  done
  timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 >> $O/share_k2000_w$W.json 2>> $O/err.log || exit $?
done
