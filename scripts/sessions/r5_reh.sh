#!/bin/bash
# round 5, final tree: the one-GPU multi-rank rehearsal (every rank on the one MI355X) at
# W = 2 / 4 / 8, K=2000 and K=20, with the three-way split of the bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5reh
mkdir -p $O
for W in 2 4 8; do
  timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 >> $O/share_w${W}.json 2>> $O/share.err || exit $?
  timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 20 --warmup 5 >> $O/share_w${W}_k20.json 2>> $O/share.err || exit $?
done
