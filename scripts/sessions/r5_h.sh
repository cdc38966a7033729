#!/bin/bash
# round 5: loss / optimizer / precision matrix of the fast steps (weak scaling, one rank,
# per-rank batch 256 / 128 / 64), K=2000 steady state
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5h
mkdir -p $O
for B in 256 128 64; do
  for cfg in "adam mse fp32" "sgd mse fp32" "adam ce fp32" "sgd ce fp32" "adam mse bf16"; do
    set -- $cfg
    timeout -k 10 150 python bench.py --scaling weak --batch $B --optimizer $1 --loss $2 --precision $3 --steps 2000 --warmup 200 >> $O/m_${B}_$1_$2_$3.json 2>> $O/m.err || exit $?
  done
done
