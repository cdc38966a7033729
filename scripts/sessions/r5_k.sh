#!/bin/bash
# round 5: split-batch exchange with pipelined polls: stamps + bench A/B at one rank
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/stamps_grp.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --groups on >> $O/bench_grp.json 2>> $O/ab.err || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --groups off >> $O/bench_nogrp.json 2>> $O/ab.err || exit $?
done
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --groups on >> $O/k20_grp.json 2>> $O/ab.err || exit $?
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --groups off >> $O/k20_nogrp.json 2>> $O/ab.err || exit $?
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lanes_gpu.py > $O/lanes.log 2>&1
