#!/bin/bash
# round 5: split-batch step after the status-load fix: bench A/B, stamps, lanes tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
for i in 1 2; do
timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_grp.json 2>> $O/bench.err || exit $?
DTP_GROUPS=1 timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_nogrp.json 2>> $O/bench.err || exit $?
done
timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/stamps_grp.log 2>&1 || exit $?
timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 128 > $O/stamps_grp128.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lanes_gpu.py > $O/lanes.log 2>&1
