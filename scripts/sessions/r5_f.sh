#!/bin/bash
# round 5: split-batch hand-off A/B: XCC-guarded plain stores (main), forced plain, first-poll
# sleep 4 / 8, plain without the publisher/poller split; one-workgroup step for reference
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
L=distributed_training_pytorch_amd/_lib
timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/stamps_main.log 2>&1 || exit $?
DTP_LIB=$L/var_plain_s4/libdtp.so timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/stamps_s4.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_main.json 2>> $O/ab.err || exit $?
  DTP_GROUPS=1 timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_nogrp.json 2>> $O/ab.err || exit $?
  for v in plain plain_s4 plain_s8 plain_nosplit; do
    DTP_LIB=$L/var_$v/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_$v.json 2>> $O/ab.err || exit $?
  done
done
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/k20_main.json 2>> $O/ab.err || exit $?
  DTP_GROUPS=1 timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/k20_nogrp.json 2>> $O/ab.err || exit $?
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lanes_gpu.py > $O/lanes.log 2>&1
