#!/bin/bash
# round 5: split-batch exchange A/B: direct publish + pipelined polls (main), single polls,
# owner-staged publish; one-workgroup reference; stamps of main
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5q
L=distributed_training_pytorch_amd/_lib
mkdir -p $O
timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/stamps_grp.log 2>&1 || exit $?
mkdir -p $O/nopipe && DTP_LIB=$L/var_nopipe/libdtp.so timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/nopipe/stamps_grp.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --groups on >> $O/ab_main.json 2>> $O/ab.err || exit $?
  for v in nopipe nodirect; do
    DTP_LIB=$L/var_$v/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --groups on >> $O/ab_$v.json 2>> $O/ab.err || exit $?
  done
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --groups off >> $O/ab_onewg.json 2>> $O/ab.err || exit $?
done
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --groups on >> $O/k20_grp.json 2>> $O/ab.err || exit $?
  DTP_LIB=$L/var_nopipe/libdtp.so timeout -k 10 150 python bench.py --steps 20 --warmup 5 --groups on >> $O/k20_nopipe.json 2>> $O/ab.err || exit $?
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --groups off >> $O/k20_onewg.json 2>> $O/ab.err || exit $?
done
