#!/bin/bash
# round 5: split-batch step: placement + plain-store vs sc1-store hand-off A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O $O/plain
V=distributed_training_pytorch_amd/_lib/var_grp_plain/libdtp.so
timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/stamps_grp.log 2>&1 || exit $?
DTP_LIB=$V timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/plain/stamps_grp.log 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_grp.json 2>> $O/bench.err || exit $?
DTP_LIB=$V timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/plain/bench_grp.json 2>> $O/bench.err || exit $?
done
