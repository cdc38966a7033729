#!/bin/bash
# round 5: split-batch step (csrc/grp_core.h) first GPU check: bench A/B, stamps, lanes + bf16 + loss/optim tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 150 python bench.py --steps 2000 --warmup 200 > $O/bench_grp.json 2> $O/bench_grp.err || exit $?
DTP_GROUPS=1 timeout -k 10 150 python bench.py --steps 2000 --warmup 200 > $O/bench_nogrp.json 2> $O/bench_nogrp.err || exit $?
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2>> $O/bench_grp.err || exit $?
timeout -k 10 150 python scripts/prof_stamps.py --groups --batch 256 > $O/stamps_grp.log 2>&1 || exit $?
for i in 1 2; do
  DTP_LIB=distributed_training_pytorch_amd/_lib/var_grp_plain/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_plain.json 2>> $O/ab.err || exit $?
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/ab_sc1.json 2>> $O/ab.err || exit $?
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lanes_gpu.py > $O/lanes.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bf16_gpu.py > $O/bf16.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_loss_optim_gpu.py > $O/lossopt.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_xgmi_gpu.py tests/test_bench_gpu.py > $O/xgmi_bench.log 2>&1
