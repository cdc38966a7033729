#!/bin/bash
# round 5: xGMI exchange with publisher / poller waves, share-GPU rehearsal A/B (W = 2 / 4 / 8),
# split-batch policy check, GPU tests of every touched path
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
V=distributed_training_pytorch_amd/_lib/var_xnosplit/libdtp.so
for W in 2 4 8; do
  timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 >> $O/share_w${W}_split.json 2>> $O/share.err || exit $?
  DTP_LIB=$V timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 >> $O/share_w${W}_nosplit.json 2>> $O/share.err || exit $?
  timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 --groups off >> $O/share_w${W}_split_goff.json 2>> $O/share.err || exit $?
  timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 --groups on >> $O/share_w${W}_split_gon.json 2>> $O/share.err || exit $?
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_xgmi_gpu.py tests/test_bench_gpu.py tests/test_lanes_gpu.py tests/test_bf16_gpu.py tests/test_loss_optim_gpu.py > $O/tests.log 2>&1
