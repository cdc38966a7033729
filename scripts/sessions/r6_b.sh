#!/bin/bash
# round 6: the 3-float cross-GPU exchange (xgmi_core.h:xgmi_allreduce_g3).  Correctness first
# (the xGMI GPU tests against host all-reduce / fp64 references), then the one-GPU multi-rank
# rehearsal W = 2 / 4 / 8 at K = 2000, A/B against the 2-float form (var_g2) and the
# publisher-wave variants, interleaved, two rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py tests/test_graph_xgmi_gpu.py tests/test_bench_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest_xgmi.log 2>&1 || exit $?
L=distributed_training_pytorch_amd/_lib
for round in 1 2; do
  for v in default g2 pubw1 pubw2; do
    lib=$L/libdtp.so; [ $v != default ] && lib=$L/var_$v/libdtp.so
    for W in 2 4 8; do
      DTP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 \
        | sed "s/^{/{\"variant\": \"$v\", /" >> $O/share_w${W}.json 2>> $O/share.err || exit $?
    done
  done
done
