#!/bin/bash
# round 6: plain-store links between split-batch stages on one XCD (split_lanes.hip link
# hello) -- split tests, then us/iteration against the write-through links (var_wt), interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_split_fused_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
L=$PWD/distributed_training_pytorch_amd/_lib
for i in 1 2 3; do
  timeout -k 10 300 python scripts/split_members_cost.py >> $O/split_plain.json 2>> $O/err.log || exit $?
  DTP_LIB=$L/var_wt/libdtp.so timeout -k 10 300 python scripts/split_members_cost.py >> $O/split_wt.json 2>> $O/err.log || exit $?
done
