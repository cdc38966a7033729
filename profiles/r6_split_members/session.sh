#!/bin/bash
# round 6: split-batch layer-split stages (csrc/split_lanes.hip) -- correctness against the
# unsplit fp64 reference, then us per iteration against the one-workgroup stages
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_split_fused_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest_split.log 2>&1 || exit $?
timeout -k 10 300 python scripts/split_members_cost.py > $O/split_cost.json 2> $O/split_cost.err || exit $?
