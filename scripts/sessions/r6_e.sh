#!/bin/bash
# round 6: K=20 fixed-cost stamps of the split-batch step (scripts/k20_prologue.py), the
# layer-split demo on the split-batch stages, the split test file pinned to both kernels
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 120 python scripts/k20_prologue.py > $O/k20_prologue.json 2> $O/k20_prologue.err || exit $?
timeout -k 10 120 python scripts/k20_prologue.py >> $O/k20_prologue.json 2>> $O/k20_prologue.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_split_fused_gpu.py "tests/test_entrypoints_gpu.py::test_demo_layer_split_microbatches_on_fused_engine" -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
