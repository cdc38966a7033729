#!/bin/bash
# round 4, session e: split stages on the pipelined schedule
export TMPDIR=/tmp
D=${1:-r4e}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "400|$D/split_tests|python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_split_fused_gpu.py tests/test_layer_split.py" \
  "300|$D/split_cost|python scripts/split_cost.py"
