#!/bin/bash
# round 4, session f: split pipelined stages vs the round-3 body (A/B), numerics
export TMPDIR=/tmp
D=${1:-r4f}
mkdir -p gpurun_out/$D
V=distributed_training_pytorch_amd/_lib/var_splitv1/libdtp.so
bash scripts/gpu_steps.sh \
  "300|$D/split_tests|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_split_fused_gpu.py" \
  "400|$D/split_ab|python scripts/split_cost.py && DTP_LIB=$V python scripts/split_cost.py && python scripts/split_cost.py"
