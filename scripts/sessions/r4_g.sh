#!/bin/bash
# round 4, session g: split stamps (K = 1, 2) and the pipelined-vs-round-3 split body A/B
export TMPDIR=/tmp
D=${1:-r4g}
mkdir -p gpurun_out/$D
V1=distributed_training_pytorch_amd/_lib/var_splitv1/libdtp.so
VP=distributed_training_pytorch_amd/_lib/var_splitprof/libdtp.so
bash scripts/gpu_steps.sh \
  "200|$D/split_stamps|DTP_LIB=$VP python scripts/split_stamps.py 1 && DTP_LIB=$VP python scripts/split_stamps.py 2" \
  "300|$D/split_tests|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_split_fused_gpu.py" \
  "400|$D/split_ab|python scripts/split_cost.py"
