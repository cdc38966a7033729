#!/bin/bash
# flat Adam: 2x unrolled nontemporal streams -- numerics tests, wide step, kernel time
export TMPDIR=/tmp
mkdir -p gpurun_out/opt
bash scripts/gpu_steps.sh \
  "300|opt/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_loss_optim_gpu.py -k 'optim or adam or sgd'" \
  "200|opt/w4096|python scripts/bench_wide.py --width 4096 --impl ours --gemm-backend mfma" \
  "200|opt/prof_w4096|timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/opt/prof -o w4096 -- python3 scripts/bench_wide.py --width 4096 --impl ours --gemm-backend mfma"
