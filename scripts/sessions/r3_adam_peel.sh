#!/bin/bash
# flat Adam with the head peel (float4 body for odd-P rows): optimizer tests, wide-step A/B vs the committed .so, kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out/ap
bash scripts/gpu_steps.sh \
  "400|ap/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_loss_optim_gpu.py tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_graph_xgmi_gpu.py" \
  "300|ap/ab|for w in 4096 2048; do for r in 1 2 3; do python scripts/bench_wide.py --impl ours --width \$w --steps 30; python scripts/bench_wide.py --impl ours --width \$w --steps 30 --shadow; done; done" \
  "200|ap/prof|timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ap/prof -o w4096 -- python3 scripts/bench_wide.py --impl ours --width 4096 --steps 20"
