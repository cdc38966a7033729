#!/bin/bash
# bf16 weight shadow written by the flat Adam kernel: tests, wide-step A/B, kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out/sh
bash scripts/gpu_steps.sh \
  "300|sh/tests|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_loss_optim_gpu.py tests/test_entrypoints_gpu.py -k 'shadow or wide or lightning or optim'" \
  "300|sh/ab|for w in 4096 2048 1024; do b=8192; [ \$w = 1024 ] && b=16384; for r in 1 2; do python scripts/bench_wide.py --impl ours --width \$w --batch \$b --steps 30; python scripts/bench_wide.py --impl ours --width \$w --batch \$b --steps 30 --no-shadow; done; done" \
  "200|sh/prof|timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sh/prof -o w4096 -- python3 scripts/bench_wide.py --impl ours --width 4096 --steps 20"
