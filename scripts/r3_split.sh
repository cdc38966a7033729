#!/bin/bash
# in-launch split-K reduction: tests, wide steps at the split-K widths, kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out/split
bash scripts/gpu_steps.sh \
  "300|split/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py" \
  "200|split/w2048|python scripts/bench_wide.py --width 2048 --impl ours --gemm-backend mfma; python scripts/bench_wide.py --width 2048 --impl ours --gemm-backend blaslt" \
  "200|split/w1024|python scripts/bench_wide.py --width 1024 --batch 16384 --impl ours --gemm-backend mfma; python scripts/bench_wide.py --width 1024 --batch 16384 --impl ours --gemm-backend blaslt" \
  "200|split/prof_w2048|timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/split/prof -o mfma_w2048 -- python3 scripts/bench_wide.py --width 2048 --impl ours --gemm-backend mfma"
