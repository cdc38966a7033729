#!/bin/bash
# split-K reduction pass (8 columns / thread, slices 4 at a time, nontemporal partial reads): tests, wide steps, trace
export TMPDIR=/tmp
mkdir -p gpurun_out/split2
bash scripts/gpu_steps.sh \
  "300|split2/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py" \
  "200|split2/w2048|python scripts/bench_wide.py --width 2048 --impl ours --gemm-backend mfma; python scripts/bench_wide.py --width 2048 --impl ours --gemm-backend blaslt" \
  "200|split2/w1024|python scripts/bench_wide.py --width 1024 --batch 16384 --impl ours --gemm-backend mfma; python scripts/bench_wide.py --width 1024 --batch 16384 --impl ours --gemm-backend blaslt" \
  "200|split2/prof_w2048|timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/split2/prof -o mfma_w2048 -- python3 scripts/bench_wide.py --width 2048 --impl ours --gemm-backend mfma"
