#!/bin/bash
# wide-MLP training step: all-MFMA (8-phase GEMM default + split-K plan) vs hipBLASLt backend vs stock PyTorch
export TMPDIR=/tmp
mkdir -p gpurun_out/wide3
bash scripts/gpu_steps.sh \
  "300|wide3/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py" \
  "200|wide3/w4096|for be in mfma blaslt; do python scripts/bench_wide.py --width 4096 --impl ours --gemm-backend \$be; done; python scripts/bench_wide.py --width 4096 --impl stock" \
  "200|wide3/w2048|for be in mfma blaslt; do python scripts/bench_wide.py --width 2048 --impl ours --gemm-backend \$be; done; python scripts/bench_wide.py --width 2048 --impl stock" \
  "200|wide3/w1024|for be in mfma blaslt; do python scripts/bench_wide.py --width 1024 --batch 16384 --impl ours --gemm-backend \$be; done; python scripts/bench_wide.py --width 1024 --batch 16384 --impl stock" \
  "200|wide3/prof_mfma|timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wide3/prof -o mfma_w4096 -- python3 scripts/bench_wide.py --width 4096 --impl ours --gemm-backend mfma" \
  "200|wide3/prof_mfma2048|timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wide3/prof -o mfma_w2048 -- python3 scripts/bench_wide.py --width 2048 --impl ours --gemm-backend mfma"
