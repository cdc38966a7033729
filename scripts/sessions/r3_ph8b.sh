#!/bin/bash
# 8-phase GEMM with opaque per-tile address state (balanced schedule on every layout): tests, A/B, wide step
export TMPDIR=/tmp
mkdir -p gpurun_out/ph8b
bash scripts/gpu_steps.sh \
  "300|ph8b/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py" \
  "200|ph8b/var_sq|VARIANTS=var2,var32,var34,torch python scripts/gemm_variants.py 5" \
  "200|ph8b/var_wide|SHAPES=wide VARIANTS=var2,var32,var34,torch python scripts/gemm_variants.py 5" \
  "200|ph8b/w4096|for be in mfma blaslt; do python scripts/bench_wide.py --width 4096 --impl ours --gemm-backend \$be; done; python scripts/bench_wide.py --width 4096 --impl stock" \
  "200|ph8b/w2048|for be in mfma blaslt; do python scripts/bench_wide.py --width 2048 --impl ours --gemm-backend \$be; done; python scripts/bench_wide.py --width 2048 --impl stock" \
  "200|ph8b/w1024|for be in mfma blaslt; do python scripts/bench_wide.py --width 1024 --batch 16384 --impl ours --gemm-backend \$be; done; python scripts/bench_wide.py --width 1024 --batch 16384 --impl stock" \
  "200|ph8b/prof_w4096|timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ph8b/prof -o mfma_w4096 -- python3 scripts/bench_wide.py --width 4096 --impl ours --gemm-backend mfma" \
  "200|ph8b/prof_w2048|timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ph8b/prof -o mfma_w2048 -- python3 scripts/bench_wide.py --width 2048 --impl ours --gemm-backend mfma"
