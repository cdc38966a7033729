#!/bin/bash
# 8-phase GEMM: correctness on every layout, then interleaved A/B vs the two-buffer kernel and hipBLASLt
export TMPDIR=/tmp
mkdir -p gpurun_out/ph8
bash scripts/gpu_steps.sh \
  "240|ph8/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k 'fast_kernel'" \
  "200|ph8/var_sq|VARIANTS=var2,var32,var33,var34,torch python scripts/gemm_variants.py 5" \
  "200|ph8/var_wide|SHAPES=wide VARIANTS=var2,var32,var33,var34,torch python scripts/gemm_variants.py 5"
