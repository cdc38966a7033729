#!/bin/bash
# GEMM tests after trimming + PMC of the 8-phase NN layer GEMM vs hipBLASLt, then the whole GPU suite
export TMPDIR=/tmp
mkdir -p gpurun_out/r3p
bash scripts/gpu_steps.sh \
  "300|r3p/gemm_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py" \
  "200|r3p/pmc_nn|bash scripts/rocprof_gemm_pmc.sh r3nn 8192 4096 4096 NN fast" \
  "200|r3p/pmc_nn_torch|bash scripts/rocprof_gemm_pmc.sh r3nn_torch 8192 4096 4096 NN torch" \
  "600|r3p/gpu_suite|python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests"
