#!/bin/bash
# whole GPU suite (no -x: report every failure)
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s
bash scripts/gpu_steps.sh \
  "1000|r3s/gpu_suite|python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests"
