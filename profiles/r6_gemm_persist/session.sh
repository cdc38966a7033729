#!/bin/bash
# round 6: the persistent 8-phase GEMM (next tile's operand fill under this tile's
# epilogue) -- GEMM tests, then interleaved TF/s against the one-tile-per-workgroup kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
VARIANTS=var32,var35,torch SHAPES=nn timeout -k 10 400 python scripts/gemm_variants.py 7 > $O/variants_nn.jsonl 2>> $O/err.log || exit $?
VARIANTS=var32,var35,torch SHAPES=wide timeout -k 10 300 python scripts/gemm_variants.py 7 > $O/variants_wide.jsonl 2>> $O/err.log || exit $?
VARIANTS=var32,var35,torch timeout -k 10 300 python scripts/gemm_variants.py 5 > $O/variants_sq.jsonl 2>> $O/err.log || exit $?
