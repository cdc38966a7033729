#!/bin/bash
# PMC counter passes (kernel-trace + counters only; no other trace domains).
# usage: bash scripts/rocprof_pmc.sh <tag> <what>   what = toy | gemm
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
tag="${1:-r1}"; what="${2:-toy}"
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
out="$R/gpurun_out/pmc_$tag"
mkdir -p "$out"
if [ "$what" = toy ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d "$out/toy" -o toy -- python3 "$R/bench.py" --steps 2000 --warmup 200 > "$out/toy.log" 2>&1
else
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
    --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    -d "$out/gemm" -o gemm -- python3 "$R/scripts/bench_gemm.py" > "$out/gemm.log" 2>&1
fi
