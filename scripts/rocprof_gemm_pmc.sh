#!/bin/bash
# PMC passes over one GEMM shape (kernel-trace + counters only, one pass per counter set).
# usage: bash scripts/rocprof_gemm_pmc.sh <tag> M N K LAYOUT [fast|classic|torch]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
tag="$1"
M="$2"; N="$3"; K="$4"; L="$5"; W="${6:-fast}"
cd /tmp && export TMPDIR=/tmp
out="$R/gpurun_out/pmc_gemm_$tag"
mkdir -p "$out"
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc "$@" -d "$out/$name" -o "$name" -- \
    python3 "$R/scripts/gemm_one.py" "$M" "$N" "$K" "$L" 20 "$W" > "$out/$name.log" 2>&1
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE &&
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE
