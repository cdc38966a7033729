#!/bin/bash
# Two SQ counter passes over the 1-GPU bench (kernel-trace + counters only, one pass per run).
# usage: bash scripts/pmc_step.sh <tag> [libdtp.so]   -> gpurun_out/pmc_<tag>/{A,B}/...
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
tag="${1:-step}"
[ -n "$2" ] && export DTP_LIB="$R/$2"
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
out="$R/gpurun_out/pmc_$tag"
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC \
  -d "$out/A" -o A -- python3 "$R/bench.py" --steps 2000 --warmup 200 > "$out/A.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAVES \
  -d "$out/B" -o B -- python3 "$R/bench.py" --steps 2000 --warmup 200 > "$out/B.log" 2>&1
