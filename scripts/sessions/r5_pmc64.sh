#!/bin/bash
# round 5: SQ counter pass B (LDS bank conflicts) of the 4-lanes step alone (batch 64, one
# workgroup per model, no exchange) and of the split-batch step with the exchange's LDS
# traffic, to place the split-batch kernel's LDS conflicts
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
out="$R/gpurun_out/pmc_r5l64"
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAVES \
  -d "$out/B" -o B -- python3 "$R/bench.py" --steps 2000 --warmup 200 --scaling weak --batch 64 > "$out/B.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC \
  -d "$out/A" -o A -- python3 "$R/bench.py" --steps 2000 --warmup 200 --scaling weak --batch 64 > "$out/A.log" 2>&1
