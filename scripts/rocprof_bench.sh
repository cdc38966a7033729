#!/bin/bash
# rocprofv3 kernel-trace/stats summaries of the bench in each launch mode (run on the GPU box).
# usage: bash scripts/rocprof_bench.sh <tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
tag="${1:-r1}"
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
out="$R/gpurun_out/rocprof_$tag"
mkdir -p "$out"
run() {  # name secs args...
  local name=$1 secs=$2; shift 2
  echo "=== $name" | tee -a "$out/steps.log"
  timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name" -o "$name" -- \
    python3 "$R/bench.py" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$out/steps.log"
  tail -2 "$out/$name.log"
  return $rc
}
run persistent 240 --steps 2000 --warmup 200 &&
run graph 240 --steps 500 --warmup 50 --launch graph --steps-per-launch 50 &&
run eager 240 --steps 300 --warmup 30 --launch eager &&
run stock 300 --steps 200 --warmup 20 --impl stock &&
timeout -k 10 60 rocprofv3 -L > "$out/counters.txt" 2>&1
