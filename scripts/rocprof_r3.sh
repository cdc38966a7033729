#!/bin/bash
# rocprofv3 kernel traces of the round-3 paths (run on the GPU box):
#   k20      the driver's bench call (K=20, W=5): timed-launch kernel time vs bench wall
#   k2000    the steady state
#   bf16     bench --precision bf16 (the bf16 fused instance)
#   split    the layer-split demo's persistent stage kernels (2 stages, one GPU)
# usage: bash scripts/rocprof_r3.sh <tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
tag="${1:-r3}"
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
out="$R/gpurun_out/rocprof_$tag"
mkdir -p "$out"
run() {  # name secs script args...
  local name=$1 secs=$2; shift 2
  echo "=== $name" | tee -a "$out/steps.log"
  timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name" -o "$name" -- \
    python3 "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$out/steps.log"
  tail -2 "$out/$name.log"
  return $rc
}
run k20 120 "$R/bench.py" --steps 20 --warmup 5 &&
run k2000 120 "$R/bench.py" --steps 2000 --warmup 200 &&
run bf16 120 "$R/bench.py" --steps 2000 --warmup 200 --precision bf16 &&
run split 180 "$R/demo_one_model_multi_gpu.py" --gpus_per_proc 2 --allow_shared_gpu --iters 2000 --seed 0 \
    --dry_run --no_progress --log_every 500 --steps_per_launch 500 --log_dir "$out/split_logs"
