#!/bin/bash
# round 4: split engine stream handling (no per-launch cross-stream waits), split demo wall
# time vs kernel time, lanes step times with the Adam change
export TMPDIR=/tmp WANDB_MODE=dryrun
D=${1:-r4s}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "400|$D/tests|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_split_fused_gpu.py tests/test_entrypoints_gpu.py tests/test_layer_split.py" \
  "300|$D/demo|for n in 1000 20000; do timeout -k 10 120 python demo_one_model_multi_gpu.py --allow_shared_gpu --iters \$n --seed 0 --no_progress | grep summary; done && timeout -k 10 120 python demo_one_model_multi_gpu.py --allow_shared_gpu --iters 20000 --seed 0 --no_progress --steps_per_launch 1000 --log_every 1000 | grep summary" \
  "200|$D/lanes|for b in 64 128 256; do python bench.py --scaling weak --batch \$b; done"
