#!/bin/bash
# round 4: where the Lightning demo's module path (Trainer without the fused engine) spends
# a batch -- host profile, then a kernel trace of the same run
export TMPDIR=/tmp WANDB_MODE=dryrun
D=${1:-r4lt}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/host_prof|python scripts/prof_lightning.py 3000" \
  "300|$D/rocprof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$D/prof -o lt -- python3 demo_pytorch_lightning.py --gpus 1 --steps 3000 --seed 0 --root_dir /tmp/ltq --engine module"
