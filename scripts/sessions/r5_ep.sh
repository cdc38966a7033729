#!/bin/bash
# round 5: the entrypoints on one GPU (scripts/entry_perf.sh) plus the module engine at 5000
# iterations and the layer split's module engine with 4 micro-batches
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
mkdir -p gpurun_out/r5ep
bash scripts/entry_perf.sh > gpurun_out/r5ep/entry_perf.txt 2>&1 || exit $?
timeout -k 10 200 python demo.py --engine module --iters 5000 --seed 0 --no_progress > gpurun_out/r5ep/module5k.log 2>&1 || exit $?
timeout -k 10 200 python demo_one_model_multi_gpu.py --allow_shared_gpu --microbatches 4 --engine module --iters 1000 --seed 0 --no_progress > gpurun_out/r5ep/split_mb4_module.log 2>&1
