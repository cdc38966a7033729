#!/bin/bash
# round 6: the whole GPU suite once more on another box (a flakiness check before the
# driver's round-end run), then the driver's K=20 line three times
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6ag
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_k20.json 2>> $O/err.log || exit $?
done
