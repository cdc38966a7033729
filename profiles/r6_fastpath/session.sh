#!/bin/bash
# round 6: FusedTrainer.train's direct path (the common persistent call straight to the
# native launch) -- the whole GPU suite, then the driver's K=20 line against the general
# path (DTP_TRAIN_FASTPATH=0), interleaved fresh processes
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6ai
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/k20_fast.json 2>> $O/err.log || exit $?
  DTP_TRAIN_FASTPATH=0 timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/k20_general.json 2>> $O/err.log || exit $?
done
