#!/bin/bash
# round 6: the Trainer module path with the fused two-prediction MSE (one launch for
# loss_X, loss_Y and their sum), the loss / trainer / entrypoint GPU tests, and the driver
# K=20 line on the new default (pool) stream
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_loss_op.py tests/test_module_path_gpu.py tests/test_trainer_fused_gpu.py tests/test_entrypoints_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python demo_pytorch_lightning.py --gpus 1 --steps 3000 --seed 0 --no_progress --engine module --root_dir /tmp/ltm$i > $O/lt_module_$i.log 2>&1 || exit $?
done
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_k20.json 2>> $O/err.log || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lt -o lt -- python3 demo_pytorch_lightning.py --gpus 1 --steps 3000 --seed 0 --no_progress --engine module --root_dir /tmp/ltp > $O/lt_prof.log 2>&1 || exit $?
