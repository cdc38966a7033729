#!/bin/bash
# round 6: prologue fill in one round trip + Trainer flat optimizer zeroing its gradient.
# stamps, driver K=20 line x6, K=2000 x2, the Trainer module path, GPU tests of the touched paths
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 120 python scripts/k20_prologue.py > $O/k20_prologue.json 2> $O/k20_prologue.err || exit $?
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_k20.json 2>> $O/err.log || exit $?
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --stream pool >> $O/bench_k20_pool.json 2>> $O/err.log || exit $?
done
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_k2000.json 2>> $O/err.log || exit $?
  DTP_GRP_NW=8 timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_k2000_2members.json 2>> $O/err.log || exit $?
done
for i in 1 2; do
  timeout -k 10 200 python demo_pytorch_lightning.py --gpus 1 --steps 3000 --seed 0 --no_progress --engine module --root_dir /tmp/ltm$i > $O/lt_module_$i.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests/test_lanes_gpu.py tests/test_split_fused_gpu.py tests/test_trainer_fused_gpu.py tests/test_loss_op.py tests/test_entrypoints_gpu.py tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
