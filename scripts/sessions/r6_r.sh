#!/bin/bash
# round 6: split-batch stage links plain only when both ends run in one launch (per-stage
# launches keep write-through links) -- split tests and us/iteration; then the Trainer
# module path and the share-GPU exchange rehearsal on the current tree; the module engine's
# ModelBank backwards fused with its flat Adam (one launch for both models), A/B
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_split_fused_gpu.py tests/test_module_path_gpu.py tests/test_entrypoints_gpu.py tests/test_loss_op.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python scripts/split_members_cost.py >> $O/split.json 2>> $O/err.log || exit $?
done
for r in 1 2; do
  timeout -k 10 200 python demo_pytorch_lightning.py --gpus 1 --steps 6000 --seed 0 --no_progress --engine module --root_dir /tmp/ltm$r > $O/lt_module_$r.log 2>&1 || exit $?
done
for r in 1 2; do
  for W in 2 4 8; do
    timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 >> $O/share_w$W.json 2>> $O/err.log || exit $?
  done
done
for r in 1 2 3; do
  timeout -k 10 300 python demo.py --engine module --iters 5000 --seed 0 --dry_run --no_progress --log_dir /tmp/dm$r > $O/dm_fused_$r.log 2>&1 || exit $?
  DTP_MODULE_FUSE_OPT=0 timeout -k 10 300 python demo.py --engine module --iters 5000 --seed 0 --dry_run --no_progress --log_dir /tmp/dn$r > $O/dm_separate_$r.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dm -o dm -- python3 demo.py --engine module --iters 3000 --seed 0 --dry_run --no_progress --log_dir /tmp/dmp > $O/dm_prof.log 2>&1 || exit $?
