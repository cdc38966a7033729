#!/bin/bash
# round 6: unshuffled samplers (one rank reading in order: the Lightning demo at 1 GPU;
# DistributedSampler(shuffle=False)) through an identity permutation table, so the fused
# step's fast instances serve them -- tests, then the Lightning demo and demo.py
# --dataloader standard (DTP_FAST=0: the generic instance, as before)
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_trainer_fused_gpu.py tests/test_kernels_gpu.py tests/test_lanes_gpu.py tests/test_entrypoints_gpu.py tests/test_graph_xgmi_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/lt$r > $O/lt_table_$r.log 2>&1 || exit $?
  DTP_FAST=0 timeout -k 10 200 python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/lg$r > $O/lt_generic_$r.log 2>&1 || exit $?
  timeout -k 10 200 python demo.py --iters 20000 --seed 0 --no_progress --dataloader standard --log_dir /tmp/ds$r > $O/demo_std_table_$r.log 2>&1 || exit $?
  DTP_FAST=0 timeout -k 10 200 python demo.py --iters 20000 --seed 0 --no_progress --dataloader standard --log_dir /tmp/dg$r > $O/demo_std_generic_$r.log 2>&1 || exit $?
done
cmp /tmp/lt1/lightning_logs/version_0/metrics.csv /tmp/lg1/lightning_logs/version_0/metrics.csv > $O/cmp.txt 2>&1 && echo "metrics.csv identical (fast vs generic instance)" >> $O/cmp.txt || true
