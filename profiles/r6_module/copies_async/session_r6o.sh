#!/bin/bash
# round 6: the Trainer's graph copies (4 replayed graphs per batch shape; the metric rows
# stacked once per 4 batches): tests, then an interleaved A/B against one copy.
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_module_path_gpu.py tests/test_loss_op.py tests/test_graph_step_gpu.py tests/test_trainer_fused_gpu.py tests/test_entrypoints_gpu.py tests/test_graph_xgmi_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python demo_pytorch_lightning.py --gpus 1 --steps 6000 --seed 0 --no_progress --engine module --root_dir /tmp/ltm_$name > $O/lt_$name.$r.log 2>&1 || exit $?
  grep -o "'steady_samples_per_s': [0-9.]*" $O/lt_$name.$r.log | sed "s/^/$name /" >> $O/summary.txt
}
for r in 1 2 3; do
  run copies4 DTP_NOP=1
  run copies1 DTP_TRAINER_GRAPH_COPIES=1
  run copies8 DTP_TRAINER_GRAPH_COPIES=8
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lt -o lt -- python3 demo_pytorch_lightning.py --gpus 1 --steps 3000 --seed 0 --no_progress --engine module --root_dir /tmp/ltp > $O/lt_prof.log 2>&1 || exit $?
