#!/bin/bash
# round 6: the Trainer module path: the epoch ring gather (no per-batch index copy) A/B,
# and HIP runtime knobs (per-kernel cost in the replayed graph is ~4.4 us whatever the
# kernel does).  Each variant in a fresh process, two interleaved rounds.
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_loss_op.py tests/test_module_path_gpu.py tests/test_trainer_fused_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python demo_pytorch_lightning.py --gpus 1 --steps 6000 --seed 0 --no_progress --engine module --root_dir /tmp/ltm_$name > $O/lt_$name.$r.log 2>&1 || exit $?
  grep -o "'steady_samples_per_s': [0-9.]*" $O/lt_$name.$r.log | sed "s/^/$name /" >> $O/summary.txt
}
for r in 1 2; do
  run ring DTP_NOP=1
  run noring DTP_TRAINER_RING=0
  run pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run pc1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
  run devka HIP_FORCE_DEV_KERNARG=1
  run skipka ROC_SKIP_KERNEL_ARG_COPY=1
  run nodd AMD_DIRECT_DISPATCH=0
done
