#!/bin/bash
# round 6: the module engine's new pieces one by one on ONE box (host speed differs a lot
# between boxes for this launch-bound loop): all on, each off, all off; interleaved
# (syncflush: the loss log read back with a device sync at every log point)
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_entrypoints_gpu.py tests/test_loss_op.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python demo.py --engine module --iters 10000 --seed 0 --dry_run --no_progress --log_dir /tmp/d_$name > $O/dm_$name.$r.log 2>&1 || exit $?
  grep -o "'samples_per_s': [0-9.]*" $O/dm_$name.$r.log | sed "s/^/$name /" >> $O/summary.txt
}
for r in 1 2 3; do
  run all DTP_NOP=1
  run noring DTP_MODULE_RING=0
  run nofuse DTP_MODULE_FUSE_OPT=0
  run nolog DTP_MODULE_LOSSLOG=0
  run syncflush DTP_MODULE_SYNC_FLUSH=1
  run none DTP_MODULE_RING=0 DTP_MODULE_FUSE_OPT=0 DTP_MODULE_LOSSLOG=0 DTP_MODULE_SYNC_FLUSH=1
done
