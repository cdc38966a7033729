#!/bin/bash
# round 6: the module engine's steady state (from step 50 on: the first kernels' code-object
# loads and the captures excluded) with its round-6 pieces on and off, interleaved
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6aa
mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python demo.py --engine module --iters 10000 --seed 0 --dry_run --no_progress --log_dir /tmp/d_$name > $O/dm_$name.$r.log 2>&1 || exit $?
  grep -o "'samples_per_s': [0-9.]*\|'steady_samples_per_s': [0-9.]*" $O/dm_$name.$r.log | tr '\n' ' ' | sed "s/^/$name /" >> $O/summary.txt
  echo >> $O/summary.txt
}
for r in 1 2 3; do
  run all DTP_NOP=1
  run none DTP_MODULE_RING=0 DTP_MODULE_FUSE_OPT=0 DTP_MODULE_LOSSLOG=0 DTP_MODULE_SYNC_FLUSH=1
done
