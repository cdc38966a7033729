#!/bin/bash
# round 6: the module engine's batch indices computed by the device sampler inside the
# replayed gather (no host index work per step or epoch) -- tests, then the steady state
# against the epoch ring (DTP_MODULE_RING=epoch) and the per-step index copy (=0)
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6ac
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_loss_op.py tests/test_entrypoints_gpu.py tests/test_module_path_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python demo.py --engine module --iters 10000 --seed 0 --dry_run --no_progress --log_dir /tmp/d_$name > $O/dm_$name.$r.log 2>&1 || exit $?
  grep -o "'steady_samples_per_s': [0-9.]*\|'final_loss': \[[^]]*\]" $O/dm_$name.$r.log | tr '\n' ' ' | sed "s/^/$name /" >> $O/summary.txt
  echo >> $O/summary.txt
}
for r in 1 2 3; do
  run sampler DTP_NOP=1
  run epoch DTP_MODULE_RING=epoch
  run copy DTP_MODULE_RING=0
done
