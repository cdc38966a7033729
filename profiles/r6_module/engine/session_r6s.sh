#!/bin/bash
# round 6: the module engine (demo.py --engine module): the ModelBank backwards fused with
# the flat Adam, the loss-log row written by the pair loss's launch, a cached backward seed
# and the device epoch ring (no index copy per step) -- tests, A/Bs, kernel trace
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_loss_op.py tests/test_module_path_gpu.py tests/test_entrypoints_gpu.py tests/test_graph_step_gpu.py tests/test_graph_xgmi_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 300 python demo.py --engine module --iters 5000 --seed 0 --dry_run --no_progress --log_dir /tmp/dm$r > $O/dm_new_$r.log 2>&1 || exit $?
  DTP_MODULE_RING=0 timeout -k 10 300 python demo.py --engine module --iters 5000 --seed 0 --dry_run --no_progress --log_dir /tmp/dn$r > $O/dm_noring_$r.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dm -o dm -- python3 demo.py --engine module --iters 3000 --seed 0 --dry_run --no_progress --log_dir /tmp/dmp > $O/dm_prof.log 2>&1 || exit $?
