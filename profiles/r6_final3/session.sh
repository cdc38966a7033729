#!/bin/bash
# round 6, last validation of the final tree: the whole GPU suite, smoke(), the driver's
# K=20 line and K=2000, the module engine's steady state, the Lightning demo; then the
# K=20 call's wait variants (scripts/launch_floor.py)
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6ae
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_k20.json 2>> $O/err.log || exit $?
done
timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_k2000.json 2>> $O/err.log || exit $?
timeout -k 10 300 python demo.py --engine module --iters 10000 --seed 0 --dry_run --no_progress --log_dir /tmp/dm > $O/demo_module.log 2>&1 || exit $?
timeout -k 10 300 python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/lf > $O/lt_fused.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python scripts/launch_floor.py >> $O/launch_floor.json 2>> $O/err.log || exit $?
done
