#!/bin/bash
# round 6: where the host time of demo.py's module engine goes on this box (cProfile of the
# loop), and the launch / completion floor against the bench's K=20 call
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6z
mkdir -p $O
timeout -k 10 200 python scripts/launch_floor.py > $O/launch_floor.json 2> $O/err.log || exit $?
timeout -k 10 300 python demo.py --engine module --iters 5000 --seed 0 --dry_run --no_progress --log_dir /tmp/dm > $O/demo_module.log 2>&1 || exit $?
timeout -k 10 300 python -m cProfile -s tottime demo.py --engine module --iters 5000 --seed 0 --dry_run --no_progress --log_dir /tmp/dp > $O/demo_module_cprofile.txt 2>&1 || exit $?
