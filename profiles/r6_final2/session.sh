#!/bin/bash
# round 6 final validation: the whole GPU suite, smoke(), the driver's K=20 line, K=2000,
# the entrypoints (demo.py fused / module, the Lightning demo fused / module, the split
# demo), the share-GPU exchange rehearsal, a rocprofv3 kernel trace of the bench
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6y
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_k20.json 2>> $O/err.log || exit $?
done
timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_k2000.json 2>> $O/err.log || exit $?
timeout -k 10 300 python demo.py --iters 20000 --seed 0 --no_progress --log_dir /tmp/df > $O/demo_fused.log 2>&1 || exit $?
timeout -k 10 300 python demo.py --engine module --iters 5000 --seed 0 --dry_run --no_progress --log_dir /tmp/dm > $O/demo_module.log 2>&1 || exit $?
timeout -k 10 300 python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/lf > $O/lt_fused.log 2>&1 || exit $?
timeout -k 10 300 python demo_pytorch_lightning.py --gpus 1 --steps 6000 --seed 0 --no_progress --engine module --root_dir /tmp/lm > $O/lt_module.log 2>&1 || exit $?
timeout -k 10 300 python demo_one_model_multi_gpu.py --gpus_per_proc 2 --allow_shared_gpu --iters 20000 --seed 0 --dry_run --no_progress --log_dir /tmp/ds > $O/demo_split.log 2>&1 || exit $?
for W in 2 4 8; do
  timeout -k 10 200 python bench.py --gpus $W --share-gpu --steps 2000 --warmup 200 >> $O/share_w$W.json 2>> $O/err.log || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 2000 --warmup 200 > $O/rocprof.log 2>&1 || exit $?
