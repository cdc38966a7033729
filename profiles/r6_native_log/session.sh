#!/bin/bash
# round 6: the fused engines' per-step loss logging formatted natively (csrc/host_log.hip)
# -- entrypoint tests, then the Lightning demo (fused engine, CSV every step) and demo.py
# (fused engine, JSONL every step) against the Python formatting, interleaved
set -o pipefail
export TMPDIR=/tmp WANDB_MODE=dryrun
O=gpurun_out/r6w
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_entrypoints_gpu.py tests/test_trainer_fused_gpu.py tests/test_logging_cpu.py tests/test_module_path_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/lt$r > $O/lt_native_$r.log 2>&1 || exit $?
  DTP_NATIVE_LOG=0 timeout -k 10 200 python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/lp$r > $O/lt_python_$r.log 2>&1 || exit $?
  timeout -k 10 200 python demo.py --iters 20000 --seed 0 --no_progress --log_dir /tmp/dn$r > $O/demo_native_$r.log 2>&1 || exit $?
  DTP_NATIVE_LOG=0 timeout -k 10 200 python demo.py --iters 20000 --seed 0 --no_progress --log_dir /tmp/dp$r > $O/demo_python_$r.log 2>&1 || exit $?
done
cmp /tmp/lt1/lightning_logs/version_0/metrics.csv /tmp/lp1/lightning_logs/version_0/metrics.csv > $O/cmp.txt 2>&1 && echo "metrics.csv identical" >> $O/cmp.txt
