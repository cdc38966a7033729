#!/bin/bash
# Trainer on the fused train-step engine: entrypoint tests, throughput fused vs module path
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
bash scripts/gpu_steps.sh \
  "400|tr/tests|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_entrypoints_gpu.py -k lightning" \
  "120|tr/fused|python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/ltf" \
  "120|tr/fused_bf16|python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/ltb --precision bf16" \
  "200|tr/module|python demo_pytorch_lightning.py --gpus 1 --steps 2000 --seed 0 --no_progress --root_dir /tmp/ltm --engine module"
