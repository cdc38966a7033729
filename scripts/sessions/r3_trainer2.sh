#!/bin/bash
# fused Trainer after pipelining the loss readback: lightning tests + throughput (whole fit and steady)
export TMPDIR=/tmp
mkdir -p gpurun_out/tr2
bash scripts/gpu_steps.sh \
  "400|tr2/tests|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_entrypoints_gpu.py tests/test_bf16_gpu.py -k 'lightning or trainer'" \
  "120|tr2/fused|python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/ltf" \
  "120|tr2/fused_40k|python demo_pytorch_lightning.py --gpus 1 --steps 40000 --seed 0 --no_progress --root_dir /tmp/ltg" \
  "120|tr2/fused_bf16|python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/ltb --precision bf16"
