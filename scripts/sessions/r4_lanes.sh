#!/bin/bash
# round 4: the several-lanes step -- numerics, per-batch step time, phase stamps
export TMPDIR=/tmp
D=${1:-r4a}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "400|$D/lanes_tests|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lanes_gpu.py tests/test_trainer_fused_gpu.py" \
  "400|$D/split|python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_split_fused_gpu.py tests/test_layer_split.py" \
  "300|$D/bench_batch|for b in 64 128 256; do python bench.py --scaling weak --batch \$b; done" \
  "200|$D/bench_forced|for l in 1 2 4; do DTP_LANES=\$l python bench.py --scaling weak --batch 64; done" \
  "200|$D/stamps|python scripts/prof_stamps.py --lanes 4 --batch 64 && python scripts/prof_stamps.py --lanes 2 --batch 128" \
  "300|$D/share8|timeout 250 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 8 --share-gpu --steps 2000 --warmup 100 && timeout 250 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --share-gpu --steps 2000 --warmup 100"
