#!/bin/bash
# round 4, session c: tests of the round's changes, K=20 pin A/B, scaling rehearsal lines
export TMPDIR=/tmp
D=${1:-r4c}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "500|$D/tests|python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_trainer_fused_gpu.py tests/test_split_fused_gpu.py tests/test_bench_gpu.py" \
  "300|$D/bench_k20|for i in 1 2 3 4 5 6; do DTP_BENCH_PIN=1 python bench.py --steps 20 --warmup 5; DTP_BENCH_PIN=0 python bench.py --steps 20 --warmup 5; done" \
  "100|$D/bench_default|python bench.py" \
  "200|$D/diag_streams|for m in per_device prio torch; do python scripts/diag_split_streams.py \$m; done" \
  "400|$D/share|for w in 2 4 8; do timeout 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node \$w --master-addr 127.0.0.1 --master-port 2962\$w bench.py --gpus \$w --share-gpu --steps 2000 --warmup 100 || exit 3; done" \
  "200|$D/stamps1|python scripts/prof_stamps.py"
