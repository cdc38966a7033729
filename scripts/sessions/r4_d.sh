#!/bin/bash
# round 4, session d: split cost breakdown, exchange-wait diagnostic (slowest thread), share rehearsal
export TMPDIR=/tmp
D=${1:-r4d}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "300|$D/split_cost|python scripts/split_cost.py" \
  "300|$D/tests|python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_bench_gpu.py tests/test_graph_xgmi_gpu.py tests/test_xgmi_gpu.py" \
  "400|$D/share|for w in 2 4 8; do timeout 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node \$w --master-addr 127.0.0.1 --master-port 2963\$w bench.py --gpus \$w --share-gpu --steps 2000 --warmup 100 || exit 3; done"
