#!/bin/bash
# round 5, round-end rehearsal of the driver: bench (K=2000, K=20), smoke, the GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5end
mkdir -p $O
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_default.json 2>> $O/err.log || exit $?
done
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_k20.json 2>> $O/err.log || exit $?
done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
