#!/bin/bash
# round 6: the driver's K=20 line on the final tree, another box, 8 fresh processes; smoke()
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6aj
mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_k20.json 2>> $O/err.log || exit $?
done
timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/bench_k2000.json 2>> $O/err.log || exit $?
