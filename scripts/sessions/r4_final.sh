#!/bin/bash
# round-4 end-of-session validation: GPU suite, smoke, driver-style bench lines, kernel trace of the K=20 call
export TMPDIR=/tmp
D=${1:-r4z}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "900|${D}/gpu_suite|python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests" \
  "180|${D}/smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "180|${D}/bench_k20|for i in 1 2 3; do python bench.py --steps 20 --warmup 5; done" \
  "180|${D}/bench_default|python bench.py" \
  "180|${D}/bench_bf16|python bench.py --precision bf16" \
  "200|${D}/rocprof_k20|timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${D}/prof -o k20 -- python3 bench.py --steps 20 --warmup 5"
