#!/bin/bash
# K=20 A/B: the 5 warm-up steps in 1 launch vs 5 one-step launches (fresh processes, interleaved)
set -o pipefail
n=$1; out=$2; shift 2
for i in $(seq 1 "$n"); do
  for w in 1 5; do
    DTP_BENCH_WARMUP_LAUNCHES=$w timeout -k 10 60 python bench.py "$@" 2>/dev/null | grep '^{' | \
      python -c "import sys,json; r=json.loads(sys.stdin.read()); r['warmup_launches']=$w; print(json.dumps(r))" >> "$out" || exit 1
  done
done
