#!/bin/bash
# K=20 A/B of the CU-pinned stream: fresh bench processes, off/on interleaved.
# usage: bash scripts/ab_cumask.sh N out.jsonl [bench args...]
set -o pipefail
n=$1; out=$2; shift 2
for i in $(seq 1 "$n"); do
  for m in off on; do
    timeout -k 10 60 python bench.py --cu-mask $m "$@" 2>/dev/null | grep '^{' >> "$out" || exit 1
  done
done
