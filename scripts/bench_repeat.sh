#!/bin/bash
# Repeat the driver's bench call in fresh processes (run-to-run spread of the K=20 number).
# usage: bash scripts/bench_repeat.sh N out.jsonl [bench args...]; stops at the first failure.
set -o pipefail
n=$1; out=$2; shift 2
for i in $(seq 1 "$n"); do
  timeout -k 10 60 python bench.py "$@" 2>/dev/null | grep '^{' >> "$out" || exit 1
done
