#!/bin/bash
# round 6: the host side of the K=20 call (train(20)'s enqueue time against the bare native
# call), two fresh processes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ah
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python scripts/launch_floor.py >> $O/launch_floor.json 2>> $O/err.log || exit $?
done
