#!/bin/bash
# Run GPU steps in sequence, each under its own time limit; stop at the first
# step that crashed / faulted / timed out (exit codes other than 0 and 1).
# usage: gpu_steps.sh "<seconds>|<name>|<command>" ...
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start )) s" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after [$name] rc=$rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
