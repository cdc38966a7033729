#!/bin/bash
# Submit tmpdir_cleanup.sh to each node given on the command line:
#   bash submit_cleanup.sh node01 node02 ...
here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
for node in "$@"; do
  sbatch -w "${node}" -N1 -n1 --time=00:05:00 --job-name="dtp-cleanup-${node}" \
    ${DTP_PARTITION:+--partition=${DTP_PARTITION}} "${here}/tmpdir_cleanup.sh"
done
