#!/bin/bash
# Remove node-local job directories left by crashed jobs (jobs remove their own
# ${SLURM_TMPDIR} on success only).  Run on a node: bash tmpdir_cleanup.sh [root]
root="${1:-${DTP_NODE_TMP:-${TMPDIR:-/tmp}}}"
shopt -s nullglob
for d in "${root}/${USER}_dtp_"*; do
  echo "removing ${d}"
  rm -rf "${d}"
done
