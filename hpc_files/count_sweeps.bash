#!/usr/bin/env bash
# Number of grid points of a wandb sweep file: product of the lengths of every
# parameter's `values` list.
set -euo pipefail
f="${1:-}"
if [[ -z "${f}" || ! -f "${f}" ]]; then
  echo "Either no argument was given or file does not exist" >&2; exit 1
fi
awk '
  /^parameters:/ { inp = 1; next }
  /^[^ \t#]/     { inp = 0 }
  inp && /values:/ { if (n) prod *= n; n = 0; invals = 1; next }
  inp && invals && /^[ \t]*-/ { n++; next }
  inp && /^[ \t]*[A-Za-z_]+:/ { invals = 0 }
  BEGIN { prod = 1; n = 0 }
  END { if (n) prod *= n; print prod }
' "${f}"
