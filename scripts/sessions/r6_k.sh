#!/bin/bash
# round 6: the ownership A/B (r6_j.sh), then the full validation (r6_i.sh)
set -o pipefail
bash scripts/sessions/r6_j.sh || exit $?
bash scripts/sessions/r6_i.sh || exit $?
