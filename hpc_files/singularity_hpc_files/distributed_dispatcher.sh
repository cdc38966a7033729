#!/bin/bash
# Singularity variant: every task runs standard_job.sh inside the container; the
# launch pattern inside is the same as the virtualenv dispatcher (torchrun per node,
# lightning/mpi per task).
here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
srun bash "${here}/standard_job.sh" "$1" "$2"
