#!/bin/bash
# mpiexec over the allocation, one rank per GPU; ranks discover themselves from the
# MPI launcher's environment (demo_assume_started_with_mpiexec.py).  Without mpi4py
# the master address travels through a rendezvous file on the shared filesystem.
nnodes=$1
gpus_per_node=$2
tarball=$3
here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "${here}/../../common.sh"
rocm_env
np=$(( nnodes * gpus_per_node ))
export TASKS_PER_NODE="${gpus_per_node}"
export DTP_RENDEZVOUS_FILE="${DTP_RENDEZVOUS_FILE:-${scratch_dir}/.rdzv_${SLURM_JOB_ID:-$$}}"
rm -f "${DTP_RENDEZVOUS_FILE}"
args="$(python_args_of "${cmd}")" || exit 1
IFS=' ' read -r -a args <<< "${args}"
make_job_tmpdir
unpack_tarball "${tarball}"
echo "COMMANDS GIVEN: ${MPIEXEC:-mpiexec} -n ${np} python ${args[*]}"
exec ${MPIEXEC:-mpiexec} -n "${np}" -x TASKS_PER_NODE -x DTP_RENDEZVOUS_FILE -x HSA_ENABLE_IPC_MODE_LEGACY \
  ${PYTHON:-python} "${args[@]}"
