#!/bin/bash
#PBS -l walltime=00:30:00,select=2:ncpus=8:ngpus=8:mpiprocs=8
#PBS -N dtp-mpiexec
#PBS -j oe
# PBS equivalent of the reference's Sockeye example (using_sockeye_arc_ubc.md):
# mpiexec starts one rank per GPU; ranks bootstrap from the MPI environment and a
# rendezvous file, gradients move over RCCL/xGMI.
cd "${PBS_O_WORKDIR:-$(dirname "$0")/..}" || exit 1
source hpc_files/common.sh
rocm_env
export TASKS_PER_NODE=8
np=$(wc -l < "${PBS_NODEFILE}")
export DTP_RENDEZVOUS_FILE="${PWD}/.rdzv_${PBS_JOBID:-$$}"
rm -f "${DTP_RENDEZVOUS_FILE}"
mpiexec -np "${np}" -x TASKS_PER_NODE -x DTP_RENDEZVOUS_FILE -x HSA_ENABLE_IPC_MODE_LEGACY \
  python demo_assume_started_with_mpiexec.py --backend=nccl
