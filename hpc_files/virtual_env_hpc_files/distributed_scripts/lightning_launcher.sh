#!/bin/bash
# One per task (srun over ntasks-per-node=G): the Trainer reads SLURM_* itself.
nnodes=$1
nproc_per_node=$2
tarball=$3
here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "${here}/../../common.sh"
rocm_env
export PL_TORCH_DISTRIBUTED_BACKEND="${PL_TORCH_DISTRIBUTED_BACKEND:-nccl}"

args="$(python_args_of "${cmd}")" || exit 1
# drop any user-provided node/gpu counts and append the allocation's
args="$(sed -r -e 's/ ?--(num_nodes|nnodes|gpus)[= ][0-9]+//g' <<< " ${args}")"
IFS=' ' read -r -a args <<< "${args} --nnodes=${nnodes} --gpus=${nproc_per_node}"
make_job_tmpdir
unpack_tarball "${tarball}"
echo "COMMANDS GIVEN: python ${args[*]}"
exec ${PYTHON:-python} "${args[@]}"
