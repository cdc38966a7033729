#!/bin/bash
# One per node: wraps the experiment command with torchrun (G workers = G GPUs).
node_rank=$1       # this node's index, 0-based
nproc_per_node=$2  # workers per node (GPUs per node)
master_addr=$3
master_port=$4
tarball=$5
here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "${here}/../../common.sh"
rocm_env

nnodes="${SLURM_JOB_NUM_NODES:-1}"
launcher=(${TORCHRUN:-torchrun} --nproc_per_node "${nproc_per_node}" --nnodes "${nnodes}")
if (( nnodes == 1 )); then
  launcher+=(--master_addr 127.0.0.1 --master_port "${master_port}" --node_rank 0)
else
  launcher+=(--rdzv_id="${SLURM_JOB_ID}" --rdzv_backend=c10d --rdzv_endpoint="${master_addr}:${master_port}"
             --max_restarts="${DTP_MAX_RESTARTS:-3}")
fi
args="$(python_args_of "${cmd}")" || exit 1
IFS=' ' read -r -a args <<< "${args}"
make_job_tmpdir
unpack_tarball "${tarball}"
echo "COMMANDS GIVEN: ${launcher[*]} ${args[*]}"
exec "${launcher[@]}" "${args[@]}"
