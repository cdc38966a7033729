#!/bin/bash
# Runs on the batch host of a distributed job (submitted by job_submitter.sh).
#   torchrun : one srun per node, each running torchrun_launcher.sh (G workers per node)
#   lightning: one srun over all tasks (one task per GPU), lightning_launcher.sh
#   mpi      : mpiexec over all tasks (one rank per GPU), demo_assume_started_with_mpiexec.py style
tarball="$1"
here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "${here}/../common.sh"
rocm_env
gpus_per_node="$(count_gpus)"

cd "${source_dir}" || exit 1
[[ -f virtual_env/bin/activate ]] && source virtual_env/bin/activate
make_job_tmpdir

nodes=($(scontrol show hostname "${SLURM_NODELIST}"))
num_nodes=${#nodes[@]}
export MASTER_ADDR="${MASTER_ADDR:-$(hostname)}"
export MASTER_PORT="${MASTER_PORT:-2345}"
scripts_dir="${here}/distributed_scripts"
status=0
case "${which_distributed}" in
  torchrun)
    pids=()
    for (( i = 0; i < num_nodes; i++ )); do
      echo "launching node ${i} on ${nodes[i]} (master ${MASTER_ADDR}:${MASTER_PORT}, ${gpus_per_node} GPUs)"
      srun -w "${nodes[i]}" -N 1 -n 1 bash "${scripts_dir}/torchrun_launcher.sh" \
        "${i}" "${gpus_per_node}" "${MASTER_ADDR}" "${MASTER_PORT}" "${tarball}" &
      pids+=($!)
    done
    for p in "${pids[@]}"; do wait "${p}" || status=$?; done
    ;;
  lightning)
    srun bash "${scripts_dir}/lightning_launcher.sh" "${num_nodes}" "${gpus_per_node}" "${tarball}" || status=$?
    ;;
  mpi)
    bash "${scripts_dir}/mpi_launcher.sh" "${num_nodes}" "${gpus_per_node}" "${tarball}" || status=$?
    ;;
  *)
    echo "Distributed specification not supported: ${which_distributed}" >&2; exit 1 ;;
esac

echo "FINISHED DISTRIBUTED JOB (status ${status})"
echo "========================"
[[ -n "${DTP_NODE_TMP}" ]] && srun rm -rf "${SLURM_TMPDIR}"
exit ${status}
