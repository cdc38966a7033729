#!/bin/bash
# sbatch front-end for the MI355X harness (counterpart of the reference's
# hpc_files/job_submitter.sh, rewritten for ROCm clusters).
#
#   bash job_submitter.sh -j distributed -W torchrun -g 8 -N 2 -e myexp
#
# Job types:  standard (1 node, 1 task) | distributed (-W torchrun|lightning|mpi) |
#             sweep (wandb agent job array).
# The command to run is read from an experiment configuration file (default
# experiment_configurations.txt, -C to override); newlines/backslashes are stripped.
# Differences from the reference, on purpose: ROCm GPU types and device counting,
# $USER instead of a hard-coded squeue user, -p honoured, the Singularity path
# reachable, arithmetic comparisons, -y/--yes for non-interactive submission and
# --print-only to show the sbatch line without submitting.
set -o pipefail

hpc_files_dir="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source_dir="$(dirname "${hpc_files_dir}")"
project_name="$(basename "${source_dir}")"
gpu_type=""
time="00-01:00:00"
cpus=2
gpus=0
job_type="standard"
num_nodes=1
mem="10G"
account="${DTP_ACCOUNT:-}"
partition="${DTP_PARTITION:-}"
re='^[0-9]+$'
exp_name=""
exp_configs_path="${hpc_files_dir}/experiment_configurations.txt"
singularity_container=""
work_dir=""
stuff_to_tmp=""
which_distributed=""
assume_yes=false
print_only=false
sweepid="${DTP_SWEEP_ID:-}"
n_sweeps="${DTP_N_SWEEPS:-}"

die() { echo "error: $*" >&2; exit 1; }

while [[ $# -gt 0 ]]; do
  case "$1" in
    -a|--account) account="$2"; shift 2 ;;
    -h|--help) cat "${hpc_files_dir}/.help_message.txt"; exit 0 ;;
    -g|--gpus)
      gpus="$2"; [[ $gpus =~ $re ]] && (( gpus > 0 )) || die "gpus must be an integer > 0"; shift 2 ;;
    -c|--cpus)
      cpus="$2"; [[ $cpus =~ $re ]] && (( cpus > 0 )) || die "cpus must be an integer > 0"; shift 2 ;;
    -W|--which-distributed)
      which_distributed="$2"
      [[ " torchrun lightning mpi " == *" ${which_distributed} "* ]] || die "supported distributed options: torchrun lightning mpi"
      shift 2 ;;
    -p|--partition) partition="$2"; shift 2 ;;
    -t|--time) time="$2"; shift 2 ;;
    -m|--mem)
      mem="$2"; mem_type="${mem##*[0-9]}"; mem_amount="${mem%%[a-zA-Z]*}"
      [[ " G M " == *" ${mem_type} "* ]] || die "supported memory units: G or M"
      [[ $mem_amount =~ $re ]] || die "amount of memory must be a non-negative integer"
      shift 2 ;;
    -G|--gpu-type)
      gpu_type="$2"
      [[ " mi355x mi350x mi325x mi300x mi250x " == *" ${gpu_type} "* ]] || die "supported gpu types: mi355x mi350x mi325x mi300x mi250x"
      shift 2 ;;
    -e|--exp-name) exp_name="$2"; shift 2 ;;
    -j|--job-type)
      job_type="$2"
      [[ " standard distributed sweep " == *" ${job_type} "* ]] || die "supported job types: standard distributed sweep"
      shift 2 ;;
    -N|-n|--nodes|--num-nodes)
      num_nodes="$2"; [[ $num_nodes =~ $re ]] && (( num_nodes > 0 )) || die "nodes must be an integer > 0"; shift 2 ;;
    -d|--data)
      shift
      while [[ $# -gt 0 && "$1" != -* ]]; do stuff_to_tmp="${stuff_to_tmp:+${stuff_to_tmp} }$1"; shift; done ;;
    -s|--singularity-container)
      singularity_container="$2"; [[ "$singularity_container" == *.sif ]] || die "singularity container must be a .sif file"
      [[ -z "${work_dir}" ]] && work_dir="workdir"
      shift 2 ;;
    -w|--workdir) work_dir="$2"; shift 2 ;;
    -C|--configs) exp_configs_path="$2"; shift 2 ;;
    -y|--yes) assume_yes=true; shift ;;
    --print-only) print_only=true; assume_yes=true; shift ;;
    *) die "unknown argument: $1" ;;
  esac
done

[[ -n "${SCRATCH}" ]] || die "SCRATCH variable not assigned"
[[ -f "${exp_configs_path}" ]] || die "experiment configuration file ${exp_configs_path} not found"
if [[ "${job_type}" == "distributed" && -z "${which_distributed}" ]]; then
  die "must specify the type of distributed job using [-W, --which-distributed]"
fi
scratch_dir="${SCRATCH}/${project_name}"
singularity_job=false
[[ -n "${singularity_container}" ]] && singularity_job=true

WANDB_CREDENTIALS_PATH="${WANDB_CREDENTIALS_PATH:-${HOME}/wandb_credentials.txt}"
WANDB_API_KEY="${WANDB_API_KEY:-}"
if [[ -z "${WANDB_API_KEY}" && -f "${WANDB_CREDENTIALS_PATH}" ]]; then
  WANDB_API_KEY="$(tr -d '\n' < "${WANDB_CREDENTIALS_PATH}")"
fi

mkdir -p "${scratch_dir}/${exp_name}/checkpoints" "${scratch_dir}/hpc_outputs"

# data staging: one tarball per distinct set of paths (relative to ${scratch_dir})
tarball=""
if [[ -n "${stuff_to_tmp}" ]]; then
  suffix="$(tr ' /' '__' <<< "${stuff_to_tmp}")"
  tarball="${scratch_dir}/tar_ball_${suffix}.tar"
  if [[ ! -f "${tarball}" ]]; then
    echo "Creating tarball ${tarball}"
    (cd "${scratch_dir}" && tar -cf "${tarball}" ${stuff_to_tmp}) || die "tar failed"
  fi
fi

if [[ "${singularity_job}" != true ]]; then
  if [[ ! -d "${source_dir}/virtual_env" && "${DTP_SKIP_VENV:-0}" != 1 ]]; then
    venv_cmd=(-W -o "${SCRATCH}/python_virtualenv_installer_output.out" --job-name="virtualenv-creator"
              --mem="10G" -n1 -N1)
    [[ -n "${partition}" ]] && venv_cmd+=(--partition="${partition}")
    [[ -n "${account}" ]] && venv_cmd+=(--account="${account}")
    echo "Submitting virtualenv installer job"
    if [[ "${print_only}" == true ]]; then
      echo "sbatch ${venv_cmd[*]} ${hpc_files_dir}/install_python_packages.sh"
    else
      (cd "${source_dir}" && sbatch "${venv_cmd[@]}" "${hpc_files_dir}/install_python_packages.sh") &
      venv_pid=$!
      reported=""
      while kill -0 "${venv_pid}" 2> /dev/null; do
        state="$(squeue -u "${USER}" -h -n virtualenv-creator -o '%i %t' 2> /dev/null | head -n1)"
        if [[ -n "${state}" && "${state}" != "${reported}" ]]; then
          echo "virtualenv job ${state% *}: ${state#* }"
          reported="${state}"
        fi
        sleep 2
      done
      wait "${venv_pid}" || die "failed to install the virtual environment"
      echo "Finished installing virtualenv"
    fi
  fi
  hpc_file_location="${hpc_files_dir}/virtual_env_hpc_files"
  args=("${tarball}")
else
  hpc_file_location="${hpc_files_dir}/singularity_hpc_files"
  args=("${tarball}" "${work_dir}")
fi

case "${job_type}" in
  sweep)
    echo "About to submit a wandb sweep: gpus=1, nodes=1"
    gpus=1; num_nodes=1; which_distributed=""
    if [[ -z "${sweepid}" ]]; then read -r -p 'Specify sweeper id: ' sweepid; fi
    if [[ -z "${n_sweeps}" ]]; then read -r -p 'Specify number of sweeps: ' n_sweeps; fi
    [[ ${n_sweeps} =~ $re ]] || die "number of sweeps must be an integer"
    hpc_file_location="${hpc_file_location}/standard_job.sh"
    sbatch_cmd=(--array "1-${n_sweeps}%${DTP_MAX_CONCURRENT_SWEEPS:-10}" --ntasks-per-node=1
                --job-name="sweep-${project_name}-${exp_name}"
                -o "${scratch_dir}/hpc_outputs/sweep_${exp_name}_%A_%a.out")
    ;;
  standard)
    echo "About to submit a standard job: nodes=1"
    num_nodes=1
    hpc_file_location="${hpc_file_location}/standard_job.sh"
    sbatch_cmd=(--ntasks-per-node=1 --job-name="standard-${project_name}-${exp_name}"
                -o "${scratch_dir}/hpc_outputs/standard_${exp_name}_%j.out")
    ;;
  distributed)
    echo "About to submit a distributed job of type \"${which_distributed}\""
    sbatch_cmd=(-o "${scratch_dir}/hpc_outputs/${which_distributed}_${exp_name}_%N_%j.out"
                --job-name="${which_distributed}_dist-${project_name}-${exp_name}")
    hpc_file_location="${hpc_file_location}/distributed_dispatcher.sh"
    if [[ "${which_distributed}" == "lightning" || "${which_distributed}" == "mpi" ]]; then
      sbatch_cmd+=(--ntasks-per-node="${gpus}")          # one task (process) per GPU
    else
      cpus=$(( cpus * (gpus > 0 ? gpus : 1) ))           # torchrun: one task per node spawning G workers
      sbatch_cmd+=(--ntasks-per-node=1)
    fi
    ;;
esac

sbatch_cmd+=(--nodes="${num_nodes}" --time="${time}" --mem="${mem}" --cpus-per-task="${cpus}")

cmd="$(tr -d '\n\r\\' < "${exp_configs_path}" | tr -s ' ')"
if [[ -n "${sweepid}" ]]; then
  cmd="$(sed -r 's#/[0-9a-zA-Z]+$#/'"${sweepid}"'#' <<< "${cmd}")"
  echo "Sweep command: ${cmd}"
fi
variables="scratch_dir=${scratch_dir},source_dir=${source_dir},exp_name=${exp_name},WANDB_API_KEY=${WANDB_API_KEY},cmd=${cmd},which_distributed=${which_distributed},singularity_container=${singularity_container},HSA_ENABLE_IPC_MODE_LEGACY=0"
[[ -n "${DTP_SLURM_TMPDIR}" ]] && variables="${variables},SLURM_TMPDIR=${DTP_SLURM_TMPDIR}"

if (( gpus > 0 )); then
  if [[ -z "${gpu_type}" ]]; then
    sbatch_cmd+=(--gres="gpu:${gpus}")
  else
    sbatch_cmd+=(--gres="gpu:${gpu_type}:${gpus}")
  fi
fi
[[ -n "${partition}" ]] && sbatch_cmd+=(--partition="${partition}")
[[ -n "${account}" ]] && sbatch_cmd+=(--account="${account}")
sbatch_cmd+=(--export="ALL,${variables}")

echo "The following sbatch options will be set:"
printf '  %s\n' "${sbatch_cmd[@]}"
if [[ "${assume_yes}" != true ]]; then
  read -r -p "Do you want to continue? [y/N] " yn
  [[ "${yn}" =~ ^[Yy] ]] || exit 0
fi
if [[ "${print_only}" == true ]]; then
  echo "sbatch ${sbatch_cmd[*]} ${hpc_file_location} ${args[*]}"
  exit 0
fi
sbatch "${sbatch_cmd[@]}" "${hpc_file_location}" "${args[@]}"
