#!/bin/bash
# Run ${cmd} inside a ROCm Singularity/Apptainer container (GPU access with --rocm).
tarball="$1"
workdir="${2:-workdir}"
here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "${here}/../common.sh"
rocm_env
[[ -n "${singularity_container}" ]] || { echo "singularity_container is not set" >&2; exit 1; }
make_job_tmpdir
SING="$(command -v apptainer || command -v singularity)"
if [[ -z "${SING}" ]]; then
  module load singularity 2> /dev/null || module load apptainer 2> /dev/null
  SING="$(command -v apptainer || command -v singularity)"
fi
[[ -n "${SING}" ]] || { echo "singularity/apptainer not found" >&2; exit 1; }
container="${SLURM_TMPDIR}/$(basename "${singularity_container}")"
rsync -a "${singularity_container}" "${container}"
mkdir -p "${SLURM_TMPDIR}"/{data,tmp,home,workdir_overlay}
unpack_tarball "${tarball}"
results="${scratch_dir}/${exp_name}"
mkdir -p "${results}"
export SINGULARITYENV_SLURM_JOB_ID="${SLURM_JOB_ID}" SINGULARITYENV_SLURM_PROCID="${SLURM_PROCID}"
export SINGULARITYENV_SLURM_LOCALID="${SLURM_LOCALID}" SINGULARITYENV_SLURM_NTASKS="${SLURM_NTASKS}"
export SINGULARITYENV_WANDB_API_KEY="${WANDB_API_KEY}" SINGULARITYENV_HSA_ENABLE_IPC_MODE_LEGACY=0
"${SING}" run --rocm --cleanenv --no-home --contain --writable-tmpfs \
  -B "${results}:/results" -B "${SLURM_TMPDIR}/data:/data" -B "${SLURM_TMPDIR}/tmp:/tmp" \
  -B "${source_dir}:/${workdir}" --pwd "/${workdir}" \
  "${container}" ${cmd}
