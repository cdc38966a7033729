#!/bin/bash
# Standard (single task) and sweep jobs: activate the venv, stage data, run ${cmd}.
tarball="$1"
here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "${here}/../common.sh"
rocm_env
[[ -n "${scratch_dir}" ]] || { echo "scratch_dir is not set (submit with job_submitter.sh)" >&2; exit 1; }
if ! command -v srun > /dev/null 2>&1 && [[ -d /opt/slurm/bin ]]; then
  PATH=/opt/slurm/bin:${PATH}
fi
make_job_tmpdir
[[ -f "${source_dir}/virtual_env/bin/activate" ]] && source "${source_dir}/virtual_env/bin/activate"
unpack_tarball "${tarball}"
cd "${source_dir}" || exit 1
IFS=' ' read -r -a cmd_arr <<< "${cmd}"
echo "COMMANDS GIVEN: ${cmd_arr[*]}"
"${cmd_arr[@]}"
status=$?
[[ -n "${DTP_NODE_TMP}" ]] && rm -rf "${SLURM_TMPDIR}"
exit ${status}
