#!/bin/bash
# Shared helpers sourced by the job scripts.

# GPUs (GCDs) visible on this node: SLURM/ROCm visibility variables first, then
# amd-smi / rocm-smi, then torch.
count_gpus() {
  local v
  for v in ROCR_VISIBLE_DEVICES HIP_VISIBLE_DEVICES CUDA_VISIBLE_DEVICES; do
    if [[ -n "${!v}" ]]; then
      awk -F, '{print NF}' <<< "${!v}"
      return
    fi
  done
  if command -v amd-smi > /dev/null 2>&1; then
    amd-smi list 2> /dev/null | grep -c '^GPU'
    return
  fi
  if command -v rocm-smi > /dev/null 2>&1; then
    rocm-smi --showid 2> /dev/null | grep -o 'GPU\[[0-9]*\]' | sort -u | wc -l
    return
  fi
  python -c 'import torch; print(torch.cuda.device_count())' 2> /dev/null || echo 0
}

# per-job node-local scratch (the reference used /scratch-ssd/$USER on one cluster)
make_job_tmpdir() {
  if [[ -n "${DTP_NODE_TMP}" ]]; then
    SLURM_TMPDIR="${DTP_NODE_TMP}/${USER}_dtp_${SLURM_JOB_ID}_${SLURM_ARRAY_TASK_ID:-0}"
  fi
  SLURM_TMPDIR="${SLURM_TMPDIR:-${TMPDIR:-/tmp}/${USER}_dtp_${SLURM_JOB_ID:-$$}}"
  mkdir -p "${SLURM_TMPDIR}"
  export SLURM_TMPDIR
}

# unpack the staged data tarball into ${SLURM_TMPDIR} (paths relative to scratch_dir)
unpack_tarball() {
  local tarball="$1"
  if [[ -n "${tarball}" ]]; then
    echo "Moving ${tarball} to local node"
    tar -xf "${tarball}" -C "${SLURM_TMPDIR}"
  fi
}

# the experiment command must be a python invocation; echo its arguments (without "python")
python_args_of() {
  local program
  program="$(cut -d ' ' -f1 <<< "$1")"
  if [[ ! "${program}" == python* ]]; then
    echo "Command must be a python execution" >&2
    return 1
  fi
  cut -s -d ' ' -f2- <<< "$1"
}

rocm_env() {
  export HSA_ENABLE_IPC_MODE_LEGACY=0        # dmabuf IPC for RCCL / xGMI peer mappings
  export TORCH_NCCL_ASYNC_ERROR_HANDLING=1   # abort on RCCL errors instead of hanging
  export NCCL_ASYNC_ERROR_HANDLING=1
  export OMP_NUM_THREADS="${OMP_NUM_THREADS:-1}"
}
