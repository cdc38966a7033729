#!/bin/bash
# Lightning-style Trainer under srun (one task per GPU), RCCL then gloo:
#   salloc -N 2 --ntasks-per-node=8 --gres=gpu:8 ; bash interactive_job_cmds/salloc_lightning.sh
cd "$(dirname "${BASH_SOURCE[0]}")/.." || exit 1
source hpc_files/common.sh
rocm_env
export TASKS_PER_NODE=$(( SLURM_NTASKS / SLURM_NNODES ))
export WORLD_SIZE=${SLURM_NTASKS}
export MASTER_ADDR=$(hostname)
export MASTER_PORT=${MASTER_PORT:-8964}
STEPS=${STEPS:-200}
export TORCH_NCCL_BLOCKING_WAIT=1   # blocking collectives with a timeout (reference: NCCL_BLOCKING_WAIT=1)
PL_TORCH_DISTRIBUTED_BACKEND=nccl srun -n "${WORLD_SIZE}" -o demo_lightning_nccl_output.out \
  python demo_pytorch_lightning.py --gpus="${TASKS_PER_NODE}" --nnodes="${SLURM_NNODES}" --steps "${STEPS}" --no_progress
PL_TORCH_DISTRIBUTED_BACKEND=gloo srun -n "${WORLD_SIZE}" -o demo_lightning_gloo_output.out \
  python demo_pytorch_lightning.py --gpus="${TASKS_PER_NODE}" --nnodes="${SLURM_NNODES}" --steps "${STEPS}" --no_progress
