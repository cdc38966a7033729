#!/bin/bash
# Layer-split demo: each process owns GPUS_PER_PROC GPUs (pipeline stages), DDP over processes.
#   salloc -N 1 --ntasks-per-node=4 --gres=gpu:8 ; bash interactive_job_cmds/salloc_one_model_multi_gpu_torchrun.sh
cd "$(dirname "${BASH_SOURCE[0]}")/.." || exit 1
source hpc_files/common.sh
rocm_env
GPUS_PER_PROC=${GPUS_PER_PROC:-2}
export TASKS_PER_NODE=$(( SLURM_NTASKS / SLURM_NNODES ))
export WORLD_SIZE=${SLURM_NTASKS}
export MASTER_ADDR=$(hostname)
export MASTER_PORT=${MASTER_PORT:-2346}
export TORCH_NCCL_BLOCKING_WAIT=1
echo "(a) plain srun, ranks from SLURM"
srun -n "${WORLD_SIZE}" -o demo_layer_split_srun_output.out \
  python demo_one_model_multi_gpu.py --gpus_per_proc "${GPUS_PER_PROC}" --iters 200 --no_progress
echo "(b) torchrun, GPipe micro-batches"
gpus_per_node=$(count_gpus)
srun -N "${SLURM_NNODES}" --ntasks-per-node=1 -o demo_layer_split_torchrun_output.out \
  torchrun --nnodes "${SLURM_NNODES}" --nproc_per_node $(( gpus_per_node / GPUS_PER_PROC )) \
  --rdzv_backend=c10d --rdzv_endpoint="${MASTER_ADDR}:${MASTER_PORT}" --rdzv_id="${SLURM_JOB_ID:-2}" \
  demo_one_model_multi_gpu.py --torchrun --gpus_per_proc "${GPUS_PER_PROC}" --microbatches 4 --iters 200 --no_progress
