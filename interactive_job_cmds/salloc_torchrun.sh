#!/bin/bash
# Interactive smoke test of every DDP launch mode inside an allocation, e.g.
#   salloc -N 2 --ntasks-per-node=8 --gres=gpu:8 -t 1:00:00
#   bash interactive_job_cmds/salloc_torchrun.sh
# Each variant writes demo_<variant>_output.out.
cd "$(dirname "${BASH_SOURCE[0]}")/.." || exit 1
source hpc_files/common.sh
rocm_env
export WANDB_MODE="${WANDB_MODE:-dryrun}"
export WORLD_SIZE=${SLURM_NTASKS}
export TASKS_PER_NODE=$(( SLURM_NTASKS / SLURM_NNODES ))
export MASTER_ADDR=$(hostname)
export MASTER_PORT=${MASTER_PORT:-2345}
nodes=($(scontrol show hostname "${SLURM_NODELIST}"))
gpus_per_node=$(srun -N1 -n1 -w "${nodes[0]}" bash -c 'source hpc_files/common.sh; count_gpus')
ITERS=${ITERS:-200}
echo "nodes=${nodes[*]} tasks/node=${TASKS_PER_NODE} gpus/node=${gpus_per_node}"

echo "(a) srun per node, global rank = NODE_RANK * TASKS_PER_NODE + SLURM_LOCALID"
for i in "${!nodes[@]}"; do
  NODE_RANK=${i} srun -w "${nodes[i]}" -N1 -n"${TASKS_PER_NODE}" -o "demo_node_rank_output_${i}.out" \
    python demo.py --backend=nccl --use_node_rank --iters "${ITERS}" --no_progress &
done
wait

echo "(b) torchrun per node (c10d rendezvous)"
srun -N "${SLURM_NNODES}" --ntasks-per-node=1 -o demo_torchrun_output.out \
  torchrun --nnodes "${SLURM_NNODES}" --nproc_per_node "${gpus_per_node}" --rdzv_id="${SLURM_JOB_ID:-1}" \
  --rdzv_backend=c10d --rdzv_endpoint="${MASTER_ADDR}:${MASTER_PORT}" \
  demo.py --backend=nccl --torchrun --iters "${ITERS}" --no_progress

echo "(c) mpiexec: ranks from the MPI environment (mpi4py optional)"
if command -v mpiexec > /dev/null 2>&1; then
  export DTP_RENDEZVOUS_FILE="${PWD}/.rdzv_${SLURM_JOB_ID:-$$}"
  rm -f "${DTP_RENDEZVOUS_FILE}"
  mpiexec -n "${WORLD_SIZE}" python demo_assume_started_with_mpiexec.py --backend=nccl --iters "${ITERS}" \
    --no_progress > demo_mpiexec_output.out 2>&1
else
  echo "mpiexec not available; skipped" | tee demo_mpiexec_output.out
fi

echo "(d) srun with the gloo backend (SLURM_PROCID ranks)"
srun -o demo_gloo_output.out python demo.py --backend=gloo --iters "${ITERS}" --no_progress
