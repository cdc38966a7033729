#!/usr/bin/env python3
"""DDP demo: two ToyModels trained data-parallel, launched by torchrun or plain srun.

Same launch contract as the reference's demo.py:
* ``torchrun --nproc_per_node G ... demo.py --torchrun`` (env:// rendezvous), or
* ``srun ... python demo.py [--use_node_rank]`` with TASKS_PER_NODE, WORLD_SIZE,
  MASTER_ADDR, MASTER_PORT exported (tcp:// init from SLURM_PROCID/SLURM_LOCALID).
On MI355X the iteration runs as fused HIP kernels with the gradient all-reduce over
xGMI (or RCCL); ``--device cpu --backend gloo`` runs the same loop on CPUs.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from argument_parser import get_args  # noqa: E402
from distributed_training_pytorch_amd.engine import runner  # noqa: E402
from distributed_training_pytorch_amd.runtime.errors import record  # noqa: E402


@record
def main(argv=None):
    config = get_args(argv)
    if config.dry_run:
        os.environ["WANDB_MODE"] = "dryrun"
    if config.backend == "nccl" and config.num_workers > 0:
        # kept for CLI parity (demo.py:163-170); batches are gathered on the device, no loader workers
        import torch.multiprocessing as tmp

        tmp.set_sharing_strategy("file_system")
    env, device, rank, world = runner.setup(config)
    summary = runner.train(config, env, device, rank, world, group="base-demo")
    if rank == 0:
        print(f"[Process {rank}] summary: {summary}", flush=True)
    runner.teardown()
    return summary


if __name__ == "__main__":
    main()
