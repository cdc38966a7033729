#!/usr/bin/env python3
"""DDP demo for MPI launches: ``mpiexec -n W python demo_assume_started_with_mpiexec.py``.

Rank, world size and local rank come from the MPI launcher's environment
(OpenMPI ``OMPI_COMM_WORLD_*``, MPICH/Intel ``PMI_*``/``MPI_LOCALRANKID``, PMIx,
MVAPICH), with ``TASKS_PER_NODE`` as the local-rank fallback like the reference
(``demo_assume_started_with_mpiexec.py:35-50``).  The master address is broadcast
with mpi4py when it is installed; otherwise it is taken from MASTER_ADDR/PORT or a
rendezvous file on a shared filesystem (``DTP_RENDEZVOUS_FILE``).  MPI only
bootstraps: gradients move over RCCL/xGMI.  The reference's reduction of a
discarded temporary (``:112-115``) is fixed: the logged global loss is correct.
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
    os.environ.setdefault("WANDB_MODE", "disabled")  # the reference's MPI demo does not use wandb
    if config.dry_run:
        os.environ["WANDB_MODE"] = "dryrun"
    env, device, rank, world = runner.setup(config, launcher="mpi")
    summary = runner.train(config, env, device, rank, world, group="mpi-demo")
    if rank == 0:
        print(f"[Process {rank}] summary: {summary}", flush=True)
    runner.teardown()
    return summary


if __name__ == "__main__":
    main()
