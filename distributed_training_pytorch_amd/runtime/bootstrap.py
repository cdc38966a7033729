"""Rank discovery and process-group bootstrap for every launch mode of the reference.

* torchrun / torch.distributed.run  -> RANK, WORLD_SIZE, LOCAL_RANK, LOCAL_WORLD_SIZE,
  MASTER_ADDR/PORT, env:// init (``demo.py:25-34``)
* plain srun (SLURM)                -> SLURM_PROCID / SLURM_LOCALID, TASKS_PER_NODE,
  optional NODE_RANK*TASKS_PER_NODE+LOCALID (``--use_node_rank``), WORLD_SIZE,
  MASTER_ADDR/PORT, tcp:// init (``demo.py:35-49``)
* mpiexec / mpirun (OpenMPI, MPICH, Intel MPI, MVAPICH, PMIx) -> rank/size/local rank
  from the launcher's env vars; the master address comes from mpi4py (bcast, as
  ``demo_assume_started_with_mpiexec.py:35-50``) when importable, else from
  MASTER_ADDR or a shared rendezvous file -- MPI is bootstrap-only, the data plane
  is RCCL.
* PBS (``using_sockeye_arc_ubc.md``) runs mpiexec, i.e. the MPI path.
* nothing set -> single process.

Device binding: one process per GCD (local_rank), or ``gpus_per_proc`` consecutive
devices per process for the layer-split demo (the reference's
``(rank*2)%local_world_size`` mapping is a latent bug).
"""
from __future__ import annotations

import datetime
import os
import socket
import time
from dataclasses import dataclass, field
from pathlib import Path

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    node_rank: int = 0
    master_addr: str = "127.0.0.1"
    master_port: int = 29500
    launcher: str = "single"  # single | torchrun | slurm | mpi
    init_method: str = "env://"
    extra: dict = field(default_factory=dict)

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1 or self.launcher != "single"


def _int(env, *names, default=None):
    for n in names:
        v = env.get(n)
        if v not in (None, ""):
            return int(v)
    return default


def _slurm_tasks_per_node(env) -> int | None:
    v = env.get("TASKS_PER_NODE") or env.get("SLURM_NTASKS_PER_NODE")
    if v:
        return int(v)
    tpn = env.get("SLURM_TASKS_PER_NODE")  # e.g. "4(x2)" or "4,2"
    if tpn:
        return int(tpn.split("(")[0].split(",")[0])
    return None


def free_port() -> int:
    s = socket.socket()
    s.bind(("", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def detect(torchrun: bool | None = None, use_node_rank: bool = False, env=None,
           rendezvous_file: str | None = None) -> DistEnv:
    """Work out rank/world/local rank/master from the environment."""
    env = dict(os.environ if env is None else env)
    is_torchrun = "TORCHELASTIC_RUN_ID" in env or ("RANK" in env and "LOCAL_RANK" in env and "WORLD_SIZE" in env)
    if torchrun or (torchrun is None and is_torchrun):
        try:
            world = int(env["WORLD_SIZE"])
            lws = int(env.get("LOCAL_WORLD_SIZE", world))
        except (KeyError, ValueError) as e:
            raise RuntimeError("WORLD_SIZE environment variable is required and must be an integer.") from e
        rank = int(env.get("RANK", "0"))
        local = int(env["LOCAL_RANK"])
        return DistEnv(rank, world, local, lws, int(env.get("GROUP_RANK", env.get("NODE_RANK", rank // max(lws, 1)))),
                       env.get("MASTER_ADDR", "127.0.0.1"), int(env.get("MASTER_PORT", 29500)), "torchrun", "env://")

    if "SLURM_PROCID" in env and "OMPI_COMM_WORLD_RANK" not in env and "PMI_RANK" not in env:
        tpn = _slurm_tasks_per_node(env)
        local = _int(env, "SLURM_LOCALID", default=0)
        if tpn is None:
            tpn = _int(env, "SLURM_NTASKS", default=1)
        if use_node_rank:
            node = _int(env, "NODE_RANK", "SLURM_NODEID", default=0)
            rank = node * tpn + local
        else:
            rank = _int(env, "SLURM_PROCID")
            node = _int(env, "SLURM_NODEID", default=rank // max(tpn, 1))
        world = _int(env, "WORLD_SIZE", "SLURM_NTASKS", default=1)
        addr, port = env.get("MASTER_ADDR"), env.get("MASTER_PORT")
        if addr is None or port is None:
            raise ValueError("MASTER_ADDR and MASTER_PORT must be provided for the SLURM (tcp://) init")
        return DistEnv(rank, world, local, tpn, node, addr, int(port), "slurm", f"tcp://{addr}:{port}")

    mpi_rank = _int(env, "OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK", "MV2_COMM_WORLD_RANK")
    if mpi_rank is not None:
        world = _int(env, "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "MV2_COMM_WORLD_SIZE", "WORLD_SIZE", default=1)
        local = _int(env, "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "MV2_COMM_WORLD_LOCAL_RANK",
                     "PALS_LOCAL_RANKID")
        lws = _int(env, "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "MV2_COMM_WORLD_LOCAL_SIZE",
                   "TASKS_PER_NODE")
        if local is None:
            tpn = _int(env, "TASKS_PER_NODE", default=1)
            local = mpi_rank % tpn  # demo_assume_started_with_mpiexec.py:40-41
            lws = tpn
        addr, port = _mpi_master(env, mpi_rank, world, rendezvous_file)
        return DistEnv(mpi_rank, world, local, lws or 1, mpi_rank // max(lws or 1, 1), addr, port, "mpi", "env://")

    return DistEnv()


def _mpi_master(env, rank, world, rendezvous_file) -> tuple[str, int]:
    """Master address/port for an MPI-launched job: mpi4py bcast > env > rendezvous file."""
    try:
        from mpi4py import MPI  # noqa: F401  (optional; absent on the MI355X image)

        comm = MPI.COMM_WORLD
        host = socket.gethostbyname(socket.getfqdn()) if rank == 0 else None
        port = free_port() if rank == 0 else None
        return comm.bcast(host, root=0), int(comm.bcast(port, root=0))
    except ImportError:
        pass
    if env.get("MASTER_ADDR") and env.get("MASTER_PORT"):
        return env["MASTER_ADDR"], int(env["MASTER_PORT"])
    path = rendezvous_file or env.get("DTP_RENDEZVOUS_FILE")
    if not path:
        if world == 1:
            return "127.0.0.1", free_port()
        raise RuntimeError("MPI launch without mpi4py: set MASTER_ADDR/MASTER_PORT or DTP_RENDEZVOUS_FILE "
                           "(a path on a shared filesystem)")
    p = Path(path)
    if rank == 0:
        tmp = p.with_suffix(".tmp")
        tmp.write_text(f"{socket.gethostbyname(socket.getfqdn())} {free_port()}\n")
        os.replace(tmp, p)
    deadline = time.time() + 300
    while not p.exists():
        if time.time() > deadline:
            raise TimeoutError(f"rendezvous file {p} never appeared")
        time.sleep(0.1)
    host, port = p.read_text().split()
    return host, int(port)


def bind_device(env: DistEnv, device: str = "auto", gpus_per_proc: int = 1) -> torch.device:
    """Select this process's device (first of its gpus_per_proc devices)."""
    if device == "cpu" or (device == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    n = torch.cuda.device_count()
    first = env.local_rank * gpus_per_proc
    if first + gpus_per_proc > n:
        raise RuntimeError(f"local rank {env.local_rank} needs GPUs {first}..{first + gpus_per_proc - 1} "
                           f"but only {n} are visible (HIP_VISIBLE_DEVICES)")
    torch.cuda.set_device(first)
    return torch.device("cuda", first)


def init_process_group(env: DistEnv, backend: str, device: torch.device,
                       timeout: datetime.timedelta = datetime.timedelta(hours=1)) -> None:
    """init_process_group for the detected launch mode (no-op for a single process)."""
    if dist.is_initialized():
        return
    if backend == "mpi" and not dist.is_mpi_available():
        raise RuntimeError("backend 'mpi' needs a torch built with MPI (this ROCm build has none); use "
                           "--backend nccl (RCCL) -- MPI still bootstraps ranks through its env vars")
    if backend == "nccl" and device.type != "cuda":
        backend = "gloo"
    if env.launcher == "single":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        dist.init_process_group(backend, init_method="env://", rank=0, world_size=1, timeout=timeout)
        return
    os.environ["MASTER_ADDR"] = env.master_addr
    os.environ["MASTER_PORT"] = str(env.master_port)
    os.environ["RANK"] = str(env.rank)
    os.environ["WORLD_SIZE"] = str(env.world_size)
    kw = {}
    if backend == "nccl":
        kw["device_id"] = device
    if env.launcher == "torchrun" and os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true":
        # connect to the elastic agent's store with an explicit per-attempt prefix:
        # after a --max_restarts restart the default env:// path can pick up the
        # previous attempt's gloo/RCCL addresses from the agent store and hang
        attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
        store = dist.TCPStore(env.master_addr, env.master_port, is_master=False, timeout=timeout)
        store = dist.PrefixStore(f"dtp/attempt_{attempt}", store)
        dist.init_process_group(backend, store=store, rank=env.rank, world_size=env.world_size, timeout=timeout, **kw)
        return
    dist.init_process_group(backend, init_method=env.init_method, rank=env.rank, world_size=env.world_size,
                            timeout=timeout, **kw)


def configure_collective_env(async_error_handling: bool = True) -> None:
    """RCCL failure-handling knobs the reference sets in its launchers
    (NCCL_ASYNC_ERROR_HANDLING, torchrun_launcher.sh:8): abort instead of hanging."""
    if async_error_handling:
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
