"""Checkpoint / resume (absent from the reference, which only creates a
``checkpoints/`` directory in job_submitter.sh:157-159).

Rank 0 writes ``{dir}/last.pt`` (and ``step_{t}.pt`` when keep>0) atomically
(tmp file + ``os.replace``) with everything needed to continue bit-exactly:
flat params, optimizer state, per-model step counters, host iteration,
sampler position (derived from the step), RNG states and the run config.
Every rank loads it on start (``--resume``) -- that is what makes
``torchrun --max_restarts`` meaningful.  Loading uses ``weights_only=True``.
"""
from __future__ import annotations

import os
from pathlib import Path

import torch
import torch.distributed as dist


def _to_plain(x):
    if isinstance(x, dict):
        return {k: _to_plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_to_plain(v) for v in x]
    if isinstance(x, torch.Tensor):
        return x.detach().cpu()
    return x


def save(state: dict, directory: str | os.PathLike, step: int, keep: int = 0, rank: int | None = None) -> Path | None:
    rank = (dist.get_rank() if dist.is_initialized() else 0) if rank is None else rank
    if rank != 0:
        return None
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    payload = _to_plain(dict(state))
    # the host iteration gets a key of its own: "step" belongs to the engines'
    # per-model optimizer step counters and must survive the round trip
    payload["iteration"] = int(step)
    payload["rng_cpu"] = torch.get_rng_state()
    tmp = d / f".last.pt.tmp.{os.getpid()}"
    torch.save(payload, tmp)
    final = d / "last.pt"
    os.replace(tmp, final)
    if keep > 0:
        snap = d / f"step_{step:09d}.pt"
        torch.save(payload, snap)
        snaps = sorted(d.glob("step_*.pt"))
        for old in snaps[:-keep]:
            old.unlink(missing_ok=True)
    return final


def load(directory: str | os.PathLike, map_location="cpu") -> dict | None:
    p = Path(directory) / "last.pt"
    if not p.exists():
        return None
    st = torch.load(p, map_location=map_location, weights_only=True)
    if "rng_cpu" in st:
        torch.set_rng_state(st["rng_cpu"])
    return st
