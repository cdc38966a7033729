"""Batch gather of the module paths: rows ``idx`` of a dataset's inputs X [n, dx] and
targets Y [n, dy] into two batch buffers in ONE launch (``csrc/loss.hip:
gather_rows2_kernel``) -- torch's form is one ``index_select`` per tensor, and inside a
replayed hipGraph every launch costs ~3.5-4 us whatever it does.  Out-of-range indices
are clamped on the device (never an out-of-bounds read); CPU / other dtypes take torch's
``index_select``.

``gather_rows2_ring`` reads the batch's indices from a device-resident epoch ring
``{cursor, indices of the epoch}`` and advances the cursor itself
(``gather_rows2_ring_kernel``), so a replayed step gathers the next batch with nothing
refreshed from the host between replays (the reference's DataLoader hands every batch
over from the host, ``/root/reference/demo_pytorch_lightning.py:61-63``)."""
from __future__ import annotations

import torch

from .. import _native as nat


def _native_ok(X, Y, ox, oy, n) -> bool:
    return (X.is_cuda and X.dim() == 2 and Y.dim() == 2 and X.dtype == Y.dtype == ox.dtype == oy.dtype == torch.float32
            and all(t.is_contiguous() for t in (X, Y, ox, oy)) and ox.shape == (n, X.shape[1])
            and oy.shape == (n, Y.shape[1]) and X.shape[0] == Y.shape[0] and n > 0 and nat.native_enabled())


def gather_rows2(X: torch.Tensor, Y: torch.Tensor, idx: torch.Tensor, ox: torch.Tensor, oy: torch.Tensor) -> None:
    if idx.dtype == torch.int64 and idx.is_contiguous() and _native_ok(X, Y, ox, oy, idx.numel()):
        nat.check(nat.load().dtp_gather_rows2(nat.ptr(X), X.shape[1], nat.ptr(Y), Y.shape[1], nat.ptr(idx),
                                              idx.numel(), X.shape[0], nat.ptr(ox), nat.ptr(oy), nat.stream_ptr()),
                  "dtp_gather_rows2")
        return
    torch.index_select(X, 0, idx, out=ox)
    torch.index_select(Y, 0, idx, out=oy)


def ring_gather_ok(X: torch.Tensor, Y: torch.Tensor, batch: int) -> bool:
    """Whether ``gather_rows2_ring`` runs its one-launch device form for batches of up to
    ``batch`` rows (a GPU, fp32 2-D data, one workgroup's worth of elements)."""
    return (X.is_cuda and X.dim() == 2 and Y.dim() == 2 and X.dtype == Y.dtype == torch.float32
            and nat.native_enabled() and batch * (X.shape[1] + Y.shape[1]) <= nat.load().dtp_gather_ring_max_elems())


def gather_rows2_ring(X: torch.Tensor, Y: torch.Tensor, ring: torch.Tensor, batch: int, steps: int,
                      ox: torch.Tensor, oy: torch.Tensor) -> None:
    """Gather batch ``ring[0] mod steps`` (rows ``ring[1 + b*batch : ...]``, as many as
    ``ox`` has) into ``ox`` / ``oy`` and advance ``ring[0]`` -- on the device, in one
    launch.  CPU: the same with torch ops (the cursor read on the host)."""
    n = ox.shape[0]
    if ring.is_cuda and ring.dtype == torch.int64 and ring.is_contiguous() and _native_ok(X, Y, ox, oy, n):
        nat.check(nat.load().dtp_gather_rows2_ring(nat.ptr(X), X.shape[1], nat.ptr(Y), Y.shape[1], nat.ptr(ring),
                                                   batch, steps, n, X.shape[0], nat.ptr(ox), nat.ptr(oy),
                                                   nat.stream_ptr()), "dtp_gather_rows2_ring")
        return
    b = int(ring[0]) % steps
    idx = ring[1 + b * batch:1 + b * batch + n].clamp(0, X.shape[0] - 1)
    torch.index_select(X, 0, idx, out=ox)
    torch.index_select(Y, 0, idx, out=oy)
    ring[0] += 1


def gather_rows2_sampler(X: torch.Tensor, Y: torch.Tensor, cfg, cursor: torch.Tensor, ox: torch.Tensor,
                         oy: torch.Tensor) -> None:
    """Gather the batch of step ``cursor[0]`` as the engine's sampler orders it (``cfg``: a
    ``SamplerCfg``, pointed at a device permutation ring for DistributedSampler's exact
    order) into ``ox`` / ``oy`` and advance ``cursor[0]`` -- indices and gather in one
    launch on the device (``gather_rows2_sampler_kernel``); no host index work per step or
    epoch.  GPU only (the engines call it where ``ring_gather_ok`` holds)."""
    n = ox.shape[0]
    if not (cursor.is_cuda and cursor.dtype == torch.int64 and _native_ok(X, Y, ox, oy, n)):
        raise RuntimeError("gather_rows2_sampler: fp32 CUDA data, an int64 CUDA cursor and the native library")
    import ctypes

    nat.check(nat.load().dtp_gather_rows2_sampler(nat.ptr(X), X.shape[1], nat.ptr(Y), Y.shape[1], ctypes.byref(cfg),
                                                  nat.ptr(cursor), n, X.shape[0], nat.ptr(ox), nat.ptr(oy),
                                                  nat.stream_ptr()), "dtp_gather_rows2_sampler")
