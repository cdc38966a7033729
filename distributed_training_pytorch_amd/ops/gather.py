"""Batch gather of the module paths: rows ``idx`` of a dataset's inputs X [n, dx] and
targets Y [n, dy] into two batch buffers in ONE launch (``csrc/loss.hip:
gather_rows2_kernel``) -- torch's form is one ``index_select`` per tensor, and inside a
replayed hipGraph every launch costs ~3.5-4 us whatever it does.  Out-of-range indices
are clamped on the device (never an out-of-bounds read); CPU / other dtypes take torch's
``index_select``."""
from __future__ import annotations

import torch

from .. import _native as nat


def gather_rows2(X: torch.Tensor, Y: torch.Tensor, idx: torch.Tensor, ox: torch.Tensor, oy: torch.Tensor) -> None:
    if (X.is_cuda and X.dim() == 2 and Y.dim() == 2 and X.dtype == Y.dtype == ox.dtype == oy.dtype == torch.float32
            and idx.dtype == torch.int64 and all(t.is_contiguous() for t in (X, Y, idx, ox, oy))
            and ox.shape == (idx.numel(), X.shape[1]) and oy.shape == (idx.numel(), Y.shape[1])
            and X.shape[0] == Y.shape[0] and idx.numel() > 0 and nat.native_enabled()):
        nat.check(nat.load().dtp_gather_rows2(nat.ptr(X), X.shape[1], nat.ptr(Y), Y.shape[1], nat.ptr(idx),
                                              idx.numel(), X.shape[0], nat.ptr(ox), nat.ptr(oy), nat.stream_ptr()),
                  "dtp_gather_rows2")
        return
    torch.index_select(X, 0, idx, out=ox)
    torch.index_select(Y, 0, idx, out=oy)
