"""xGMI peer-mapped exchange buffers for the in-kernel one-shot all-reduce.

Each rank allocates a fine-grained, uncached receive buffer
(``hipExtMallocWithFlags(hipDeviceMallocUncached)``), exports its IPC handle,
and maps every peer's buffer into its address space (``hipIpcOpenMemHandle``,
peer access over xGMI).  The device pointer table is handed to the fused
train kernel (``MODE_XGMI_*``), whose granule protocol is documented in
``csrc/xgmi_core.h``.

Handle exchange rides the torch.distributed store of the default group
(``all_gather_object``), i.e. the same TCPStore rendezvous torchrun already set
up -- no MPI, no extra sockets.

The exchange is self-validating: :meth:`XgmiExchange.selftest` runs one tiny
fused step through the buffers and compares against an RCCL/gloo all-reduce;
callers fall back to RCCL when it fails (timeouts are bounded in-kernel).
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from .. import _native as nat


def slot_granules(P: int) -> int:
    return (P + 1 + 7) & ~7


class XgmiExchange:
    def __init__(self, n_models: int, P: int, device: torch.device, group=None):
        self.lib = nat.require(device)
        self.device = device
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.n_models = n_models
        self.P = P
        self.bytes = 2 * n_models * self.world * slot_granules(P) * 8
        self._own = ctypes.c_void_p()
        self._opened: list[int] = []
        torch.cuda.set_device(device)
        nat.check(self.lib.dtp_malloc_uncached(self.bytes, ctypes.byref(self._own)), "dtp_malloc_uncached")
        ptrs = [0] * self.world
        ptrs[self.rank] = self._own.value
        if self.world > 1:
            hs = self.lib.dtp_ipc_handle_size()
            buf = ctypes.create_string_buffer(hs)
            nat.check(self.lib.dtp_ipc_get_handle(self._own, buf), "dtp_ipc_get_handle")
            dev_index = device.index if device.index is not None else torch.cuda.current_device()
            mine = (bytes(buf.raw), dev_index, os.getpid())
            allh = [None] * self.world
            dist.all_gather_object(allh, mine, group=group)
            for r, (h, peer_dev, pid) in enumerate(allh):
                if r == self.rank:
                    continue
                if peer_dev != dev_index:
                    can = ctypes.c_int(0)
                    nat.check(self.lib.dtp_can_access_peer(dev_index, peer_dev, ctypes.byref(can)),
                              "dtp_can_access_peer")
                    if not can.value:
                        raise RuntimeError(f"GPU {dev_index} cannot access peer GPU {peer_dev} over xGMI")
                    nat.check(self.lib.dtp_enable_peer_access(peer_dev), "dtp_enable_peer_access")
                p = ctypes.c_void_p()
                hb = ctypes.create_string_buffer(h, hs)
                nat.check(self.lib.dtp_ipc_open_handle(hb, ctypes.byref(p)), "dtp_ipc_open_handle")
                self._opened.append(p.value)
                ptrs[r] = p.value
        self.peer_table = torch.tensor(ptrs, dtype=torch.int64, device=device)
        self.epoch = torch.zeros(n_models, dtype=torch.int32, device=device)
        self.status = torch.zeros(16, dtype=torch.int32, device=device)
        self.ptrs = ptrs

    def check_status(self):
        s = self.status[:2].tolist()
        if s[0]:
            raise RuntimeError(f"xGMI exchange timed out on rank {self.rank} at epoch {s[1]} (peer not responding)")

    def close(self):
        for p in self._opened:
            self.lib.dtp_ipc_close_handle(ctypes.c_void_p(p))
        self._opened = []
        if self._own.value:
            self.lib.dtp_free(self._own)
            self._own = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass
