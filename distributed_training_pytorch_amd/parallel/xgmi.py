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
    """8-byte granules per slot of the stand-alone all-reduce (XgmiAllReduce)."""
    return (P + 1 + 7) & ~7


class PeerBuffers:
    """One zeroed, uncached device buffer per rank, IPC-mapped into every rank.

    ``ptrs[r]`` is rank r's buffer as seen from this process; ``peer_table`` is
    the same list as a device int64 tensor (what the kernels index).  The handle
    exchange (``all_gather_object``) happens after every rank zeroed its buffer,
    so it doubles as the barrier that orders initialisation before first use.
    """

    def __init__(self, nbytes: int, device: torch.device, group=None):
        self.lib = nat.require(device)
        self.device = device
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.bytes = nbytes
        self._own = ctypes.c_void_p()
        self._opened: list[int] = []
        torch.cuda.set_device(device)
        nat.check(self.lib.dtp_malloc_uncached(nbytes, ctypes.byref(self._own)), "dtp_malloc_uncached")
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
        self.ptrs = ptrs
        self.peer_table = torch.tensor(ptrs, dtype=torch.int64, device=device)

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


class XgmiExchange:
    """Receive buffers of the fused train kernel's in-kernel exchange (MODE_XGMI_*)."""

    def __init__(self, n_models: int, P: int, device: torch.device, group=None):
        self.device = device
        self.n_models = n_models
        self.P = P
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        # the fused kernel's 16-byte-granule layout, sized by the library itself
        nbytes = nat.require(device).dtp_xgmi_fused_buffer_bytes(P, n_models, world)
        self.nbytes = int(nbytes)  # handed to every launch (DtpTrainArgs.xbuf_bytes), which checks it
        self.bufs = PeerBuffers(nbytes, device, group)
        self.lib = self.bufs.lib
        self.world, self.rank = self.bufs.world, self.bufs.rank
        self.peer_table = self.bufs.peer_table
        self.ptrs = self.bufs.ptrs
        self.epoch = torch.zeros(n_models, dtype=torch.int32, device=device)
        self.status = torch.zeros(16, dtype=torch.int32, device=device)

    def check_status(self):
        s = self.status[:2].tolist()
        if s[0]:
            raise RuntimeError(f"xGMI exchange timed out on rank {self.rank} at epoch {s[1]} (peer not responding)")

    def close(self):
        self.bufs.close()


class XgmiAllReduce:
    """Stand-alone one-shot all-reduce of small fp32 buffers over xGMI
    (``csrc/xgmi_allreduce.hip``): FlatDDP's path for buckets up to ``cap``
    floats on a single node (W <= 8).

    ``all_reduce_(t, scale)`` is asynchronous on the current stream.  The exchange
    epochs are device counters the kernel advances itself (one per workgroup), so a
    call captured in a hipGraph is a fresh exchange on every replay: the module
    engine and the Trainer replay their whole step, xGMI buckets included.
    ``check()`` reads the sticky timeout word (one host sync) -- call it at
    logging/checkpoint boundaries, not per step.
    """

    MAX_CAP = 1 << 16  # 64 Ki floats: <= 64 blocks, always co-resident with other work

    def __init__(self, cap: int, device: torch.device, group=None, timeout_us: int = 2_000_000):
        if cap > self.MAX_CAP:
            raise ValueError(f"xGMI all-reduce capacity {cap} > {self.MAX_CAP} floats; use RCCL for large buckets")
        self.cap = int(cap)
        self.device = device
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.world > 8:
            raise ValueError("the xGMI all-reduce serves one node (<= 8 ranks)")
        self.bufs = PeerBuffers(2 * self.world * self.cap * 8, device, group)
        self.lib = self.bufs.lib
        self.rank = self.bufs.rank
        self.status = torch.zeros(16, dtype=torch.int32, device=device)
        self.timeout_us = int(timeout_us)
        # per-workgroup exchange counters, local to this rank: every rank counts the
        # same sequence of calls from zero, so the k-th call carries epoch k everywhere
        self.epochs = torch.zeros(max(1, self.lib.dtp_xgmi_allreduce_epoch_slots(self.cap)), dtype=torch.int32,
                                  device=device)

    def all_reduce_(self, t: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.device:
            raise ValueError("xGMI all-reduce takes a contiguous fp32 tensor on this rank's GPU")
        n = t.numel()
        if n > self.cap:
            raise ValueError(f"{n} floats exceed the xGMI all-reduce capacity {self.cap}")
        nat.check(self.lib.dtp_xgmi_allreduce(nat.ptr(t), n, self.cap, nat.ptr(self.bufs.peer_table), self.world,
                                              self.rank, nat.ptr(self.epochs), float(scale), nat.ptr(self.status),
                                              self.timeout_us, nat.stream_ptr()), "dtp_xgmi_allreduce")
        return t

    def check(self):
        s = self.status[:2].tolist()
        if s[0]:
            raise RuntimeError(f"xGMI all-reduce timed out on rank {self.rank} at epoch {s[1]}")

    def close(self):
        self.bufs.close()


class DeviceBarrier:
    """All-rank barrier queued on the GPU stream: a one-float one-shot xGMI
    all-reduce (``csrc/xgmi_allreduce.hip``), i.e. one hop of xGMI latency instead
    of an RCCL collective.

    ``barrier()`` then ``torch.cuda.synchronize()`` returns only after every rank
    has queued its barrier -- and so finished everything queued before it: the
    same guarantee as ``dist.barrier`` + synchronize, at the cost of a kernel
    launch and one exchange.  If the xGMI buffers cannot be set up on every rank,
    every rank agrees (one 1-element all-reduce) and falls back to the
    process-group barrier.
    """

    def __init__(self, device: torch.device, group=None):
        from . import comm_util

        self.group = group
        self.device = device
        self._ar = None
        ok = True
        try:
            self._ar = XgmiAllReduce(1, device, group)
        except Exception:  # IPC / peer access unavailable on this rank
            ok = False
        flag = torch.tensor([0.0 if ok else 1.0])
        comm_util.all_reduce_(flag, group)
        if flag.item() != 0.0 and self._ar is not None:
            self._ar.close()
            self._ar = None
        self._tok = torch.zeros(1, dtype=torch.float32, device=device)

    @property
    def native(self) -> bool:
        return self._ar is not None

    def __call__(self):
        if self._ar is None:
            from . import comm_util

            comm_util.barrier(self.group)
        else:
            self._ar.all_reduce_(self._tok)

    def check(self):
        if self._ar is not None:
            self._ar.check()

    def close(self):
        if self._ar is not None:
            self._ar.close()
            self._ar = None
