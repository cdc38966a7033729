"""Distributed sampling.

Two interchangeable index sources with the semantics of
``torch.utils.data.DistributedSampler`` + ``DataLoader(batch_size, drop_last=False)``
as the reference uses them (``demo.py:139-154``):

* :class:`SamplerGeometry` / :func:`feistel_permute` -- the *device* sampler.  A
  keyed Feistel permutation evaluated per index inside the fused train kernel
  (``csrc/sampler.h``), so graph replays and persistent multi-step kernels draw
  their own batches without a host round trip.  This module is the bit-exact
  Python twin used by the tests.
* :func:`torch_distributed_indices` -- the exact torch order (``randperm`` with
  ``seed + epoch``), uploaded per step (``SAMPLER_EXPLICIT``) when bitwise parity
  with the reference's sample order is wanted.
"""
from __future__ import annotations

import atexit
import math
import weakref
from dataclasses import dataclass, field

import numpy as np
import torch

M32 = 0xFFFFFFFF

SAMPLER_EXPLICIT = 0
SAMPLER_DIST_SHUFFLE = 1
SAMPLER_SEQUENTIAL = 2
SAMPLER_DIST_NOSHUFFLE = 3


def hash32(x: int) -> int:
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


def round_key(seed: int, epoch: int, r: int) -> int:
    lo, hi = seed & M32, (seed >> 32) & M32
    return hash32(lo ^ hash32((hi + epoch * 0x9E3779B9 + r * 0x85EBCA6B) & M32))


def epoch_keys(seed: int, epoch: int) -> list[int]:
    return [round_key(seed, epoch, r) for r in range(4)]


def feistel_permute(q: int, n: int, bits: int, keys: list[int]) -> int:
    """Bijection on [0, 2**bits) (4 rounds of lo ^= F(hi); rotate), cycle-walked into [0, n)."""
    r = bits >> 1 if bits > 1 else 1
    rmask = (1 << r) - 1
    dmask = (1 << bits) - 1
    while True:
        for i in range(4):
            hi = q >> r
            lo = (q & rmask) ^ (hash32(hi ^ keys[i]) & rmask)
            q = ((lo << (bits - r)) | hi) & dmask
        if q < n:
            return q


def _hash32_np(x: np.ndarray) -> np.ndarray:
    """hash32 over a uint32 array (numpy uint32 products wrap mod 2**32, like the device)."""
    x = x ^ (x >> 16)
    x = x * np.uint32(0x7FEB352D)
    x = x ^ (x >> 15)
    x = x * np.uint32(0x846CA68B)
    return x ^ (x >> 16)


def feistel_permute_array(q: np.ndarray, n: int, bits: int, keys: list[int]) -> np.ndarray:
    """:func:`feistel_permute` of every element of ``q`` at once (same cycle walk)."""
    r = bits >> 1 if bits > 1 else 1
    rmask = np.uint32((1 << r) - 1)
    dmask = np.uint32((1 << bits) - 1)
    ks = [np.uint32(k & M32) for k in keys]
    cur = np.asarray(q, dtype=np.uint32)
    out = np.empty(cur.shape, dtype=np.int64)
    todo = np.arange(cur.size)
    while todo.size:
        for i in range(4):
            hi = cur >> np.uint32(r)
            lo = (cur & rmask) ^ (_hash32_np(hi ^ ks[i]) & rmask)
            cur = ((lo << np.uint32(bits - r)) | hi) & dmask
        ok = cur < n
        out[todo[ok]] = cur[ok]
        todo, cur = todo[~ok], cur[~ok]
    return out


def bits_for(n: int) -> int:
    return max(1, math.ceil(math.log2(max(n, 2))))


@dataclass
class SamplerGeometry:
    """Per-rank epoch/batch geometry shared with the device sampler (SamplerCfg)."""

    n: int
    world: int = 1
    rank: int = 0
    batch: int = 256
    shuffle: bool = True
    distributed: bool = True
    seed: int = 0
    _epoch_cache: tuple = field(default=(-1, None), init=False, repr=False, compare=False)

    @property
    def mode(self) -> int:
        if not self.distributed:
            return SAMPLER_SEQUENTIAL
        return SAMPLER_DIST_SHUFFLE if self.shuffle else SAMPLER_DIST_NOSHUFFLE

    @property
    def num_samples(self) -> int:
        if not self.distributed:
            return self.n
        return math.ceil(self.n / self.world)

    @property
    def steps_per_epoch(self) -> int:
        return math.ceil(self.num_samples / self.batch)

    @property
    def bits(self) -> int:
        return bits_for(self.n)

    def batch_pos(self, t: int) -> tuple[int, int, int]:
        epoch, bi = divmod(t, self.steps_per_epoch)
        start = bi * self.batch
        return epoch, start, min(self.batch, self.num_samples - start)

    def batch_size_at(self, t: int) -> int:
        return self.batch_pos(t)[2]

    def epoch_indices(self, epoch: int) -> np.ndarray:
        """This rank's whole epoch in device-sampler order (int64 array of num_samples),
        computed vectorised once per epoch (the last epoch is cached)."""
        if self._epoch_cache[0] == epoch:
            return self._epoch_cache[1]
        j = np.arange(self.num_samples, dtype=np.int64)
        if self.mode == SAMPLER_SEQUENTIAL:
            idx = j
        else:
            q = (self.rank + j * self.world) % self.n  # padded list (padding repeats from the start)
            idx = feistel_permute_array(q, self.n, self.bits, epoch_keys(self.seed, epoch)) \
                if self.mode == SAMPLER_DIST_SHUFFLE else q
        self._epoch_cache = (epoch, idx)
        return idx

    def indices(self, t: int) -> list[int]:
        """Dataset indices of global step t on this rank (device-sampler order)."""
        epoch, start, size = self.batch_pos(t)
        return self.epoch_indices(epoch)[start:start + size].tolist()

    def to_native(self):
        from .._native import SamplerCfg

        return SamplerCfg(self.mode, self.n, self.world, self.rank, self.batch, self.num_samples,
                          self.steps_per_epoch, self.bits, self.seed & 0xFFFFFFFFFFFFFFFF)


def torch_distributed_indices(n: int, world: int, rank: int, epoch: int, seed: int = 0,
                              shuffle: bool = True) -> list[int]:
    """Exactly what torch.utils.data.DistributedSampler yields for this epoch."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        indices = torch.randperm(n, generator=g).tolist()
    else:
        indices = list(range(n))
    total = math.ceil(n / world) * world
    pad = total - len(indices)
    if pad <= len(indices):
        indices += indices[:pad]
    else:
        indices += (indices * math.ceil(pad / len(indices)))[:pad]
    return indices[rank:total:world]


class EpochIndexStream:
    """Host-side exact-torch index stream: batches of DistributedSampler order."""

    def __init__(self, geom: SamplerGeometry):
        self.geom = geom
        self._epoch = -1
        self._idx: list[int] = []

    def epoch_list(self, epoch: int) -> list[int]:
        if epoch != self._epoch:
            g = self.geom
            if g.distributed:
                self._idx = torch_distributed_indices(g.n, g.world, g.rank, epoch, g.seed, g.shuffle)
            else:
                self._idx = list(range(g.n))
            self._epoch = epoch
        return self._idx

    def indices(self, t: int) -> list[int]:
        epoch, start, size = self.geom.batch_pos(t)
        return self.epoch_list(epoch)[start:start + size]


class BatchIndexer:
    """Per-step batch indices as a tensor on ``device``, for the engines that gather
    batches with ``index_select`` (module engine, layer split).

    * device sampler on a GPU: ``block`` steps of indices at a time straight into a
      device buffer by the native sampler kernel (``csrc/sampler.h``,
      ``dtp_sampler_indices``): no host index math and no host-to-device copy per
      step, stream-ordered with the steps that read them;
    * exact torch order (``exact_torch``) with shuffling on a GPU: the epoch
      permutations come from a device ``PermutationRing`` (torch's randperm order, filled
      by the native generator in blocks of epochs ahead of use); an epoch's per-rank list
      is ONE device gather of the padded positions ``rank + k * world`` -- no host
      permutation, list building or copy per epoch (it was ~50 us per step of the module
      engine at 2 steps per epoch);
    * otherwise (CPU, or unshuffled exact order): one vectorised epoch on the host,
      uploaded once per epoch (pinned, asynchronous).
    A returned tensor is a view that stays valid until ``block`` steps later.
    """

    def __init__(self, geom: SamplerGeometry, device: torch.device, exact_torch: bool = False, block: int = 64):
        self.geom = geom
        self.device = torch.device(device)
        self.exact = exact_torch
        self.block = max(1, int(block))
        self._native = None
        self._b0 = None
        self._buf = None
        self._epoch = -1
        self._ep_idx = None
        self._stream = EpochIndexStream(geom) if exact_torch else None
        self._ring = None
        if self.device.type == "cuda" and exact_torch and geom.distributed and geom.shuffle:
            self._ring = PermutationRing(geom, self.device, kind="torch")
            k = torch.arange(geom.num_samples, dtype=torch.int64)
            # DistributedSampler: the permutation padded by repeating from its start, then [rank::world]
            self._q = ((geom.rank + k * geom.world) % geom.n).to(self.device)
        if self.device.type == "cuda" and not exact_torch:
            from .. import _native as nat

            if nat.native_enabled():
                self._native = nat.require(self.device)
                self._cfg = geom.to_native()
                self._buf = torch.empty(self.block, geom.batch, dtype=torch.int32, device=self.device)

    def permutation_ring(self):
        """The device ``PermutationRing`` this indexer reads (DistributedSampler's exact
        shuffled order on a GPU), or None."""
        return self._ring

    def needs_ring(self) -> bool:
        """Whether the order needs a permutation table the native sampler cannot compute
        itself: torch's exact shuffled order (the keyed Feistel order and the unshuffled
        orders are computed on the device from the step number)."""
        return self.exact and self.geom.distributed and self.geom.shuffle

    def can_fill_epoch(self) -> bool:
        """Whether ``epoch_into`` is available (the device permutation ring or the host
        epoch list; not the native per-step sampler's blocks)."""
        return self._native is None

    def epoch_into(self, epoch: int, out: torch.Tensor) -> None:
        """Epoch ``epoch``'s per-rank indices (``num_samples`` int64) into ``out`` on the
        current stream -- the module engine's device epoch ring, which its replayed gather
        reads with a cursor (``ops.gather.gather_rows2_ring``)."""
        if self._ring is not None:
            self._ring.ensure(epoch, epoch)
            perm = self._ring.table[epoch & (self._ring.E - 1)]
            out.copy_(perm.index_select(0, self._q))
            return
        if self.exact:
            host = torch.tensor(self._stream.epoch_list(epoch), dtype=torch.int64)
        else:
            host = torch.from_numpy(self.geom.epoch_indices(epoch))
        if out.is_cuda:
            host = host.pin_memory()
        out.copy_(host, non_blocking=True)

    def __call__(self, t: int) -> torch.Tensor:
        epoch, start, size = self.geom.batch_pos(t)
        if self._native is not None:
            if self._b0 is None or not (self._b0 <= t < self._b0 + self.block):
                import ctypes

                from .. import _native as nat

                nat.check(self._native.dtp_sampler_indices(ctypes.byref(self._cfg), t, self.block,
                                                           nat.ptr(self._buf), nat.stream_ptr()),
                          "dtp_sampler_indices")
                self._b0 = t
            return self._buf[t - self._b0, :size]
        if self._ring is not None:
            if epoch != self._epoch:
                self._ring.ensure(epoch, epoch)  # stream-ordered refill when the ring runs out
                perm = self._ring.table[epoch & (self._ring.E - 1)]
                self._ep_idx = perm.index_select(0, self._q).long()
                self._epoch = epoch
            return self._ep_idx[start:start + size]
        if epoch != self._epoch:
            if self.exact:
                host = torch.tensor(self._stream.epoch_list(epoch), dtype=torch.int64)
            else:
                host = torch.from_numpy(self.geom.epoch_indices(epoch))
            if self.device.type == "cuda":
                host = host.pin_memory()
            self._ep_idx = host.to(self.device, non_blocking=True)
            self._epoch = epoch
        return self._ep_idx[start:start + size]


def randperm_torch(n: int, seed: int) -> list[int]:
    """``torch.randperm(n, generator=torch.Generator().manual_seed(seed))`` (CPU): the
    permutation DistributedSampler draws per epoch (with seed + epoch)."""
    g = torch.Generator()
    g.manual_seed(seed)
    return torch.randperm(n, generator=g).tolist()


_live_rings: "weakref.WeakSet" = weakref.WeakSet()  # rings with a generator thread started


@atexit.register
def _join_ring_threads() -> None:
    for r in list(_live_rings):
        r.close()


class PermutationRing:
    """Device ring of upcoming epoch permutations for the SAMPLER_TABLE sampler.

    Slot ``e & (epochs-1)`` holds epoch e's permutation of [0, n): torch's exact
    DistributedSampler order (``kind="torch"``: ``randperm(n)`` seeded with seed+epoch,
    generated by the native MT19937 replica ``csrc/randperm.hip`` on host threads) or
    the keyed Feistel permutation of the in-kernel device sampler (``kind="feistel"``), or
    the identity for the unshuffled orders (``kind="identity"``: one slot every epoch reads).
    The fused train kernel reads a lane's dataset index from the ring a step ahead,
    so the reference's exact sample order costs no host work per step.

    ``ensure(e_lo, e_hi)`` makes epochs [e_lo, e_hi] resident before a launch that
    reads them (one stream-ordered H2D copy of the missing epochs); a background thread
    keeps the next block generated in pinned memory, so long runs refill from a ready
    buffer.  The constructor fills the whole ring: a short run never refills."""

    def __init__(self, geom: SamplerGeometry, device: torch.device, kind: str = "torch", epochs: int | None = None,
                 budget_ints: int = 1 << 24):
        import threading

        if kind not in ("torch", "feistel", "identity"):
            raise ValueError(f"permutation kind {kind!r}: torch, feistel or identity")
        self.geom = geom
        self.n = geom.n
        self.kind = kind
        self.device = torch.device(device)
        if kind == "identity":
            # the unshuffled orders (DistributedSampler(shuffle=False), or one rank reading the
            # dataset in order) as one identity "permutation" every epoch shares: the fused
            # step's FAST sampler path then serves them too (it reads a SAMPLER_TABLE ring)
            epochs = 1
        elif epochs is None:
            epochs = max(2, min(8192, budget_ints // max(self.n, 1)))
        self.E = 1 << (int(epochs).bit_length() - 1)  # power of two
        self.table = torch.empty(self.E, self.n, dtype=torch.int32, device=self.device)
        self.lo, self.hi = 0, -1  # resident epochs [lo, hi]
        self._lock = threading.Lock()
        self._ahead = None  # (e0, count, pinned host tensor) of a prefetched block
        self._thread = None
        self._keep = []  # pinned buffers of in-flight copies
        self._write(0, self._generate(0, self.E))

    # ---------------------------------------------------------------- generation
    def _generate(self, e0: int, count: int) -> torch.Tensor:
        host = torch.empty(count, self.n, dtype=torch.int32, pin_memory=self.device.type == "cuda")
        if self.kind == "identity":
            host.copy_(torch.arange(self.n, dtype=torch.int32).expand(count, self.n))
        elif self.kind == "torch":
            self._fill_torch(e0, count, host)
        else:
            for k in range(count):
                keys = epoch_keys(self.geom.seed, e0 + k)
                host[k] = torch.from_numpy(
                    feistel_permute_array(np.arange(self.n), self.n, self.geom.bits, keys).astype(np.int32))
        return host

    def _fill_torch(self, e0: int, count: int, host: torch.Tensor) -> None:
        try:
            from .. import _native as nat

            lib = nat.load()
        except Exception:  # no native library (CPU-only checkouts): torch's own generator
            lib = None
        if lib is not None:
            import os

            threads = min(16, os.cpu_count() or 1)  # the box's CPU share per GPU
            nat.check(lib.dtp_randperm_fill(self.geom.seed & 0xFFFFFFFFFFFFFFFF, self.n, e0, count,
                                            host.data_ptr(), threads), "dtp_randperm_fill")
            return
        for k in range(count):
            host[k] = torch.tensor(randperm_torch(self.n, self.geom.seed + e0 + k), dtype=torch.int32)

    def _prefetch(self, e0: int, count: int) -> None:
        import threading

        def work():
            blk = self._generate(e0, count)
            with self._lock:
                self._ahead = (e0, count, blk)

        self._thread = threading.Thread(target=work, daemon=True)
        _live_rings.add(self)
        self._thread.start()

    def close(self) -> None:
        """Wait for the background generator (it may be inside the native randperm): a
        daemon thread still running native code when the interpreter exits is killed
        mid-call while the library unloads.  Idempotent; also run at exit."""
        t, self._thread = self._thread, None
        if t is not None:
            t.join()
        _live_rings.discard(self)

    # ---------------------------------------------------------------- residency
    def _write(self, e0: int, host: torch.Tensor) -> None:
        """Copy epochs [e0, e0 + len(host)) into their slots (stream-ordered)."""
        count = host.shape[0]
        s0 = e0 & (self.E - 1)
        first = min(count, self.E - s0)
        self.table[s0:s0 + first].copy_(host[:first], non_blocking=True)
        if first < count:
            self.table[:count - first].copy_(host[first:], non_blocking=True)
        self._keep = [host]
        self.hi = max(self.hi, e0 + count - 1)
        self.lo = max(self.lo, self.hi - self.E + 1)

    def needs_write(self, e_lo: int, e_hi: int) -> bool:
        """Would :meth:`ensure` copy into the table (and so overwrite slots)?"""
        return e_lo < self.lo or e_hi > self.hi

    def ensure(self, e_lo: int, e_hi: int) -> None:
        if self.kind == "identity":  # every epoch is the one resident table
            return
        if e_hi - e_lo + 1 > self.E:
            raise ValueError(f"a launch spanning {e_hi - e_lo + 1} epochs exceeds the {self.E}-epoch ring: "
                             "launch fewer steps at a time")
        if e_lo < self.lo:  # rewound (e.g. a checkpoint restored an earlier step)
            self.lo, self.hi = e_lo, e_lo - 1
        if e_hi > self.hi:
            need0 = max(self.hi + 1, e_lo)
            blk = None
            if self._thread is not None:
                self._thread.join()
                self._thread = None
                with self._lock:
                    ahead, self._ahead = self._ahead, None
                if ahead is not None and ahead[0] <= need0 and ahead[0] + ahead[1] - 1 >= e_hi:
                    blk = ahead[2][need0 - ahead[0]:]
            # never evict an epoch this launch still reads: at most e_lo + E - 1
            cap = e_lo + self.E - 1
            if blk is None:
                need_hi = min(max(e_hi, need0 + self.E // 2 - 1), cap)
                blk = self._generate(need0, need_hi - need0 + 1)
            blk = blk[:cap - need0 + 1]
            if need0 > self.hi + 1:
                self.lo, self.hi = need0, need0 - 1
            self._write(need0, blk)
        # keep the next block generating while the GPU works through this one
        if self._thread is None and self._ahead is None and self.hi - e_hi < self.E // 2:
            self._prefetch(self.hi + 1, self.E // 2)

    def native(self, cfg):
        """Point a SamplerCfg (``SamplerGeometry.to_native()``) at the ring."""
        from .. import _native as nat

        cfg.mode = nat.SAMPLER_TABLE
        cfg.perm = self.table.data_ptr()
        cfg.perm_epochs = self.E
        return cfg

    def epochs_of_steps(self, t0: int, t1: int) -> tuple[int, int]:
        """Epochs read by steps [t0, t1] (the kernel also prefetches step t1 + 1)."""
        spe = self.geom.steps_per_epoch
        return t0 // spe, (t1 + 1) // spe
