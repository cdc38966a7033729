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

import math
from dataclasses import dataclass

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

    def indices(self, t: int) -> list[int]:
        """Dataset indices of global step t on this rank (device-sampler order)."""
        epoch, start, size = self.batch_pos(t)
        if self.mode == SAMPLER_SEQUENTIAL:
            return list(range(start, start + size))
        keys = epoch_keys(self.seed, epoch)
        out = []
        for k in range(size):
            q = (self.rank + (start + k) * self.world) % self.n
            out.append(feistel_permute(q, self.n, self.bits, keys) if self.mode == SAMPLER_DIST_SHUFFLE else q)
        return out

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

    def indices(self, t: int) -> list[int]:
        epoch, start, size = self.geom.batch_pos(t)
        if epoch != self._epoch:
            g = self.geom
            if g.distributed:
                self._idx = torch_distributed_indices(g.n, g.world, g.rank, epoch, g.seed, g.shuffle)
            else:
                self._idx = list(range(g.n))
            self._epoch = epoch
        return self._idx[start:start + size]
