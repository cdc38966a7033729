"""Host-side batch indexing: the vectorised device-sampler twin is bit-exact with the
scalar Feistel reference, BatchIndexer hands out the same batches as the host
lists (device sampler and exact DistributedSampler order), and LossRing reduces a
chunk of per-step losses to the same global means as a per-step all-reduce."""
import torch
import pytest

from distributed_training_pytorch_amd.data import sampler as S

from .dist_utils import run_ranks


def _scalar_indices(g: S.SamplerGeometry, t: int) -> list[int]:
    epoch, start, size = g.batch_pos(t)
    keys = S.epoch_keys(g.seed, epoch)
    return [S.feistel_permute((g.rank + (start + k) * g.world) % g.n, g.n, g.bits, keys) for k in range(size)]


def test_vectorised_feistel_matches_scalar_twin():
    # power-of-two and cycle-walked (non power-of-two) domains, padded last batches
    for n, W, r, B, seed in [(512, 1, 0, 256, 0), (512, 8, 3, 64, 1234), (1000, 3, 2, 100, 7),
                             (4096, 8, 7, 256, 99), (37, 4, 1, 5, 3), (2, 1, 0, 1, 5)]:
        g = S.SamplerGeometry(n=n, world=W, rank=r, batch=B, seed=seed)
        for t in range(3 * g.steps_per_epoch + 1):
            assert g.indices(t) == _scalar_indices(g, t), (n, W, r, t)


def test_batch_indexer_cpu_orders():
    g = S.SamplerGeometry(n=300, world=2, rank=1, batch=64, seed=11)
    dev = torch.device("cpu")
    ix = S.BatchIndexer(g, dev)
    ex = S.BatchIndexer(g, dev, exact_torch=True)
    stream = S.EpochIndexStream(g)
    for t in range(2 * g.steps_per_epoch + 2):
        assert ix(t).tolist() == g.indices(t)
        assert ex(t).tolist() == stream.indices(t)
    seq = S.BatchIndexer(S.SamplerGeometry(n=10, batch=4, distributed=False), dev)
    assert [seq(t).tolist() for t in range(4)] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9], [0, 1, 2, 3]]


def _ring_fn(rank, world):
    from distributed_training_pytorch_amd.utils.logging import LossRing

    ring = LossRing(3, 2, torch.device("cpu"), world)
    got = []
    for step in range(7):
        ring.put(step, torch.tensor(float(step + rank)), torch.tensor(10.0 * rank))
        if ring.full():
            got += ring.flush()
    got += ring.flush()
    return got


def test_loss_ring_reduces_chunks_like_per_step_all_reduce():
    outs = run_ranks(_ring_fn, 2)
    for got in outs.values():
        assert [s for s, _ in got] == list(range(7))
        for s, (vx, vy) in got:
            assert vx == (s + s + 1) / 2 and vy == 5.0


def test_native_randperm_is_torch_randperm():
    """csrc/randperm.hip (MT19937 + Fisher-Yates, host threads) reproduces
    torch.randperm(n, generator seeded with seed + epoch) bit for bit -- the order the
    fused kernels read from the permutation ring by default."""
    import torch

    from distributed_training_pytorch_amd import _native as nat

    lib = nat.load()
    for n, seed, e0, ne in [(512, 0, 0, 5), (512, 7, 1000, 3), (100, 3, 0, 4), (4096, 12345, 17, 2), (3, 0, 0, 8)]:
        out = torch.empty(ne, n, dtype=torch.int32)
        nat.check(lib.dtp_randperm_fill(seed, n, e0, ne, out.data_ptr(), 4), "dtp_randperm_fill")
        for k in range(ne):
            g = torch.Generator()
            g.manual_seed(seed + e0 + k)
            assert out[k].tolist() == torch.randperm(n, generator=g).tolist(), (n, seed, e0 + k)


def test_permutation_ring_cpu_refill_and_order():
    """PermutationRing: slot e & (E-1) holds epoch e; ensure() refills across the ring's
    wrap and after a rewind; the padded per-rank positions read through it give exactly
    DistributedSampler's indices."""
    import torch

    from distributed_training_pytorch_amd.data.sampler import (PermutationRing, SamplerGeometry,
                                                               torch_distributed_indices)

    g = SamplerGeometry(n=100, world=3, rank=1, batch=16, seed=4)
    ring = PermutationRing(g, torch.device("cpu"), epochs=8)
    assert ring.E == 8 and (ring.lo, ring.hi) == (0, 7)
    for lo, hi in [(0, 3), (6, 12), (20, 27), (2, 5)]:
        ring.ensure(lo, hi)
        for e in range(lo, hi + 1):
            perm = ring.table[e & 7].tolist()
            ref = torch_distributed_indices(100, 3, 1, e, seed=4)
            pos = [(1 + j * 3) % 100 for j in range(g.num_samples)]
            assert [perm[q] for q in pos] == ref, e
    if ring._thread is not None:
        ring._thread.join()


def test_library_build_stamp_ties_the_kernels_to_the_sources(monkeypatch):
    """libdtp.so carries the hash of the csrc tree and flags it was built from
    (``dtp_source_hash``); loading it next to different sources fails loudly instead of
    running stale kernels."""
    from distributed_training_pytorch_amd import _native as nat
    from distributed_training_pytorch_amd import build

    lib = nat.load()
    assert nat.source_hash() == build.source_hash() and len(build.source_hash()) >= 16
    monkeypatch.delenv("DTP_SKIP_STAMP", raising=False)
    monkeypatch.delenv("DTP_LIB", raising=False)
    monkeypatch.setattr(build, "source_hash", lambda: "f" * 64)
    with pytest.raises(nat.NativeUnavailable, match="stale"):
        nat.check_stamp(lib)
