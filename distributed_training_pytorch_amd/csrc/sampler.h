// Device-side distributed sampler.
//
// Semantics mirror torch.utils.data.DistributedSampler + DataLoader(drop_last=
// False) as used by the reference (demo.py:139-154):
//   * per epoch a permutation of [0, n) (shuffle) or the identity (standard),
//   * padded to total = ceil(n / W) * W by repeating from the start,
//   * rank r takes positions r, r + W, r + 2W, ...  (num_samples = total / W),
//   * batches of `batch` consecutive positions, last batch may be short.
// The permutation is a keyed 4-round Feistel network on 2*half bits with
// cycle-walking into [0, n): O(1) per index, no storage, no host round trip, so
// a hipGraph replay or a persistent multi-step kernel can draw its own batches.
// It is a different (but equally uniform) permutation than torch.randperm; the
// host-index path (SAMPLER_EXPLICIT) reproduces torch's exact order when parity
// with DistributedSampler matters.  The identical function exists in Python
// (data/sampler.py) and is checked bit-for-bit by the GPU tests.
#pragma once
#include "dtp_common.h"

namespace dtp {

enum SamplerMode : int {
  SAMPLER_EXPLICIT = 0,    // indices supplied in a device buffer
  SAMPLER_DIST_SHUFFLE = 1,  // DistributedSampler(shuffle=True)
  SAMPLER_SEQUENTIAL = 2,  // DataLoader without sampler (every rank reads all of n in order)
  SAMPLER_DIST_NOSHUFFLE = 3,  // DistributedSampler(shuffle=False)
  SAMPLER_TABLE = 4,       // DistributedSampler(shuffle=True) with the epoch permutations read from a
                           // device ring `perm` filled by the host (randperm.hip: torch's exact order)
};

struct SamplerCfg {
  int mode;
  int n;            // dataset size
  int world;
  int rank;
  int batch;        // per-rank batch size
  int num_samples;  // per-rank samples per epoch
  int steps_per_epoch;
  int bits;         // Feistel domain = 2^bits >= n
  uint64_t seed;
  const int* perm;  // SAMPLER_TABLE: [perm_epochs][n] ring, epoch e in slot e & (perm_epochs - 1)
  int perm_epochs;  // power of two
  int pad_;
};

// the permutation of epoch e in the SAMPLER_TABLE ring
DTP_HD const int* table_epoch(const SamplerCfg& s, int epoch) {
  return s.perm + (size_t)(epoch & (s.perm_epochs - 1)) * s.n;
}

DTP_HD uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

DTP_HD uint32_t round_key(uint64_t seed, uint32_t epoch, uint32_t r) {
  const uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
  return hash32(lo ^ hash32(hi + epoch * 0x9E3779B9U + r * 0x85EBCA6BU));
}

// Bijection on [0, 2^bits): 4 rounds of  lo ^= F(hi, key) ; rotate (lo to the
// top).  Works for any bits (no even-width restriction), so a power-of-two n
// needs no cycle-walking at all; other n cycle-walk into [0, n).
DTP_HD uint32_t feistel_permute(uint32_t q, uint32_t n, int bits, const uint32_t (&k)[4]) {
  const int r = bits > 1 ? (bits >> 1) : 1;
  const uint32_t rmask = (1u << r) - 1u;
  const uint32_t dmask = bits >= 32 ? 0xffffffffu : ((1u << bits) - 1u);
  do {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t hi = q >> r;
      const uint32_t lo = (q & rmask) ^ (hash32(hi ^ k[i]) & rmask);
      q = ((lo << (bits - r)) | hi) & dmask;
    }
  } while (q >= n);
  return q;
}

// feistel_permute for n == 2^bits: one pass lands in [0, n), no cycle-walk loop
// (straight-line code the scheduler can interleave with other work)
DTP_HD uint32_t feistel_permute_pow2(uint32_t q, int bits, const uint32_t (&k)[4]) {
  const int r = bits > 1 ? (bits >> 1) : 1;
  const uint32_t rmask = (1u << r) - 1u;
  const uint32_t dmask = bits >= 32 ? 0xffffffffu : ((1u << bits) - 1u);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t hi = q >> r;
    const uint32_t lo = (q & rmask) ^ (hash32(hi ^ k[i]) & rmask);
    q = ((lo << (bits - r)) | hi) & dmask;
  }
  return q;
}

// Batch geometry of global step t on this rank.
struct BatchPos {
  int epoch;
  int start;  // first per-rank position of the batch
  int size;   // samples in this batch
};

DTP_HD BatchPos batch_pos(const SamplerCfg& s, long long t) {
  BatchPos b;
  b.epoch = (int)(t / s.steps_per_epoch);
  const int bi = (int)(t % s.steps_per_epoch);
  b.start = bi * s.batch;
  const int rem = s.num_samples - b.start;
  b.size = rem < s.batch ? rem : s.batch;
  return b;
}

// dataset index of the k-th sample of the batch described by bp.
DTP_HD int sample_index(const SamplerCfg& s, const BatchPos& bp, const uint32_t (&keys)[4], int k) {
  const int pos = bp.start + k;
  if (s.mode == SAMPLER_SEQUENTIAL) return pos;
  int q = s.rank + pos * s.world;  // position in the padded list
  if (q >= s.n) q %= s.n;           // padding repeats from the start
  if (s.mode == SAMPLER_DIST_SHUFFLE) return (int)feistel_permute((uint32_t)q, (uint32_t)s.n, s.bits, keys);
  if (s.mode == SAMPLER_TABLE) return table_epoch(s, bp.epoch)[q];
  return q;
}

DTP_HD void epoch_keys(const SamplerCfg& s, int epoch, uint32_t (&k)[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) k[r] = round_key(s.seed, (uint32_t)epoch, (uint32_t)r);
}

}  // namespace dtp
