// Host-side check of the device sampler (csrc/sampler.h), built with
// AddressSanitizer + UBSan on the host pass only (tests/test_native_host_sanitize.py).
// The same DTP_HD functions the persistent train kernel calls per sample are run
// here on the CPU:
//   * feistel_permute is a bijection on [0, n) for every n, including n = 2^k
//     (no cycle-walk) and n = 2^k + 1 (worst-case cycle-walk);
//   * over one epoch the ranks of DistributedSampler(shuffle) / (no shuffle)
//     cover every index, with the padding repeats and per-rank counts torch uses;
//   * batch_pos splits an epoch into ceil(num_samples / batch) batches, last one short;
//   * pow_int matches std::pow to 1 ulp-level tolerance for the Adam bias corrections.
// Reference semantics: torch DistributedSampler as used at demo.py:139-154 of the
// reference (SURVEY.md §2.3 "Data sharding").
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sampler.h"

using namespace dtp;

static int fails = 0;
#define CHECK(c, ...)                         \
  do {                                        \
    if (!(c)) {                               \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);      \
      std::fprintf(stderr, "\n");             \
      ++fails;                                \
    }                                         \
  } while (0)

static int bits_for(int n) {
  int b = 1;
  while ((1 << b) < n) ++b;
  return b;
}

static SamplerCfg make_cfg(int mode, int n, int world, int rank, int batch, uint64_t seed) {
  SamplerCfg s{};
  s.mode = mode;
  s.n = n;
  s.world = world;
  s.rank = rank;
  s.batch = batch;
  s.num_samples = (mode == SAMPLER_SEQUENTIAL) ? n : (n + world - 1) / world;
  s.steps_per_epoch = (s.num_samples + batch - 1) / batch;
  s.bits = bits_for(n);
  s.seed = seed;
  return s;
}

int main() {
  const int ns[] = {1, 2, 3, 7, 64, 65, 255, 256, 257, 512, 1000, 4096, 4097};
  for (int n : ns) {
    SamplerCfg s = make_cfg(SAMPLER_DIST_SHUFFLE, n, 1, 0, 256, 0x1234abcdULL + n);
    for (int epoch = 0; epoch < 3; ++epoch) {
      uint32_t k[4];
      epoch_keys(s, epoch, k);
      std::vector<int> seen(n, 0);
      for (int q = 0; q < n; ++q) {
        const uint32_t p = feistel_permute((uint32_t)q, (uint32_t)n, s.bits, k);
        CHECK(p < (uint32_t)n, "n=%d q=%d -> %u out of range", n, q, p);
        if (p < (uint32_t)n) ++seen[p];
      }
      for (int i = 0; i < n; ++i) CHECK(seen[i] == 1, "n=%d epoch=%d index %d hit %d times", n, epoch, i, seen[i]);
    }
  }

  const int worlds[] = {1, 2, 3, 4, 8};
  const int modes[] = {SAMPLER_DIST_SHUFFLE, SAMPLER_DIST_NOSHUFFLE};
  for (int mode : modes)
    for (int n : {512, 1000, 7, 4097})
      for (int world : worlds) {
        const int total = ((n + world - 1) / world) * world;
        std::vector<int> hits(n, 0);
        int drawn = 0;
        for (int rank = 0; rank < world; ++rank) {
          SamplerCfg s = make_cfg(mode, n, world, rank, 64, 42);
          int rank_drawn = 0;
          for (long long t = 0; t < s.steps_per_epoch; ++t) {
            const BatchPos bp = batch_pos(s, t);
            CHECK(bp.epoch == 0, "epoch of step %lld is %d", t, bp.epoch);
            CHECK(bp.size > 0 && bp.size <= s.batch, "batch size %d", bp.size);
            uint32_t k[4];
            epoch_keys(s, bp.epoch, k);
            for (int j = 0; j < bp.size; ++j) {
              const int idx = sample_index(s, bp, k, j);
              CHECK(idx >= 0 && idx < n, "index %d out of [0,%d)", idx, n);
              if (idx >= 0 && idx < n) ++hits[idx];
              ++rank_drawn;
            }
          }
          CHECK(rank_drawn == s.num_samples, "rank %d drew %d, expected %d", rank, rank_drawn, s.num_samples);
          drawn += rank_drawn;
        }
        CHECK(drawn == total, "world %d drew %d, expected padded total %d", world, drawn, total);
        for (int i = 0; i < n; ++i)
          CHECK(hits[i] >= 1 && hits[i] <= 2, "mode %d n=%d W=%d index %d hit %d times", mode, n, world, i, hits[i]);
      }

  {  // sequential: every rank reads the whole set in order
    SamplerCfg s = make_cfg(SAMPLER_SEQUENTIAL, 512, 4, 3, 256, 0);
    uint32_t k[4];
    epoch_keys(s, 0, k);
    for (long long t = 0; t < 2 * s.steps_per_epoch; ++t) {
      const BatchPos bp = batch_pos(s, t);
      for (int j = 0; j < bp.size; ++j)
        CHECK(sample_index(s, bp, k, j) == bp.start + j, "sequential order broken at step %lld", t);
    }
  }

  for (double b : {0.9, 0.999})
    for (uint64_t e : {0ull, 1ull, 2ull, 10ull, 1000ull, 123457ull}) {
      const double want = std::pow(b, (double)e), got = pow_int(b, e);
      CHECK(std::fabs(got - want) <= 1e-12 * std::fmax(1.0, std::fabs(want)) + 1e-300,
            "pow_int(%g,%llu)=%.17g want %.17g", b, (unsigned long long)e, got, want);
    }

  if (fails) {
    std::fprintf(stderr, "%d failures\n", fails);
    return 1;
  }
  std::printf("sampler host test OK\n");
  return 0;
}
