// Host-side permutation generator for the exact DistributedSampler order.
//
// torch.utils.data.DistributedSampler draws, per epoch, torch.randperm(n) from a CPU
// generator seeded with seed + epoch (the reference's loader, demo.py:141-148).  On
// the CPU, torch.randperm(n < 2^32/20) is a Fisher-Yates shuffle driven by the
// generator's 32-bit MT19937 stream: r = iota(n); for i < n-1: z = mt() % (n-i);
// swap(r[i], r[i+z]), with MT19937 seeded by init_with_uint32(seed).  This file
// reproduces that bit for bit (checked against torch.randperm by the CPU tests) so
// the fused train kernel can read the reference's exact sample order from a device
// table of upcoming epochs (SAMPLER_TABLE) instead of the host handing it indices
// step by step.  Epochs are generated in parallel on host threads.
#include <algorithm>
#include <cstdint>
#include <thread>
#include <vector>

namespace {

class Mt19937 {
 public:
  explicit Mt19937(uint32_t seed) {
    st_[0] = seed;
    for (int j = 1; j < kN; ++j) st_[j] = 1812433253u * (st_[j - 1] ^ (st_[j - 1] >> 30)) + (uint32_t)j;
    idx_ = kN;
  }
  uint32_t operator()() {
    if (idx_ >= kN) twist();
    uint32_t y = st_[idx_++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }

 private:
  static constexpr int kN = 624, kM = 397;
  void twist() {
    for (int k = 0; k < kN; ++k) {
      const uint32_t y = (st_[k] & 0x80000000u) | (st_[(k + 1) % kN] & 0x7fffffffu);
      st_[k] = st_[(k + kM) % kN] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    idx_ = 0;
  }
  uint32_t st_[kN];
  int idx_;
};

// torch.randperm(n, generator=torch.Generator().manual_seed(seed)) on the CPU
void randperm(uint64_t seed, int n, int32_t* r) {
  Mt19937 mt((uint32_t)(seed & 0xffffffffu));  // at::mt19937 keeps the low 32 bits of the seed
  for (int i = 0; i < n; ++i) r[i] = i;
  for (int i = 0; i < n - 1; ++i) {
    const int64_t z = (int64_t)(mt() % (uint32_t)(n - i));
    std::swap(r[i], r[i + z]);
  }
}

}  // namespace

extern "C" {

// out[e][n] = randperm(n, seed + epoch0 + e) for e in [0, n_epochs); threads <= 0: all cores
int dtp_randperm_fill(unsigned long long seed, int n, long long epoch0, int n_epochs, int* out, int threads) {
  if (n <= 0 || n_epochs <= 0 || !out) return -1;
  if ((long long)n >= 4294967295ll / 20) return -2;  // torch switches to 64-bit draws there
  int nt = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
  nt = std::max(1, std::min(nt, n_epochs));
  std::vector<std::thread> pool;
  pool.reserve(nt);
  for (int w = 0; w < nt; ++w) {
    pool.emplace_back([=] {
      for (int e = w; e < n_epochs; e += nt)
        randperm((unsigned long long)(seed + (unsigned long long)(epoch0 + e)), n, out + (size_t)e * n);
    });
  }
  for (auto& t : pool) t.join();
  return 0;
}

}  // extern "C"
