// Microbenchmark: on-chip hand-off round trip between two workgroups of one launch
// (blocks 0 and 8: one XCD under round-robin dispatch; block 1: another XCD), the
// primitive under the split-batch step's exchange (csrc/grp_core.h).
// Ping-pong: A stores epoch e into granule 0 (16 B), B polls until it sees e, stores e
// into granule 1, A polls for it; N round trips, timed with s_memtime on A.
// Variants: store cache bits (0 = plain, 16 = sc1) x poll-load cache bits (16 = sc1, 1 = sc0,
// 17 = sc0 sc1) x lanes per poll (1 lane, or a whole wave polling 64 contiguous granules, as
// the exchange's poller waves do).  A load form that can hit a stale line in the CU's L1
// never sees the peer's epoch: its run ends at the spin bound and prints "stale".
// Second part: dependent-load latency (one lane, a pointer chase over 64 lines that stay in
// L2) per load cache-bit form.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000);
}

template <int ST, bool WAVE, int LD = 16>
__global__ void pingpong(void* buf, int peer_block, int n, unsigned long long* out) {
  const int b = blockIdx.x;
  if (b != 0 && b != peer_block) return;
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  const bool a = b == 0;
  __amdgpu_buffer_rsrc_t rs = rsrc(buf);
  const int my_off = (a ? 0 : 4096) + (WAVE ? lane * 16 : 0);
  const int peer_off = (a ? 4096 : 0) + (WAVE ? lane * 16 : 0);
  unsigned long long t0 = 0;
  if (a) t0 = __builtin_amdgcn_s_memtime();
  for (int e = 1; e <= n; ++e) {
    if (a) {
      if (WAVE || lane == 0) __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)e, 0, 0, 0}, rs, my_off, 0, ST);
      unsigned long long spins = 0;
      while (true) {
        asm volatile("" ::: "memory");
        u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, peer_off, 0, LD);
        if (__all((int)(x.x == (unsigned)e))) break;
        if (++spins > 2000000ull) return;  // bounded: a lost hand-off ends the kernel
      }
    } else {
      unsigned long long spins = 0;
      while (true) {
        asm volatile("" ::: "memory");
        u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, peer_off, 0, LD);
        if (__all((int)(x.x == (unsigned)e))) break;
        if (++spins > 2000000ull) return;  // bounded: a lost hand-off ends the kernel
      }
      if (WAVE || lane == 0) __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)e, 0, 0, 0}, rs, my_off, 0, ST);
    }
  }
  if (a && lane == 0) {
    out[0] = __builtin_amdgcn_s_memtime() - t0;
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    out[1] = x;
  }
  if (!a && lane == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    out[2] = x;
  }
}

template <int ST, bool WAVE, int LD = 16>
void run(const char* name, void* buf, unsigned long long* d_out, int peer) {
  const int n = 2000;
  (void)hipMemset(buf, 0, 8192);
  (void)hipMemset(d_out, 0, 64);
  hipLaunchKernelGGL((pingpong<ST, WAVE, LD>), dim3(16), dim3(64), 0, 0, buf, peer, n, d_out);
  unsigned long long h[3];
  (void)hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost);
  if (!h[0]) printf("{\"variant\": \"%s\", \"peer_block\": %d, \"stale\": true}\n", name, peer);
  else
    printf("{\"variant\": \"%s\", \"peer_block\": %d, \"xcc\": [%llu, %llu], \"cycles_per_round_trip\": %.1f}\n", name,
           peer, h[1], h[2], (double)h[0] / n);
}

// one lane chases next = buf[cur].x over 64 lines (16 KB, L2-resident after the first lap)
template <int LD>
__global__ void chase(void* buf, int n, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  __amdgpu_buffer_rsrc_t rs = rsrc(buf);
  unsigned off = 0;
  for (int i = 0; i < 64; ++i) { const u32x4 v_ = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, LD); off = v_.x; }  // warm lap
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) { const u32x4 v_ = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, LD); off = v_.x; }
  out[0] = __builtin_amdgcn_s_memtime() - t0;
  out[1] = off;
}

template <int LD>
void run_chase(const char* name, void* buf, unsigned long long* d_out) {
  const int n = 4096;
  unsigned h_init[64 * 64] = {};
  for (int i = 0; i < 64; ++i) h_init[i * 64] = ((i * 37 + 1) % 64) * 256;  // line i -> line (37 i + 1) mod 64
  (void)hipMemcpy(buf, h_init, sizeof h_init, hipMemcpyHostToDevice);
  hipLaunchKernelGGL((chase<LD>), dim3(1), dim3(64), 0, 0, buf, n, d_out);
  unsigned long long h[2];
  (void)hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost);
  printf("{\"chase\": \"%s\", \"cycles_per_load\": %.1f}\n", name, (double)h[0] / n);
}

int main() {
  void* buf;
  unsigned long long* d_out;
  (void)hipMalloc(&buf, 65536);
  (void)hipMalloc(&d_out, 64);
  for (int peer : {8, 1}) {
    run<16, false>("sc1 store, 1 lane", buf, d_out, peer);
    if (peer == 8) run<0, false>("plain store, 1 lane", buf, d_out, peer);
    run<16, true>("sc1 store, 64 lanes x 16 B", buf, d_out, peer);
    if (peer == 8) run<0, true>("plain store, 64 lanes x 16 B", buf, d_out, peer);
  }
  run<0, false, 1>("plain store, sc0 poll, 1 lane", buf, d_out, 8);
  run<0, false, 17>("plain store, sc0 sc1 poll, 1 lane", buf, d_out, 8);
  run<0, true, 1>("plain store, sc0 poll, 64 lanes x 16 B", buf, d_out, 8);
  run<0, true, 17>("plain store, sc0 sc1 poll, 64 lanes x 16 B", buf, d_out, 8);
  run_chase<0>("plain", buf, d_out);
  run_chase<1>("sc0", buf, d_out);
  run_chase<16>("sc1", buf, d_out);
  run_chase<17>("sc0 sc1", buf, d_out);
  return 0;
}
