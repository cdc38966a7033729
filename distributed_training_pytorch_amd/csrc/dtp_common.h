// Shared device helpers for the MI355X (gfx950 / CDNA4) kernels of the
// distributed-training harness.  Everything here is wave64-native: block sizes
// are multiples of 64, cross-lane reductions use 64-lane shuffles, and the
// matrix work goes through the exact-fp32 MFMA (v_mfma_f32_16x16x4_f32).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include <utility>

#define DTP_DEV __device__ __forceinline__
#define DTP_HD __host__ __device__ __forceinline__

namespace dtp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kBlock = 256;  // 4 waves = one wave per SIMD of a CU

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).
// Guarantees every register-array index is a constant expression, so the
// per-sample activation arrays never spill to scratch.
template <int B, int E, class F>
DTP_DEV void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(static_cast<F&&>(f));
  }
}

DTP_DEV float leaky(float z, float slope) { return z > 0.f ? z : z * slope; }
// derivative expressed through the activation OUTPUT (sign(a) == sign(z) for
// slope > 0; at z == 0 torch uses the negative slope, and so do we).
DTP_DEV float leaky_grad_from_out(float a, float slope) { return a > 0.f ? 1.f : slope; }

DTP_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// x^e for a non-negative integer e by repeated squaring, in double: the Adam
// bias corrections 1 - beta^t are formed in double exactly as torch does on the
// host (python float), without a libm pow() on the device.
DTP_HD double pow_int(double b, uint64_t e) {
  double r = 1.0;
  while (e) {
    if (e & 1) r *= b;
    b *= b;
    e >>= 1;
  }
  return r;
}

typedef __attribute__((address_space(3))) void dtp_lds_void_t;
typedef __attribute__((address_space(1))) void dtp_gbl_void_t;

// dst[0 .. na) = A[0 .. na), dst[na .. na + nb) = B[0 .. nb) (global -> LDS) by LDS-DMA
// (global_load_lds_dword: no staging registers, no wait inside the loop -- every wave
// issues its ceil((na + nb) / NTH) copies back to back; the caller's next __syncthreads
// waits them out).  The launch prologue is instruction-fetch bound (its code runs once per
// launch on CUs whose caches do not hold it): a compact loop beats both a register-staged
// loop with a runtime trip count (one memory round trip per unrolled chunk) and a fully
// unrolled register-staged fill (16 load + 16 store blocks: 9.0-9.7 k instead of 7.4 k
// cycles to the first barrier, scripts/k20_prologue.py).  The LDS destination of one wave
// instruction is 64 consecutive floats (wave-uniform base + lane x 4): the last one may run
// past na + nb, so dst must have room up to the next multiple of 64 (the lanes there copy
// the last element).  Requires na + nb >= 1.
template <int NTH>
DTP_DEV void lds_dma_fill2(float* dst, const float* A, int na, const float* B, int nb, int tid) {
  const int n = na + nb;
  const int wave = tid / kWave, lane = tid - (tid / kWave) * kWave;
  for (int c = wave * kWave; c < n; c += NTH) {
    int e = c + lane;
    e = e < n ? e : n - 1;
    const float* g = e < na ? A + e : B + (e - na);
    __builtin_amdgcn_global_load_lds((dtp_gbl_void_t*)const_cast<float*>(g), (dtp_lds_void_t*)(dst + c), 4, 0, 0);
  }
}

// error reporting shared by every translation unit (defined in runtime.hip)
int set_err(int code, const char* msg);
int check_launch(const char* what);

}  // namespace dtp
