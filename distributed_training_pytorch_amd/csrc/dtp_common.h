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

// dst[0 .. na) = A[0 .. na), dst[na .. na + nb) = B[0 .. nb) (global -> LDS) in two halves:
// load() issues every global load of this thread into registers, store() writes them to
// LDS.  A plain `for (e = tid; e < n; e += NTH) dst[e] = src[e]` loop with a runtime trip
// count waits out its loads chunk by chunk before the stores -- several memory round trips
// per launch prologue (scripts/k20_prologue.py: 7.4 k cycles from kernel entry to the
// first barrier); issued with the prologue's other loads, the fill costs none of its own.
// Requires na + nb <= MAXE (checked by the host).
template <int MAXE, int NTH>
struct LdsFill2 {
  static constexpr int J = (MAXE + NTH - 1) / NTH;
  float v[J];
  int n;
  DTP_DEV void load(const float* __restrict__ A, int na, const float* __restrict__ B, int nb, int tid) {
    n = na + nb;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int e = tid + j * NTH;
      v[j] = 0.f;
      if (e < na) v[j] = A[e];
      else if (e - na < nb) v[j] = B[e - na];
    }
  }
  DTP_DEV void store(float* __restrict__ dst, int tid) const {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int e = tid + j * NTH;
      if (e < n) dst[e] = v[j];
    }
  }
};

// error reporting shared by every translation unit (defined in runtime.hip)
int set_err(int code, const char* msg);
int check_launch(const char* what);

}  // namespace dtp
