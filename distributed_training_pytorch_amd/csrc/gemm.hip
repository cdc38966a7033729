// LDS-tiled MFMA GEMM for gfx950 (CDNA4) with fused Linear-layer epilogues.
//
// C[M,N] (+)= epi( alpha * sum_k A(m,k) * B(n,k) )
//   A(m,k) = A[m*lda + k] (trans_a = 0)  or  A[k*lda + m] (trans_a = 1)
//   B(n,k) = B[n*ldb + k] (trans_b = 0)  or  B[k*ldb + n] (trans_b = 1)
// so the three GEMMs of an MLP layer y = act(x W^T + b) are
//   forward   y  = x W^T        (0, 0)   epilogue: + bias, LeakyReLU
//   grad in   dx = dz W         (0, 1)   epilogue: * act'(h_prev)   (h_prev = aux)
//   grad W    dW = dz^T x       (1, 1)   optional split-K (f32 atomics into C)
// (the addmm / mm / leaky_relu(_backward) kernels the
// reference runs through cuBLAS/ATen, `toy_model_and_data.py:12-25`.)
//
// MI355X-first design:
//  * 128x128 block tile, 256 threads = 4 waves (2x2), each wave a 64x64 tile of
//    4x4 MFMA 16x16 fragments: v_mfma_f32_16x16x32_bf16 for bf16 inputs,
//    v_mfma_f32_16x16x4_f32 (exact fp32) for f32 inputs.
//  * the LDS image of both operands is K-contiguous, 128-byte rows (BK = 64
//    bf16 / 32 f32) of eight 16-byte chunks XOR-swizzled by (row ^ row>>3) & 7:
//    every MFMA fragment is one conflict-free ds_read_b128.  A K-contiguous
//    source is staged with global_load_dwordx4 -> ds_write_b128; an M/N-contiguous
//    (transposed) source is loaded as 4 k-rows x 16 B and transposed in registers
//    before the LDS write, so all layouts share one MFMA inner loop.
//  * two LDS buffers, the next K-tile's global loads issued before the current
//    tile's MFMAs, one barrier per K-tile.
//  * blockIdx is remapped so that consecutive tiles land on the same XCD (the
//    dispatcher deals workgroups round-robin over the 8 XCDs, each with its own
//    L2), then grouped 8 M-tiles at a time for operand reuse in that L2.
#include "dtp_common.h"
#include "dtp_api.h"
#include "gemm_epi.h"

namespace dtp {
namespace gemm {

constexpr int kBM = 128, kBN = 128, kThreads = 256;
constexpr int kChunks = 8;  // 16-byte chunks per 128-byte LDS row


DTP_DEV int swz(int row) { return (row ^ (row >> 3)) & 7; }
DTP_DEV int slot(int row, int chunk) { return row * kChunks + (chunk ^ swz(row)); }


// 16 bytes of row `r` (memory row), elements [c, c+EPC) of a matrix with `rows` rows,
// `cols` columns and leading dimension `ld`; out-of-range elements read as 0.
// LEAN: the caller guarantees 16-byte aligned rows and cols % EPC == 0 (no
// partial chunks): one predicated dwordx4 load, no per-element fallback code.
template <int DT, bool LEAN = false>
DTP_DEV uint4 load_chunk(const char* base, long long ld, int r, int c, int rows, int cols, bool vec) {
  using T = Ty<DT>;
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (r >= rows || c >= cols) return v;
  const char* p = base + (static_cast<long long>(r) * ld + c) * T::ES;
  if constexpr (LEAN) return *reinterpret_cast<const uint4*>(p);
  if (vec && c + T::EPC <= cols) return *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int e = 0; e < T::EPC; ++e) {
    if (c + e < cols) {
      if constexpr (DT == DTP_DT_BF16) {
        const uint32_t h = *reinterpret_cast<const uint16_t*>(p + e * 2);
        w[e >> 1] |= h << ((e & 1) * 16);
      } else {
        w[e] = *reinterpret_cast<const uint32_t*>(p + e * 4);
      }
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Staging registers of one operand tile (ROWS rows x BK) for one thread: ROWS/32
// 16-byte chunks (ROWS x 8 chunks over 256 threads).
template <int ROWS>
struct Stage {
  uint4 v[ROWS / 32];
};

// Operand X(row, k), rows [row0, row0+ROWS), k [k0, k0+BK).
//   trans = 0: X(row,k) at base[row*ld + k]    (memory rows = operand rows)
//   trans = 1: X(row,k) at base[k*ld + row]    (memory rows = k): each thread loads
//              (4 k-rows x 16 B) blocks and transposes them in registers
template <int DT, bool TRANS, int ROWS, bool LEAN = false>
DTP_DEV void stage_load(Stage<ROWS>& s, const char* base, long long ld, int row0, int k0, int R, int K, bool vec,
                        int tid) {
  using T = Ty<DT>;
  if constexpr (!TRANS) {
    const int c = tid & 7;
#pragma unroll
    for (int i = 0; i < ROWS / 32; ++i) {
      const int r = (tid >> 3) + 32 * i;
      s.v[i] = load_chunk<DT, LEAN>(base, ld, row0 + r, k0 + c * T::EPC, R, K, vec);
    }
  } else {
    constexpr int RC = ROWS / T::EPC;  // row chunks per tile
#pragma unroll
    for (int b = 0; b < ROWS / 128; ++b) {
      const int combo = tid + kThreads * b;
      const int mc = combo % RC, kq = combo / RC;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        s.v[4 * b + i] = load_chunk<DT, LEAN>(base, ld, k0 + 4 * kq + i, row0 + mc * T::EPC, K, R, vec);
    }
  }
}

template <int DT, bool TRANS, int ROWS>
DTP_DEV void stage_store(const Stage<ROWS>& s, uint4* __restrict__ lds, int tid) {
  using T = Ty<DT>;
  if constexpr (!TRANS) {
    const int c = tid & 7;
#pragma unroll
    for (int i = 0; i < ROWS / 32; ++i) lds[slot((tid >> 3) + 32 * i, c)] = s.v[i];
  } else {
    constexpr int RC = ROWS / T::EPC;
#pragma unroll
    for (int b = 0; b < ROWS / 128; ++b) {
      const int combo = tid + kThreads * b;
      const int mc = combo % RC, kq = combo / RC;
      const uint32_t* w0 = reinterpret_cast<const uint32_t*>(&s.v[4 * b + 0]);
      const uint32_t* w1 = reinterpret_cast<const uint32_t*>(&s.v[4 * b + 1]);
      const uint32_t* w2 = reinterpret_cast<const uint32_t*>(&s.v[4 * b + 2]);
      const uint32_t* w3 = reinterpret_cast<const uint32_t*>(&s.v[4 * b + 3]);
      if constexpr (DT == DTP_DT_F32) {
        // 4 k-rows x 4 rows of floats -> for each row one 16-byte chunk (k = 4kq .. 4kq+3)
#pragma unroll
        for (int e = 0; e < 4; ++e) lds[slot(mc * 4 + e, kq)] = make_uint4(w0[e], w1[e], w2[e], w3[e]);
      } else {
        // bf16: 4 k-rows x 8 rows -> for each row 8 bytes (k = 4kq .. 4kq+3) = half a chunk
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int sh = (e & 1) * 16, q = e >> 1;
          const uint32_t lo = ((w0[q] >> sh) & 0xffffu) | (((w1[q] >> sh) & 0xffffu) << 16);
          const uint32_t hi = ((w2[q] >> sh) & 0xffffu) | (((w3[q] >> sh) & 0xffffu) << 16);
          uint2* dst = reinterpret_cast<uint2*>(lds + slot(mc * 8 + e, kq >> 1)) + (kq & 1);
          *dst = make_uint2(lo, hi);
        }
      }
    }
  }
}

template <int DT, bool TA, bool TB>
__global__ __launch_bounds__(kThreads) void gemm_kernel(DtpGemmArgs a) {
  using T = Ty<DT>;
  __shared__ uint4 lds[2][2][kBM * kChunks];  // [buffer][A|B][row*8 + chunk]: 64 KiB

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, lr = lane & 15, lg = lane >> 4;

  const TileId id = decode_tile<kBM, kBN>(a);
  const int m0 = id.m0, n0 = id.n0, ks = id.ks;

  const int ktiles = (a.K + T::BK - 1) / T::BK;
  const int kper = (ktiles + a.splitk - 1) / a.splitk;
  const int kt0 = ks * kper, kt1 = min(ktiles, kt0 + kper);

  const char* A = static_cast<const char*>(a.A);
  const char* B = static_cast<const char*>(a.B);
  const bool va = a.vec_a != 0, vb = a.vec_b != 0;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stage<kBM> sa, sb;
  if (kt0 < kt1) {
    stage_load<DT, TA, kBM>(sa, A, a.lda, m0, kt0 * T::BK, a.M, a.K, va, tid);
    stage_load<DT, TB, kBN>(sb, B, a.ldb, n0, kt0 * T::BK, a.N, a.K, vb, tid);
    stage_store<DT, TA, kBM>(sa, lds[0][0], tid);
    stage_store<DT, TB, kBN>(sb, lds[0][1], tid);
  }
  __syncthreads();

  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) {
      stage_load<DT, TA, kBM>(sa, A, a.lda, m0, (kt + 1) * T::BK, a.M, a.K, va, tid);
      stage_load<DT, TB, kBN>(sb, B, a.ldb, n0, (kt + 1) * T::BK, a.N, a.K, vb, tid);
    }
    const uint4* la = lds[buf][0];
    const uint4* lb = lds[buf][1];
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      uint4 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = la[slot(wm * 64 + 16 * i + lr, 4 * kc + lg)];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = lb[slot(wn * 64 + 16 * j + lr, 4 * kc + lg)];
      if constexpr (DT == DTP_DT_BF16) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                                __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
      } else {
        // lane group lg supplies k = 4*(4kc+lg) + s at step s, for A and B alike
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float av = __uint_as_float(s == 0 ? fa[i].x : s == 1 ? fa[i].y : s == 2 ? fa[i].z : fa[i].w);
              const float bv = __uint_as_float(s == 0 ? fb[j].x : s == 1 ? fb[j].y : s == 2 ? fb[j].z : fb[j].w);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i][j], 0, 0, 0);
            }
      }
    }
    if (more) {
      stage_store<DT, TA, kBM>(sa, lds[buf ^ 1][0], tid);
      stage_store<DT, TB, kBN>(sb, lds[buf ^ 1][1], tid);
    }
    __syncthreads();
  }

  // ---- epilogue: element (m, n) = acc[i][j][r], m = .. + 4*lg + r, n = .. + lr ----
  char* C = static_cast<char*>(a.C);
  const char* aux = static_cast<const char*>(a.aux);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + 16 * j + lr;
    if (n >= a.N) continue;
    const float bias = (a.bias && ks == 0) ? a.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + 16 * i + 4 * lg + r;
        if (m < a.M) epilogue_store<DT>(a, C, aux, m, n, acc[i][j][r], bias);
      }
    }
  }
}

// 256x256 block tile for large bf16 problems: 4 waves (2x2), each a 128x128 tile
// of 4x4 v_mfma_f32_32x32x16_bf16 fragments (256 accumulators/lane, one wave per
// SIMD).  Per K-tile a wave reads 32 ds_read_b128 for 64 MFMAs (2048 MFMA
// cycles): the LDS port runs at ~25 % instead of the 128x128 kernel's ~100 %
// (64x64 wave tiles re-read every fragment for only 4 MFMAs).
template <bool TA, bool TB>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_big_kernel(DtpGemmArgs a) {
  using T = Ty<DTP_DT_BF16>;
  constexpr int BM = 256, BN = 256;
  __shared__ uint4 lds[2][2][BM * kChunks];  // [buffer][A|B][row*8 + chunk]: 128 KiB
  typedef float f32x16 __attribute__((ext_vector_type(16)));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, lr = lane & 31, lh = lane >> 5;
  const TileId id = decode_tile<BM, BN>(a);
  const int m0 = id.m0, n0 = id.n0;
  const int ktiles = (a.K + T::BK - 1) / T::BK;
  const char* A = static_cast<const char*>(a.A);
  const char* B = static_cast<const char*>(a.B);
  const bool va = a.vec_a != 0, vb = a.vec_b != 0;

  f32x16 acc[16];  // fragment (i, j) = acc[4 * i + j]; every index below is a compile-time constant
  static_for<0, 16>([&](auto IC) { acc[decltype(IC)::value] = f32x16{}; });

  Stage<BM> sa, sb;
  stage_load<DTP_DT_BF16, TA, BM, true>(sa, A, a.lda, m0, 0, a.M, a.K, va, tid);
  stage_load<DTP_DT_BF16, TB, BN, true>(sb, B, a.ldb, n0, 0, a.N, a.K, vb, tid);
  stage_store<DTP_DT_BF16, TA, BM>(sa, lds[0][0], tid);
  stage_store<DTP_DT_BF16, TB, BN>(sb, lds[0][1], tid);
  __syncthreads();

  for (int kt = 0; kt < ktiles; ++kt) {
    const int buf = kt & 1;
    const bool more = kt + 1 < ktiles;
    if (more) {
      stage_load<DTP_DT_BF16, TA, BM, true>(sa, A, a.lda, m0, (kt + 1) * T::BK, a.M, a.K, va, tid);
      stage_load<DTP_DT_BF16, TB, BN, true>(sb, B, a.ldb, n0, (kt + 1) * T::BK, a.N, a.K, vb, tid);
    }
    const uint4* la = lds[buf][0];
    const uint4* lb = lds[buf][1];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {  // K = 16 per MFMA: chunks 2ks (lanes 0-31), 2ks+1 (lanes 32-63)
      uint4 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = la[slot(wm * 128 + 32 * i + lr, 2 * ks + lh)];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = lb[slot(wn * 128 + 32 * j + lr, 2 * ks + lh)];
      static_for<0, 16>([&](auto IC) {
        constexpr int q = decltype(IC)::value;
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, fa[q / 4]),
                                                         __builtin_bit_cast(bf16x8, fb[q % 4]), acc[q], 0, 0, 0);
      });
    }
    if (more) {
      stage_store<DTP_DT_BF16, TA, BM>(sa, lds[buf ^ 1][0], tid);
      stage_store<DTP_DT_BF16, TB, BN>(sb, lds[buf ^ 1][1], tid);
    }
    __syncthreads();
  }

  // epilogue: acc[4i+j][r] is (row = (r&3) + 8*(r>>2) + 4*lh, col = lr) of fragment (i, j)
  char* C = static_cast<char*>(a.C);
  const char* aux = static_cast<const char*>(a.aux);
  static_for<0, 4>([&](auto JC) {
    constexpr int j = decltype(JC)::value;
    const int n = n0 + wn * 128 + 32 * j + lr;
    if (n < a.N) {
      const float bias = a.bias ? a.bias[n] : 0.f;
      static_for<0, 4>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        static_for<0, 16>([&](auto RC) {
          constexpr int r = decltype(RC)::value;
          const int m = m0 + wm * 128 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (m < a.M) epilogue_store<DTP_DT_BF16>(a, C, aux, m, n, acc[4 * i + j][r], bias);
        });
      });
    }
  });
}

// ---------------------------------------------------------------------------
// Fast bf16 GEMM: 256x256x64 tiles, 8 waves (2 x 4, each 128 x 64 of
// v_mfma_f32_16x16x32_bf16), operands staged global -> LDS by the gfx950 LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave instruction): no staging registers
// and no ds_write pass, so each SIMD's two waves hold 128 accumulators plus a
// k-step of fragments and one wave's MFMAs cover the other's LDS reads.  Every
// operand layout of an MLP layer runs here:
//  * K-contiguous operand (x and W of the forward, dz of dx = dz W): LDS image
//    [256 rows][8 x 16-B chunks]; a fragment is one ds_read_b128;
//  * M/N-contiguous operand (W of dx = dz W; dz and h of dW = dz^T h): LDS image
//    [64 k][256 columns] exactly as in memory; a fragment is two
//    ds_read_b64_tr_b16 (gfx950's transposing LDS read): no register transpose.
// Bank swizzles ride on the DMA SOURCE address (the DMA writes lane-linear),
// both with fswz(x) = (x & 3) | ((x >> 1) & 4):
//  * row image: physical chunk p of row r holds logical chunk p ^ fswz(r); the
//    four 16-lane groups of a ds_read_b128 ({0-3,12-15,20-27}, ...) then hit 16
//    distinct 16-B bank slots (conflict-free), and fswz depends on r & 15 only,
//    so all fragments of a wave share one lane address + immediate offsets;
//  * k-major image: the 32-B granule g of k-row k sits at g ^ fswz(k); the eight
//    k-rows one 32-lane half of a transposing read touches land in 8 distinct
//    32-B windows of the 256-B bank row (conflict-free).
// Pipeline: tile t+1's DMA is issued before tile t's ds_read/MFMA block; one
// vmcnt(0) + barrier per K-tile retires it (RAW) and frees tile t's buffer for
// tile t+2's DMA (WAR).  Preconditions (dtp_gemm checks them): K % 64 == 0,
// 16-byte aligned rows, a transposed operand's M/N a multiple of 8.  Rows or
// columns past M / N are clamped on load and never stored.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

constexpr int kFastThreads = 512;
constexpr int kFastImg = 256 * 64 * 2;  // bytes of one operand image (one K-tile)

DTP_DEV int fswz(int x) { return (x & 3) | ((x >> 1) & 4); }

// Per-lane DMA sources of the 4 instructions that fill one operand image:
// instruction i of wave w fills image bytes [(8 i + w) KiB, +1 KiB).
template <bool TRANS>
DTP_DEV void fast_sources(const char* (&src)[4], const char* base, long long ld, int r0, int R, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (!TRANS) {  // 8 rows x 128 B: row (8i+w)*8 + lane/8, physical chunk lane%8
      const int row = (8 * i + wave) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ fswz(row);
      const int rr = min(r0 + row, R - 1);
      src[i] = base + (static_cast<long long>(rr) * ld + c * 8) * 2;
    } else {  // 2 k-rows x 512 B: k = (8i+w)*2 + lane/32, physical chunk lane%32
      const int k = (8 * i + wave) * 2 + (lane >> 5);
      const int c = (lane & 31) ^ (fswz(k) << 1);
      const int col = min(r0 + c * 8, R - 8);
      src[i] = base + (static_cast<long long>(k) * ld + col) * 2;
    }
  }
}

// Byte offsets (inside an image) of this lane's fragment reads.  Row image:
// off[ks] for k-step ks, fragment f adds 2048 f.  k-major image: off[f] for
// fragment f at k-step 0; k-step 1 adds 16384, the upper 4 k of a fragment 2048.
template <bool TRANS, int NF>
DTP_DEV void fast_offsets(int (&off)[TRANS ? NF : 2], int rb, int lane) {
  const int lr = lane & 15, lg = lane >> 4;
  if constexpr (!TRANS) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) off[ks] = ((rb + lr) * 8 + ((4 * ks + lg) ^ fswz(lr))) * 16;
  } else {
    // lane 4q+p of group lg supplies k-row 8 lg + q (+ 32 ks, + 4), columns 4p..4p+3
    const int q = lr >> 2, p = lr & 3, sw = q | ((lg & 1) << 2);
#pragma unroll
    for (int f = 0; f < NF; ++f) off[f] = (8 * lg + q) * 512 + (((rb + 16 * f) * 2) ^ (sw << 5)) + 8 * p;
  }
}

template <bool TRANS>
DTP_DEV bf16x8 fast_frag(const char* img, const int* off, int f, int ks) {
  if constexpr (!TRANS) {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(img + off[ks] + f * 2048));
  } else {
    const char* p = img + off[f] + ks * 16384;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(p));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(p + 2048));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

DTP_DEV void fast_epilogue_lds(const DtpGemmArgs& a, const f32x4 (&acc)[8][4], char* lds, int m0, int n0, int wave,
                               int wr, int wc, int lane) {
  float* buf = reinterpret_cast<float*>(lds) + wave * kEpiWaveFloats;
  const int ncol = n0 + wc * 64 + 8 * (lane & 7);
  const uintptr_t cp = reinterpret_cast<uintptr_t>(a.C), ap = reinterpret_cast<uintptr_t>(a.aux);
  const bool vec = ncol + 8 <= a.N && a.ldc % 8 == 0 && (cp & 15) == 0 && (!a.aux || (a.ldaux % 8 == 0 && (ap & 15) == 0));
  float bias[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) bias[c] = (a.bias && ncol + c < a.N) ? a.bias[ncol + c] : 0.f;
  fast_epilogue_pass<0>(a, acc, buf, bias, m0 + wr * 128, ncol, vec, lane);
  fast_epilogue_pass<1>(a, acc, buf, bias, m0 + wr * 128 + 64, ncol, vec, lane);
}

// Schedule: the next tile's DMA split over the two k-steps (4 pieces ahead of each MFMA
// cluster), per-cluster s_setprio.  The other round-1/2 schedule experiments (static
// priority, unsplit DMA, direct epilogue, one wave per SIMD, the no-DMA / no-MFMA
// diagnostics) lost to this one and were removed in round 3 (profiles/gemm_r1_fast).
// Since round 3 the 8-phase kernel (gemm_ph8.hip) is the default; this one serves the
// shapes it cannot take (a transposed operand spanning >= 4 GiB) and A/B runs.
template <bool TA, bool TB>
__global__ __launch_bounds__(kFastThreads) void gemm_fast_kernel(DtpGemmArgs a) {
  constexpr int BM = 256, BN = 256, BK = 64;
  // [buffer][A | B] images: 128 KiB; after the K loop, 8 waves x 64 x 68 f32 epilogue staging (136 KiB)
  constexpr int kLdsBytes = 2 * 2 * kFastImg > 8 * kEpiWaveFloats * 4 ? 2 * 2 * kFastImg : 8 * kEpiWaveFloats * 4;
  __shared__ __align__(16) char lds[kLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3, lr = lane & 15, lg = lane >> 4;
  const TileId id = decode_tile<BM, BN>(a);
  const int m0 = id.m0, n0 = id.n0, nk = a.K / BK;

  const char* srcA[4];
  const char* srcB[4];
  fast_sources<TA>(srcA, static_cast<const char*>(a.A), a.lda, m0, a.M, wave, lane);
  fast_sources<TB>(srcB, static_cast<const char*>(a.B), a.ldb, n0, a.N, wave, lane);
  const long long kbA = TA ? static_cast<long long>(BK) * a.lda * 2 : BK * 2;
  const long long kbB = TB ? static_cast<long long>(BK) * a.ldb * 2 : BK * 2;
  auto stage = [&](int buf, int kt, int i0, int i1) {
    char* img = lds + buf * 2 * kFastImg;
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(srcA[i] + kt * kbA), (lds_void_t*)(img + (8 * i + wave) * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(srcB[i] + kt * kbB),
                                       (lds_void_t*)(img + kFastImg + (8 * i + wave) * 1024), 16, 0, 0);
    }
  };
  int offA[TA ? 8 : 2], offB[TB ? 4 : 2];
  fast_offsets<TA, 8>(offA, wr * 128, lane);
  fast_offsets<TB, 4>(offB, wc * 64, lane);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0, 0, 4);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) stage(buf ^ 1, kt + 1, 0, 2);
    const char* ia = lds + buf * 2 * kFastImg;
    const char* ib = ia + kFastImg;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = fast_frag<TB>(ib, offB, j, ks);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = fast_frag<TA>(ia, offA, i, ks);
      if (ks == 1 && more) stage(buf ^ 1, kt + 1, 2, 4);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  fast_epilogue_lds(a, acc, lds, m0, n0, wave, wr, wc, lane);
}

int launch_fast(const DtpGemmArgs& a, hipStream_t s) {
  const long long tiles = (long long)((a.M + 255) / 256) * ((a.N + 255) / 256);
  const dim3 gf((unsigned)tiles), bf(kFastThreads);
  switch ((a.trans_a ? 2 : 0) | (a.trans_b ? 1 : 0)) {
    case 0: hipLaunchKernelGGL((gemm_fast_kernel<false, false>), gf, bf, 0, s, a); break;
    case 1: hipLaunchKernelGGL((gemm_fast_kernel<false, true>), gf, bf, 0, s, a); break;
    case 2: hipLaunchKernelGGL((gemm_fast_kernel<true, false>), gf, bf, 0, s, a); break;
    default: hipLaunchKernelGGL((gemm_fast_kernel<true, true>), gf, bf, 0, s, a); break;
  }
  return check_launch("dtp_gemm(LDS-DMA 256x256)");
}


// Skinny-K GEMM (K <= 16): an outer-product-like layer (the first Linear of an MLP,
// K = in_features, and the input gradient of the last one, K = out_features) is
// pure output bandwidth -- write C (and read aux) in 16-byte vectors instead of
// running a 128x128 MFMA tile with 1/16th of its K used.  Block = kSkinnyRows rows x
// 256 columns (the B block staged once per 128 rows, not per 16); thread t owns
// columns 8 (t & 31) .. +8 of rows 2 (t >> 5) + 16 q .. +2, q < kSkinnyRows / 16.
// KC = K at compile time (1, 2: the usual MLP in/out widths; 0 = K read at run time):
// the thread's 8 B columns then live in registers for all of its rows.
constexpr int kSkinnyRows = 128;
template <int DT, bool TA, bool TB, int KC = 0>
__global__ __launch_bounds__(256) void gemm_skinny_k_kernel(DtpGemmArgs a) {
  __shared__ float sa[kSkinnyRows][17];
  __shared__ float sb[256][17];
  const int tid = threadIdx.x;
  const int n0 = blockIdx.x * 256, m0 = blockIdx.y * kSkinnyRows;
  const char* A = static_cast<const char*>(a.A);
  const char* B = static_cast<const char*>(a.B);
  constexpr int ES = Ty<DT>::ES;
  for (int e = tid; e < kSkinnyRows * 16; e += 256) {
    const int r = e >> 4, k = e & 15, m = m0 + r;
    float v = 0.f;
    if (m < a.M && k < a.K) v = load_elem<DT>(A + (TA ? (long long)k * a.lda + m : (long long)m * a.lda + k) * ES);
    sa[r][k] = v;
  }
  for (int e = tid; e < 256 * 16; e += 256) {
    const int c = e >> 4, k = e & 15, n = n0 + c;
    float v = 0.f;
    if (n < a.N && k < a.K) v = load_elem<DT>(B + (TB ? (long long)k * a.ldb + n : (long long)n * a.ldb + k) * ES);
    sb[c][k] = v;
  }
  __syncthreads();
  const int cc = (tid & 31) * 8, rr = (tid >> 5) * 2;
  float bias[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) bias[c] = (a.bias && n0 + cc + c < a.N) ? a.bias[n0 + cc + c] : 0.f;
  char* C = static_cast<char*>(a.C);
  const char* aux = static_cast<const char*>(a.aux);
  const bool vec_c = (a.ldc % 8 == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) && n0 + cc + 8 <= a.N;
  float breg[8][KC > 0 ? KC : 1];
  if constexpr (KC > 0) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int k = 0; k < KC; ++k) breg[c][k] = sb[cc + c][k];
  }
  for (int rq = 0; rq < kSkinnyRows * 2 / 16; ++rq) {
    const int r = rq & 1, lr = rr + r + 16 * (rq >> 1);
    const int m = m0 + lr;
    if (m >= a.M) break;
    float acc[8], v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float t = 0.f;
      if constexpr (KC > 0) {
#pragma unroll
        for (int k = 0; k < KC; ++k) t = fmaf(sa[lr][k], breg[c][k], t);
      } else {
        for (int k = 0; k < a.K; ++k) t = fmaf(sa[lr][k], sb[cc + c][k], t);
      }
      acc[c] = t;
      v[c] = a.alpha * t + bias[c];
    }
    if (vec_c && a.out_dtype == DTP_DT_BF16 && !a.accumulate) {
      if (aux) {
        const uint4 g = *reinterpret_cast<const uint4*>(aux + ((long long)m * a.ldaux + n0 + cc) * ES);
        float gv[8];
        if constexpr (DT == DTP_DT_BF16) {
          const uint32_t w[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            gv[2 * q] = __uint_as_float(w[q] << 16);
            gv[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
          }
        } else {
#pragma unroll
          for (int c = 0; c < 8; ++c) gv[c] = load_elem<DT>(aux + ((long long)m * a.ldaux + n0 + cc + c) * ES);
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] *= leaky_grad_from_out(gv[c], a.slope);
      }
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float x0 = a.act ? leaky(v[2 * q], a.slope) : v[2 * q];
        const float x1 = a.act ? leaky(v[2 * q + 1], a.slope) : v[2 * q + 1];
        o[q] = uint32_t(f32_to_bf16(x0)) | (uint32_t(f32_to_bf16(x1)) << 16);
      }
      *reinterpret_cast<uint4*>(C + ((long long)m * a.ldc + n0 + cc) * 2) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int n = n0 + cc + c;
        if (n < a.N) epilogue_store<DT>(a, C, aux, m, n, acc[c], bias[c]);
      }
    }
  }
}

// out[n] (+)= sum_m X[m*ld + n]: bias gradients.  64 columns x 4 row groups per block,
// kColsumRows rows per block (enough blocks to cover the chip for skinny N), four
// independent loads in flight per thread; row blocks meet in f32 atomics.
constexpr int kColsumRows = 256;
template <int DT>
__global__ __launch_bounds__(256) void colsum_kernel(const void* X, long long ld, int M, int N, float* out) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  const int r0 = blockIdx.y * kColsumRows;
  const int r1 = min(M, r0 + kColsumRows);
  float s = 0.f;
  if (n < N) {
    const char* base = static_cast<const char*>(X);
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    int m = r0 + g;
    for (; m + 12 < r1; m += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        p[u] += load_elem<DT>(base + (static_cast<long long>(m + 4 * u) * ld + n) * Ty<DT>::ES);
    }
    for (; m < r1; m += 4) p[0] += load_elem<DT>(base + (static_cast<long long>(m) * ld + n) * Ty<DT>::ES);
    s = (p[0] + p[1]) + (p[2] + p[3]);
  }
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && n < N) {
    s = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    if (gridDim.y > 1) atomicAdd(out + n, s);
    else out[n] += s;
  }
}

// bf16 column sums with 16-byte loads: a thread owns 8 adjacent columns, 32 threads
// span 256 columns, 8 row groups x 32 rows per block (rows 16-byte aligned, N % 8 == 0).
// 256-row blocks: an [8192 x 4096] gradient is 512 blocks (two per CU) instead of
// 128, and each thread keeps its 4 row loads in flight before adding.
constexpr int kColsumX8Rows = 256;
__global__ __launch_bounds__(256) void colsum_bf16x8_kernel(const void* X, long long ld, int M, int N, float* out) {
  __shared__ float red[8][256];
  const int cc = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int n0 = blockIdx.x * 256 + cc * 8;
  const int r0 = blockIdx.y * kColsumX8Rows;
  const int r1 = min(M, r0 + kColsumX8Rows);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto add = [&](const uint4& v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s[2 * e] += __uint_as_float(w[e] << 16);
      s[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
    }
  };
  if (n0 < N) {
    const uint16_t* base = static_cast<const uint16_t*>(X) + n0;
    int m = r0 + g;
    for (; m + 24 < r1; m += 32) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(base + static_cast<long long>(m + 8 * u) * ld);
#pragma unroll
      for (int u = 0; u < 4; ++u) add(v[u]);
    }
    for (; m < r1; m += 8) add(*reinterpret_cast<const uint4*>(base + static_cast<long long>(m) * ld));
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[g][cc * 8 + e] = s[e];
  __syncthreads();
  const int c = threadIdx.x, n = blockIdx.x * 256 + c;
  if (n < N) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q][c];
    if (gridDim.y > 1) atomicAdd(out + n, t);
    else out[n] += t;
  }
}


// Skinny-output weight gradient (an MLP's first Linear, dW [out, in <= 4], or its last,
// dW [out <= 4, in]): C (+)= alpha A^T B with both operands K-major ([K, M], [K, N]) and
// min(M, N) <= 4 -- the wide operand's column sums weighted by the J skinny columns.
// Pure read bandwidth of the wide operand: a thread owns 8 adjacent wide columns
// (16-byte loads, 4 rows in flight), 8 row groups x 32 rows per block, row blocks meet
// in f32 atomics.  out[w * so + j * sj] for wide index w and skinny index j.
constexpr int kSkinnyOutRows = 256;
template <int J>
__global__ __launch_bounds__(256) void gemm_skinny_out_kernel(const uint16_t* X, long long ldx, const uint16_t* Y,
                                                              long long ldy, int K, int W, float* out, long long so,
                                                              long long sj, float alpha) {
  __shared__ float red[8][256 * J];
  const int cc = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int w0 = blockIdx.x * 256 + cc * 8;
  const int r0 = blockIdx.y * kSkinnyOutRows;
  const int r1 = min(K, r0 + kSkinnyOutRows);
  float s[J][8];
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) s[j][e] = 0.f;
  auto add = [&](const uint4& v, int m) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    float x[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[2 * e] = __uint_as_float(w[e] << 16);
      x[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const float y = bf16_to_f32(Y[static_cast<long long>(m) * ldy + j]);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[j][e] = fmaf(x[e], y, s[j][e]);
    }
  };
  if (w0 < W) {
    const uint16_t* base = X + w0;
    int m = r0 + g;
    for (; m + 24 < r1; m += 32) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(base + static_cast<long long>(m + 8 * u) * ldx);
#pragma unroll
      for (int u = 0; u < 4; ++u) add(v[u], m + 8 * u);
    }
    for (; m < r1; m += 8) add(*reinterpret_cast<const uint4*>(base + static_cast<long long>(m) * ldx), m);
  }
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) red[g][j * 256 + cc * 8 + e] = s[j][e];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int c = threadIdx.x, w = blockIdx.x * 256 + c;
    if (w < W) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) t += red[q][j * 256 + c];
      atomicAdd(out + static_cast<long long>(w) * so + static_cast<long long>(j) * sj, alpha * t);
    }
  }
}

}  // namespace gemm
}  // namespace dtp

using namespace dtp;

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// the 8-phase kernel's preconditions (bf16, whole 64-deep K-tiles, 16-byte aligned rows,
// a transposed operand in whole 8-element chunks); its DMA offsets are 32-bit: a
// transposed operand's K rows, and a K-contiguous operand's 256 tile rows, must span
// < 4 GiB
static bool ph8_shape(const DtpGemmArgs& a) {
  return a.dtype == DTP_DT_BF16 && a.K % 64 == 0 && a.vec_a && a.vec_b && (!a.trans_a || a.M % 8 == 0) &&
         (!a.trans_b || a.N % 8 == 0) && !a.force_big && a.fast >= 0 &&
         (a.trans_a ? a.K * a.lda * 2 : 256 * a.lda * 2) < (1LL << 32) &&
         (a.trans_b ? a.K * a.ldb * 2 : 256 * a.ldb * 2) < (1LL << 32);
}

extern "C" long long dtp_gemm_workspace(const DtpGemmArgs* in) {
  if (!in || in->splitk != 0 || in->M <= 0 || in->N <= 0 || in->K <= 0) return 0;
  DtpGemmArgs a = *in;
  a.vec_a = (a.lda % 8 == 0) && aligned16(a.A);
  a.vec_b = (a.ldb % 8 == 0) && aligned16(a.B);
  if (!ph8_shape(a)) return 0;
  const int sp = gemm::ph8_split_plan(a);
  return sp > 1 ? gemm::ph8_split_bytes(a, sp) : 0;
}

extern "C" int dtp_gemm(const DtpGemmArgs* in, void* stream) {
  if (!in) return set_err(1, "dtp_gemm: null args");
  DtpGemmArgs a = *in;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return set_err(1, "dtp_gemm: empty problem");
  if (a.dtype != DTP_DT_F32 && a.dtype != DTP_DT_BF16) return set_err(1, "dtp_gemm: dtype must be f32 or bf16");
  if (a.out_dtype != DTP_DT_F32 && a.out_dtype != DTP_DT_BF16) return set_err(1, "dtp_gemm: bad out dtype");
  if (!a.A || !a.B || !a.C) return set_err(1, "dtp_gemm: null operand");
  // skinny-output weight gradient: bandwidth kernel over the wide operand (any split-K
  // request is moot: every row block already meets in atomics)
  if (a.dtype == DTP_DT_BF16 && a.trans_a && a.trans_b && a.out_dtype == DTP_DT_F32 && !a.act && !a.aux &&
      !a.bias && (a.M <= 4 || a.N <= 4) && a.K >= 64) {
    const bool wide_a = a.N <= 4;  // dW [out, in <= 4]: A = dz is the wide operand
    const void* X = wide_a ? a.A : a.B;
    const void* Y = wide_a ? a.B : a.A;
    const long long ldx = wide_a ? a.lda : a.ldb, ldy = wide_a ? a.ldb : a.lda;
    const int W = wide_a ? a.M : a.N, J = wide_a ? a.N : a.M;
    if (W % 8 == 0 && ldx % 8 == 0 && aligned16(X)) {
      hipStream_t s = static_cast<hipStream_t>(stream);
      if (!a.accumulate) {
        hipError_t e = hipMemset2DAsync(a.C, sizeof(float) * static_cast<size_t>(a.ldc), 0, sizeof(float) * a.N, a.M, s);
        if (e != hipSuccess) return set_err(2, "dtp_gemm: clearing the skinny-output C failed");
      }
      const long long so = wide_a ? a.ldc : 1, sj = wide_a ? 1 : a.ldc;
      const dim3 g((W + 255) / 256, (a.K + gemm::kSkinnyOutRows - 1) / gemm::kSkinnyOutRows), b(256);
      const auto* Xh = static_cast<const uint16_t*>(X);
      const auto* Yh = static_cast<const uint16_t*>(Y);
      float* C = static_cast<float*>(a.C);
      switch (J) {
        case 1: hipLaunchKernelGGL(gemm::gemm_skinny_out_kernel<1>, g, b, 0, s, Xh, ldx, Yh, ldy, a.K, W, C, so, sj, a.alpha); break;
        case 2: hipLaunchKernelGGL(gemm::gemm_skinny_out_kernel<2>, g, b, 0, s, Xh, ldx, Yh, ldy, a.K, W, C, so, sj, a.alpha); break;
        case 3: hipLaunchKernelGGL(gemm::gemm_skinny_out_kernel<3>, g, b, 0, s, Xh, ldx, Yh, ldy, a.K, W, C, so, sj, a.alpha); break;
        default: hipLaunchKernelGGL(gemm::gemm_skinny_out_kernel<4>, g, b, 0, s, Xh, ldx, Yh, ldy, a.K, W, C, so, sj, a.alpha); break;
      }
      return check_launch("dtp_gemm(skinny output)");
    }
  }
  const bool auto_split = a.splitk == 0;  // 0: the 8-phase split-K plan when it applies, else no split
  if (a.splitk < 1) a.splitk = 1;
  if (a.splitk > 1 && (a.out_dtype != DTP_DT_F32 || a.act || a.aux))
    return set_err(1, "dtp_gemm: split-K needs an f32 output and no activation epilogue");
  const int epc = a.dtype == DTP_DT_BF16 ? 8 : 4;
  a.vec_a = (a.lda % epc == 0) && aligned16(a.A);
  a.vec_b = (a.ldb % epc == 0) && aligned16(a.B);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (auto_split && ph8_shape(a)) {
    const int sp = gemm::ph8_split_plan(a);
    if (sp > 1 && a.work && a.work_bytes >= gemm::ph8_split_bytes(a, sp)) {
      a.splitk = sp;
      return gemm::launch_ph8(a, s, -1);
    }
  }
  const int tm = (a.M + gemm::kBM - 1) / gemm::kBM, tn = (a.N + gemm::kBN - 1) / gemm::kBN;
  const int bk = a.dtype == DTP_DT_BF16 ? 64 : 32;
  const int ktiles = (a.K + bk - 1) / bk;
  if (a.splitk > ktiles) a.splitk = ktiles;
  if (a.splitk > 1 && !a.accumulate) {  // atomics accumulate into C: clear it first
    hipError_t e = hipMemset2DAsync(a.C, sizeof(float) * static_cast<size_t>(a.ldc), 0, sizeof(float) * a.N, a.M, s);
    if (e != hipSuccess) return set_err(2, "dtp_gemm: clearing the split-K output failed");
  }
  // K <= 16 (an MLP's first layer / last layer's input gradient): output-bandwidth kernel
  if (a.K <= 16 && a.splitk == 1) {
    const dim3 gs((a.N + 255) / 256, (a.M + gemm::kSkinnyRows - 1) / gemm::kSkinnyRows), bs(256);
    const int k3 = (a.dtype == DTP_DT_BF16 ? 4 : 0) | (a.trans_a ? 2 : 0) | (a.trans_b ? 1 : 0);
    switch (k3) {
      case 0: hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_F32, false, false>), gs, bs, 0, s, a); break;
      case 1: hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_F32, false, true>), gs, bs, 0, s, a); break;
      case 2: hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_F32, true, false>), gs, bs, 0, s, a); break;
      case 3: hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_F32, true, true>), gs, bs, 0, s, a); break;
      case 4:
        if (a.K == 2) hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_BF16, false, false, 2>), gs, bs, 0, s, a);
        else if (a.K == 1) hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_BF16, false, false, 1>), gs, bs, 0, s, a);
        else hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_BF16, false, false>), gs, bs, 0, s, a);
        break;
      case 5:
        if (a.K == 1) hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_BF16, false, true, 1>), gs, bs, 0, s, a);
        else if (a.K == 2) hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_BF16, false, true, 2>), gs, bs, 0, s, a);
        else hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_BF16, false, true>), gs, bs, 0, s, a);
        break;
      case 6: hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_BF16, true, false>), gs, bs, 0, s, a); break;
      default: hipLaunchKernelGGL((gemm::gemm_skinny_k_kernel<DTP_DT_BF16, true, true>), gs, bs, 0, s, a); break;
    }
    return check_launch("dtp_gemm(skinny K)");
  }
  // big bf16 problems (>= 256 tiles of 256x256, no split-K): the 256x256 kernel
  const long long big_tiles = (long long)((a.M + 255) / 256) * ((a.N + 255) / 256);
  // the LDS-DMA 256x256 kernel: whole 64-deep K tiles, 16-byte aligned rows, a
  // transposed operand in whole 8-element chunks; by default once there are
  // enough 256x256 tiles to occupy half the chip's CUs
  const bool fast_shape = a.dtype == DTP_DT_BF16 && a.splitk == 1 && a.K % 64 == 0 && a.vec_a && a.vec_b &&
                          (!a.trans_a || a.M % 8 == 0) && (!a.trans_b || a.N % 8 == 0) && !a.force_big;
  if (fast_shape && a.fast >= 0 && (a.fast > 0 || big_tiles >= 128)) {
    // default: the 8-phase kernel (gemm_ph8.hip)
    if (a.fast < 2 && ph8_shape(a)) return gemm::launch_ph8(a, s, -1);
    // fast = 2 + variant pins a kernel (A/B runs, tests): 32 / 34 the 8-phase schedules,
    // anything else the two-buffer kernel
    switch (a.fast - 2) {
      case 32: return gemm::launch_ph8(a, s, 0);  // 8-phase, balanced reads (gemm_ph8.hip)
      case 34: return gemm::launch_ph8(a, s, 2);  // 8-phase, reads 12/4/8/0 per phase
      case 35: return gemm::launch_ph8(a, s, 3);  // 8-phase balanced, persistent tile walk
      default: return gemm::launch_fast(a, s);    // two-buffer LDS-DMA kernel
    }
  }
  // lean loads need every row 16-byte aligned and whole 8-element chunks
  const bool lean = a.vec_a && a.vec_b && (a.trans_a ? a.M : a.K) % 8 == 0 && (a.trans_b ? a.N : a.K) % 8 == 0;
  // measured (scripts/bench_gemm.py): it beats the 128x128 kernel only with both
  // operands K-contiguous and >= 2 waves of 256 CUs (8192^2: 790 vs 720 TF/s); its
  // one-wave-per-SIMD register-transpose staging loses on transposed operands
  const bool big_ok = a.dtype == DTP_DT_BF16 && a.splitk == 1 && big_tiles >= 512 && a.K >= 256 && lean &&
                      (a.force_big || (!a.trans_a && !a.trans_b));
  if (big_ok) {
    const dim3 gb((unsigned)big_tiles), bb(gemm::kThreads);
    const int kb = (a.trans_a ? 2 : 0) | (a.trans_b ? 1 : 0);
    switch (kb) {
      case 0: hipLaunchKernelGGL((gemm::gemm_big_kernel<false, false>), gb, bb, 0, s, a); break;
      case 1: hipLaunchKernelGGL((gemm::gemm_big_kernel<false, true>), gb, bb, 0, s, a); break;
      case 2: hipLaunchKernelGGL((gemm::gemm_big_kernel<true, false>), gb, bb, 0, s, a); break;
      default: hipLaunchKernelGGL((gemm::gemm_big_kernel<true, true>), gb, bb, 0, s, a); break;
    }
    return check_launch("dtp_gemm(256x256)");
  }
  const dim3 grid(tm * tn * a.splitk), block(gemm::kThreads);
  const int key = (a.dtype == DTP_DT_BF16 ? 4 : 0) | (a.trans_a ? 2 : 0) | (a.trans_b ? 1 : 0);
  switch (key) {
    case 0: hipLaunchKernelGGL((gemm::gemm_kernel<DTP_DT_F32, false, false>), grid, block, 0, s, a); break;
    case 1: hipLaunchKernelGGL((gemm::gemm_kernel<DTP_DT_F32, false, true>), grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((gemm::gemm_kernel<DTP_DT_F32, true, false>), grid, block, 0, s, a); break;
    case 3: hipLaunchKernelGGL((gemm::gemm_kernel<DTP_DT_F32, true, true>), grid, block, 0, s, a); break;
    case 4: hipLaunchKernelGGL((gemm::gemm_kernel<DTP_DT_BF16, false, false>), grid, block, 0, s, a); break;
    case 5: hipLaunchKernelGGL((gemm::gemm_kernel<DTP_DT_BF16, false, true>), grid, block, 0, s, a); break;
    case 6: hipLaunchKernelGGL((gemm::gemm_kernel<DTP_DT_BF16, true, false>), grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL((gemm::gemm_kernel<DTP_DT_BF16, true, true>), grid, block, 0, s, a); break;
  }
  return check_launch("dtp_gemm");
}

extern "C" int dtp_colsum(const void* X, long long ld, int M, int N, int dtype, float* out, int accumulate,
                          void* stream) {
  if (!X || !out || M <= 0 || N <= 0) return set_err(1, "dtp_colsum: bad arguments");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (!accumulate) (void)hipMemsetAsync(out, 0, sizeof(float) * N, s);
  if (dtype == DTP_DT_BF16 && N % 8 == 0 && ld % 8 == 0 && aligned16(X)) {
    hipLaunchKernelGGL(gemm::colsum_bf16x8_kernel, dim3((N + 255) / 256, (M + gemm::kColsumX8Rows - 1) / gemm::kColsumX8Rows),
                       dim3(256), 0, s, X, ld, M, N, out);
    return check_launch("dtp_colsum(bf16x8)");
  }
  const dim3 grid((N + 63) / 64, (M + gemm::kColsumRows - 1) / gemm::kColsumRows), block(256);
  if (dtype == DTP_DT_BF16)
    hipLaunchKernelGGL((gemm::colsum_kernel<DTP_DT_BF16>), grid, block, 0, s, X, ld, M, N, out);
  else
    hipLaunchKernelGGL((gemm::colsum_kernel<DTP_DT_F32>), grid, block, 0, s, X, ld, M, N, out);
  return check_launch("dtp_colsum");
}
