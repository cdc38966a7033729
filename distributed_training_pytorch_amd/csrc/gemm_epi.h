// Shared pieces of the MFMA GEMM kernels (gemm.hip, gemm_ph8.hip): bf16 helpers,
// the per-element fused epilogue, and the LDS-staged vector epilogue of the 256x256
// tiles (one wave's 64-row x 64-column slab of f32 accumulators written back as
// 16-byte rows with bias / LeakyReLU / LeakyReLU'(aux) / accumulate fused).
#pragma once

#include "dtp_api.h"
#include "dtp_common.h"

namespace dtp {
namespace gemm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int DT>
struct Ty {
  static constexpr int ES = DT == DTP_DT_BF16 ? 2 : 4;  // element bytes
  static constexpr int EPC = 16 / ES;                    // elements per 16-byte chunk
  static constexpr int BK = 128 / ES;                    // K per tile (one LDS row)
};

DTP_DEV float bf16_to_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }
DTP_DEV uint16_t f32_to_bf16(float f) {  // round to nearest even
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return uint16_t((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
  u += 0x7fffu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

template <int DT>
DTP_DEV float load_elem(const char* p) {
  if constexpr (DT == DTP_DT_BF16) return bf16_to_f32(*reinterpret_cast<const uint16_t*>(p));
  else return *reinterpret_cast<const float*>(p);
}

// tile decode shared by the GEMM kernels: XCD-aware remap (workgroups are dealt
// round-robin over the 8 XCDs: consecutive tile ids land on one XCD's L2), then
// 8-row groups of M tiles, split-K innermost
struct TileId {
  int m0, n0, ks;
};
// (b, nb): the tile id and the id count -- a workgroup's blockIdx.x / gridDim.x, or a
// persistent workgroup's current tile of all tiles (its XCD is b & 7 whenever the grid
// is a multiple of 8, so its tiles stay in its XCD's range)
template <int BMT, int BNT>
DTP_DEV TileId decode_tile_at(const DtpGemmArgs& a, int b, int nb) {
  const int tm = (a.M + BMT - 1) / BMT, tn = (a.N + BNT - 1) / BNT;
  if ((nb & 7) == 0) b = (b & 7) * (nb >> 3) + (b >> 3);
  TileId id;
  id.ks = b % a.splitk;
  const int t = b / a.splitk;
  const int group = t / (8 * tn), first_m = group * 8;
  const int gsz = min(tm - first_m, 8);
  id.m0 = (first_m + (t % (8 * tn)) % gsz) * BMT;
  id.n0 = ((t % (8 * tn)) / gsz) * BNT;
  return id;
}
template <int BMT, int BNT>
DTP_DEV TileId decode_tile(const DtpGemmArgs& a) {
  return decode_tile_at<BMT, BNT>(a, blockIdx.x, gridDim.x);
}


// fused epilogue of one output element
template <int DT>
DTP_DEV void epilogue_store(const DtpGemmArgs& a, char* C, const char* aux, int m, int n, float acc, float bias) {
  float v = a.alpha * acc + bias;
  if (aux) v *= leaky_grad_from_out(load_elem<DT>(aux + (static_cast<long long>(m) * a.ldaux + n) * Ty<DT>::ES),
                                    a.slope);
  if (a.act) v = leaky(v, a.slope);
  const long long off = static_cast<long long>(m) * a.ldc + n;
  if (a.out_dtype == DTP_DT_BF16) {
    uint16_t* p = reinterpret_cast<uint16_t*>(C) + off;
    if (a.accumulate) v += bf16_to_f32(*p);
    *p = f32_to_bf16(v);
  } else {
    float* p = reinterpret_cast<float*>(C) + off;
    if (a.splitk > 1) {
      atomicAdd(p, v);
    } else {
      if (a.accumulate) v += *p;
      *p = v;
    }
  }
}

// LDS-staged epilogue of the 256x256 LDS-DMA kernel (the operand images are dead
// once the K loop ends).  The MFMA layout gives a lane one column and 4 rows per
// fragment, so a direct store writes 2-4 bytes per lane and the aux / accumulate
// operands come back one scalar load at a time.  Instead each wave parks its
// 128x64 f32 sub-tile in its own LDS region, 64 rows per pass (row stride 68
// floats: the ds_write_b32 of one fragment register hits 64 distinct banks), and
// reads it back row-major: lane L owns 8 adjacent columns 8 (L & 7) .. +8 of rows
// L / 8 + 8 t, so aux, the old C (accumulate) and C itself move as 16-byte vectors
// (8 lanes = one 128-byte bf16 row segment).  Columns past N (ragged last tile) or
// unaligned operands take the per-element path.
constexpr int kEpiStride = 68;
constexpr int kEpiWaveFloats = 64 * kEpiStride;

DTP_DEV void bf16x8_to_f32(const uint4& g, float (&x)[8]) {
  const uint32_t w[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    x[2 * q] = __uint_as_float(w[q] << 16);
    x[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}

// one pass = fragment rows 4H .. 4H+3 (H a template parameter: acc is indexed
// statically, so it stays in registers)
// (J0: first of the 4 fragment columns staged, for waves holding more than 4)
// ROWS (64 or 16): rows staged per pass -- 16 = one fragment row (II0) of the row half,
// a quarter of the LDS staging (the persistent GEMM stages while the next tile's operands
// stream into the rest of LDS); row0 is then the fragment row's first row
template <int H, int J0 = 0, int NJ = 4, int ROWS = 64, int II0 = 0>
DTP_DEV void fast_epilogue_pass(const DtpGemmArgs& a, const f32x4 (&acc)[8][NJ], float* buf, const float (&bias)[8],
                                int row0, int ncol, bool vec, int lane) {
  static_assert(ROWS == 64 || ROWS == 16, "64- or 16-row passes");
  constexpr int NII = ROWS / 16, NU = ROWS / 8 < 4 ? ROWS / 8 : 4;
  const int lr = lane & 15, lg = lane >> 4, c8 = lane & 7, rl = lane >> 3;
  char* C = static_cast<char*>(a.C);
  const uint16_t* aux = static_cast<const uint16_t*>(a.aux);
  const bool bf16_out = a.out_dtype == DTP_DT_BF16;
  constexpr int h = H;
  {
#pragma unroll
    for (int ii = 0; ii < NII; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          buf[(16 * ii + 4 * lg + r) * kEpiStride + 16 * j + lr] = acc[4 * h + II0 + ii][J0 + j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's stores land before its own reads (LDS is in order per wave)
#pragma unroll
    for (int t0 = 0; t0 < ROWS / 8; t0 += NU) {
      float v[NU][8];
      int mrow[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int lrow = rl + 8 * (t0 + u);
        mrow[u] = row0 + lrow;
        const float4 x0 = *reinterpret_cast<const float4*>(buf + lrow * kEpiStride + 8 * c8);
        const float4 x1 = *reinterpret_cast<const float4*>(buf + lrow * kEpiStride + 8 * c8 + 4);
        const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int c = 0; c < 8; ++c) v[u][c] = xs[c];
      }
      if (vec) {
        // every operand of the 4 rows requested before any is used (rows past M clamped, never stored)
        uint4 g[NU], oc[NU][2];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const long long mr = min(mrow[u], a.M - 1);
          if (aux) g[u] = *reinterpret_cast<const uint4*>(aux + mr * a.ldaux + ncol);
          if (a.accumulate) {
            if (bf16_out) {
              oc[u][0] = *reinterpret_cast<const uint4*>(C + (mr * a.ldc + ncol) * 2);
            } else {
              oc[u][0] = *reinterpret_cast<const uint4*>(C + (mr * a.ldc + ncol) * 4);
              oc[u][1] = *reinterpret_cast<const uint4*>(C + (mr * a.ldc + ncol + 4) * 4);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          float y[8];
#pragma unroll
          for (int c = 0; c < 8; ++c) y[c] = a.alpha * v[u][c] + bias[c];
          if (aux) {
            float gv[8];
            bf16x8_to_f32(g[u], gv);
#pragma unroll
            for (int c = 0; c < 8; ++c) y[c] *= leaky_grad_from_out(gv[c], a.slope);
          }
          if (a.act) {
#pragma unroll
            for (int c = 0; c < 8; ++c) y[c] = leaky(y[c], a.slope);
          }
          if (mrow[u] >= a.M) continue;
          const long long off = static_cast<long long>(mrow[u]) * a.ldc + ncol;
          if (bf16_out) {
            if (a.accumulate) {
              float ov[8];
              bf16x8_to_f32(oc[u][0], ov);
#pragma unroll
              for (int c = 0; c < 8; ++c) y[c] += ov[c];
            }
            uint32_t o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = uint32_t(f32_to_bf16(y[2 * q])) | (uint32_t(f32_to_bf16(y[2 * q + 1])) << 16);
            *reinterpret_cast<uint4*>(C + off * 2) = make_uint4(o[0], o[1], o[2], o[3]);
          } else {
            if (a.accumulate) {
              const uint32_t w[8] = {oc[u][0].x, oc[u][0].y, oc[u][0].z, oc[u][0].w,
                                     oc[u][1].x, oc[u][1].y, oc[u][1].z, oc[u][1].w};
#pragma unroll
              for (int c = 0; c < 8; ++c) y[c] += __uint_as_float(w[c]);
            }
            *reinterpret_cast<float4*>(C + off * 4) = make_float4(y[0], y[1], y[2], y[3]);
            *reinterpret_cast<float4*>(C + (off + 4) * 4) = make_float4(y[4], y[5], y[6], y[7]);
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          if (mrow[u] >= a.M) continue;
#pragma unroll
          for (int c = 0; c < 8; ++c)
            if (ncol + c < a.N)
              epilogue_store<DTP_DT_BF16>(a, C, static_cast<const char*>(a.aux), mrow[u], ncol + c, v[u][c], bias[c]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of this pass done before the next pass overwrites
  }
}

// the 8-phase LDS-DMA 256x256 kernel (gemm_ph8.hip); variant 0 staggered, 1 lockstep
int launch_ph8(const DtpGemmArgs& a, hipStream_t s, int variant);
int ph8_split_plan(const DtpGemmArgs& a);
long long ph8_split_bytes(const DtpGemmArgs& a, int splitk);

}  // namespace gemm
}  // namespace dtp
