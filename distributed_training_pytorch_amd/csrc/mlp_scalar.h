// Weight layouts and per-layer building blocks of the fused train step
// (mlp_train.hip, mlp_pipe.h): one lane per sample.
//
//   * LDS forward block of layer l: W_l^T [in][pad4(out)] then bias [pad4(out)], so
//     consecutive outputs (j, j+1) of one input i are adjacent and
//     z[j:j+1] += W^T[i][j:j+1] * h_i is one v_pk_fma_f32 straight from a broadcast
//     ds_read_b128;
//   * LDS backward block of layer l >= 1: W_l [out][pad4(in)] (the torch layout,
//     rows padded), so g[i:i+1] += W[j][i:i+1] * dz_j is one v_pk_fma_f32;
//   * pad entries are zero and are never written by the optimizer;
//   * the dW tiles: per-wave staging of (dz, h) columns and 16 MFMA K-steps per tile,
//     the first and last layers packed into one tile when they fit.
// The round-1 variant that streamed the forward weights through SGPRs (s_load from
// a global workspace) measured slower than the LDS blocks and was removed in round 2
// (docs/perf_notes.md, v3); the workspace size query (WS) stays as the shape check.
#pragma once
#include <type_traits>

#include "mlp_core.h"

namespace dtp {

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <class S>
struct Scal {
  static constexpr int NL = S::NL;
  static constexpr int pad2(int x) { return (x + 1) & ~1; }
  static constexpr int FT(int l) { return S::din(l) * pad2(S::dout(l)) + pad2(S::dout(l)); }
  static constexpr int fwo(int l) {
    int o = 0;
    for (int k = 0; k < l; ++k) o += FT(k);
    return o;
  }
  static constexpr int fbo(int l) { return fwo(l) + S::din(l) * pad2(S::dout(l)); }
  static constexpr int LF = fwo(NL);
  // per-model global workspace (forward blocks only), 64-float (256 B) aligned;
  // 64-byte scalar-cache lines it spans
  static constexpr int WS = (LF + 63) & ~63;
  static constexpr int NLINES = (LF + 15) / 16;
  // backward blocks live in LDS: W_l [out][pad4(in)], read as broadcast ds_read_b128
  static constexpr int pad4(int x) { return (x + 3) & ~3; }
  static constexpr int lbo(int l) {
    int o = 0;
    for (int k = 1; k < l; ++k) o += S::dout(k) * pad4(S::din(k));
    return o;
  }
  static constexpr int LB = lbo(NL) > 0 ? lbo(NL) : 4;
  // forward blocks in LDS: W_l^T [in][pad4(out)] then bias [pad4(out)]
  static constexpr int FT4(int l) { return S::din(l) * pad4(S::dout(l)) + pad4(S::dout(l)); }
  static constexpr int lfo(int l) {
    int o = LB;
    for (int k = 0; k < l; ++k) o += FT4(k);
    return o;
  }
  static constexpr int lfb(int l) { return lfo(l) + S::din(l) * pad4(S::dout(l)); }
  static constexpr int LW = lfo(NL);  // all weight blocks in LDS
  // MFMA tiles: first + last layer (and the loss row) packed into one tile when they fit
  static constexpr int O0 = S::dout(0);
  static constexpr int IL = S::din(NL - 1);
  static constexpr bool PACK = NL >= 2 && (O0 + S::OUT + 1 <= 16) && (S::IN + 1 + IL + 1 <= 16);
  static constexpr int NT = PACK ? NL - 1 : NL;
  static constexpr int tile(int l) { return PACK ? (l == NL - 1 ? 0 : l) : l; }
  static constexpr int rowoff(int l) { return (PACK && l == NL - 1) ? O0 : 0; }
  static constexpr int coloff(int l) { return (PACK && l == NL - 1) ? S::IN + 1 : 0; }
  static constexpr int lossrow() { return rowoff(NL - 1) + S::OUT; }
  static constexpr int losscol() { return coloff(NL - 1) + S::din(NL - 1); }  // last layer's bias column
  // a parked dW tile (cross-wave reduction): column-major, column stride 20 floats, so a
  // lane's 4 accumulator rows are one conflict-free ds_write_b128 (8 lanes of one column
  // quarter hit 8 distinct 4-bank windows)
  static constexpr int TSZ = 16 * 20;
  static constexpr int tslot(int row, int col) { return col * 20 + row; }
  static constexpr int losspos() { return tile(NL - 1) * TSZ + tslot(lossrow(), losscol()); }
  static_assert(S::OUT + 1 <= 16, "the loss row must fit under the output rows");
};

// positions of torch-order parameter p: pf in the global forward workspace, pb in
// the LDS backward blocks (-1: biases, layer-0 weights), tpos in the dW tiles
template <class S>
DTP_DEV void scal_pos(int p, int& pf, int& pb, int& tpos, int& pfl) {
  using SC = Scal<S>;
  pfl = 0;
  pf = 0;
  pb = -1;
  tpos = 0;
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l);
    constexpr int base = SC::tile(l) * SC::TSZ, ro = SC::rowoff(l), co = SC::coloff(l);
    if (p >= S::gw(l) && p < S::gb(l)) {
      const int q = p - S::gw(l), j = q / I, i = q - j * I;
      pf = SC::fwo(l) + i * SC::pad2(O) + j;
      if constexpr (l >= 1) pb = SC::lbo(l) + j * SC::pad4(I) + i;
      pfl = SC::lfo(l) + i * SC::pad4(O) + j;
      tpos = base + SC::tslot(ro + j, co + i);
    } else if (p >= S::gb(l) && p < S::gb(l) + O) {
      const int j = p - S::gb(l);
      pf = SC::fbo(l) + j;
      pfl = SC::lfb(l) + j;
      tpos = base + SC::tslot(ro + j, co + I);  // bias column = constant-1 input
    }
  });
}

// q-th float4 of a row of N valid floats (row padded to 4): when only 2 floats of the
// last float4 are valid it is read as a b64 (LDS reads cost by bytes: a 10-float
// row costs 2.5 b128 instead of 3)
template <int N, int Q>
DTP_DEV float4 row_quad(const float* __restrict__ p) {
  if constexpr (4 * Q + 2 >= N) {
    const float2 t = *reinterpret_cast<const float2*>(p + 4 * Q);
    return make_float4(t.x, t.y, 0.f, 0.f);
  } else {
    return *reinterpret_cast<const float4*>(p + 4 * Q);
  }
}

// forward of one sample from the LDS forward blocks: each layer's whole W^T block
// (+ bias) is pulled out with broadcast ds_read_b128 (all in flight; LDS returns in
// order, so the FMAs start as the first rows land), then consumed input-major:
// every output pair is an independent v_pk_fma_f32 chain.
template <class S>
DTP_DEV void lds_forward(const float* __restrict__ wl, float (&h)[S::NL + 1][16], float slope) {
  using SC = Scal<S>;
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l), OP = SC::pad4(O), NQ = OP / 4;
    float4 bq[NQ];
    float4 w4[I][NQ];
    static_for<0, NQ>([&](auto QC) {
      constexpr int q = decltype(QC)::value;
      bq[q] = row_quad<O, q>(wl + SC::lfb(l));
    });
    static_for<0, I>([&](auto IC) {
      constexpr int i = decltype(IC)::value;
      static_for<0, NQ>([&](auto QC) {
        constexpr int q = decltype(QC)::value;
        w4[i][q] = row_quad<O, q>(wl + SC::lfo(l) + i * OP);
      });
    });
    f32x2 z[2 * NQ];
    static_for<0, NQ>([&](auto QC) {
      constexpr int q = decltype(QC)::value;
      z[2 * q] = f32x2{bq[q].x, bq[q].y};
      z[2 * q + 1] = f32x2{bq[q].z, bq[q].w};
    });
    static_for<0, I>([&](auto IC) {
      constexpr int i = decltype(IC)::value;
      const f32x2 hi = f32x2{h[l][i], h[l][i]};
      static_for<0, NQ>([&](auto QC) {
        constexpr int q = decltype(QC)::value;
        if constexpr (4 * q < O) z[2 * q] = __builtin_elementwise_fma(f32x2{w4[i][q].x, w4[i][q].y}, hi, z[2 * q]);
        if constexpr (4 * q + 2 < O)
          z[2 * q + 1] = __builtin_elementwise_fma(f32x2{w4[i][q].z, w4[i][q].w}, hi, z[2 * q + 1]);
      });
    });
    static_for<0, O>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      const float v = (j & 1) ? z[j / 2].y : z[j / 2].x;
      h[l + 1][j] = S::rnd(S::act(l) ? leaky(S::rnd(v), slope) : v);
    });
  });
}

// input gradient of layer l >= 1 for one sample: dz_{l-1} = (W_l^T dz_l) * act'(h_l).
// The layer's whole row-major block is pulled out of LDS first (broadcast
// ds_read_b128, all in flight at once: LDS returns in order, so the FMAs start
// as soon as the first rows land), then consumed output-major with input pairs
// as independent v_pk_fma_f32 chains.
// MFMA interleave: a wave issues in order, and each v_mfma_f32_16x16x4_f32 holds
// the MFMA pipe for 32 cycles, so the caller's NK MFMA K-steps are spread one or
// two per weight row -- between two MFMAs the wave issues that row's ~5 FMAs
// (the sched_group_barrier pipeline pins the MFMA/VALU alternation), and the
// layer costs ~NK x 32 cycles instead of MFMA time + FMA time.
template <class S, int l, int NK, class MfmaK>
DTP_DEV void lds_backward_dx(const float* __restrict__ wl, const float (&h)[S::NL + 1][16], float (&dz)[16],
                             float slope, MfmaK&& mfma_k) {
  using SC = Scal<S>;
  constexpr int I = S::din(l), O = S::dout(l), IP = SC::pad4(I), NQ = IP / 4;
  float4 w4[O][NQ];
  static_for<0, O>([&](auto JC) {
    constexpr int j = decltype(JC)::value;
    static_for<0, NQ>([&](auto QC) {
      constexpr int q = decltype(QC)::value;
      w4[j][q] = row_quad<I, q>(wl + SC::lbo(l) + j * IP);
    });
  });
  f32x2 g[2 * NQ];
  static_for<0, 2 * NQ>([&](auto QC) { g[decltype(QC)::value] = f32x2{0.f, 0.f}; });
  static_for<0, O>([&](auto JC) {
    constexpr int j = decltype(JC)::value;
    constexpr int k0 = NK * j / O, k1 = NK * (j + 1) / O;
    static_for<k0, k1>([&](auto KC) { mfma_k(KC); });
    const f32x2 d = f32x2{dz[j], dz[j]};
    static_for<0, NQ>([&](auto QC) {
      constexpr int q = decltype(QC)::value;
      if constexpr (4 * q < I) g[2 * q] = __builtin_elementwise_fma(f32x2{w4[j][q].x, w4[j][q].y}, d, g[2 * q]);
      if constexpr (4 * q + 2 < I)
        g[2 * q + 1] = __builtin_elementwise_fma(f32x2{w4[j][q].z, w4[j][q].w}, d, g[2 * q + 1]);
    });
    if constexpr (k1 > k0) {
      constexpr int nv = (I + 1) / 2;  // this row's v_pk_fma_f32 count
      static_for<k0, k1>([&](auto) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, nv / (k1 - k0), 0);     // then VALU
      });
    }
  });
  static_for<0, I>([&](auto IC) {
    constexpr int i = decltype(IC)::value;
    const float v = (i & 1) ? g[i / 2].y : g[i / 2].x;
    dz[i] = S::rnd(S::rnd(v) * (S::act(l - 1) ? leaky_grad_from_out(h[l][i], slope) : 1.f));
  });
}

// the wave's MFMA operands of one staged tile (see wave_outer_acc): 16 K-steps
struct TileOps {
  float4 a[4], b[4];
};
DTP_DEV TileOps tile_ops(const float* __restrict__ dzb, const float* __restrict__ hb, int lane) {
  const int off = (lane >> 4) * kStgQ + (lane & 15) * 16;
  TileOps t;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    t.a[i] = reinterpret_cast<const float4*>(dzb + off)[i];
    t.b[i] = reinterpret_cast<const float4*>(hb + off)[i];
  }
  return t;
}
// one K-step of the tile on two alternating accumulators
template <int K>
DTP_DEV void tile_kstep(const TileOps& t, f32x4& acc0, f32x4& acc1) {
  const float4& a = t.a[K / 4];
  const float4& b = t.b[K / 4];
  const float av = (K % 4 == 0) ? a.x : (K % 4 == 1) ? a.y : (K % 4 == 2) ? a.z : a.w;
  const float bv = (K % 4 == 0) ? b.x : (K % 4 == 1) ? b.y : (K % 4 == 2) ? b.z : b.w;
  if constexpr (K & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc1, 0, 0, 0);
  else acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc0, 0, 0, 0);
}

// K-steps [K0, K1) of the tile on two alternating accumulators
template <int K0, int K1>
DTP_DEV void tile_ksteps(const TileOps& t, f32x4& acc0, f32x4& acc1) {
  static_for<K0, K1>([&](auto KC) {
    constexpr int k = decltype(KC)::value;
    const float4& a = t.a[k / 4];
    const float4& b = t.b[k / 4];
    const float av = (k % 4 == 0) ? a.x : (k % 4 == 1) ? a.y : (k % 4 == 2) ? a.z : a.w;
    const float bv = (k % 4 == 0) ? b.x : (k % 4 == 1) ? b.y : (k % 4 == 2) ? b.z : b.w;
    if constexpr (k & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc1, 0, 0, 0);
    else acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc0, 0, 0, 0);
  });
}

// staging helper: write columns [c0, c0+n) of this lane's row (v1 [q][col][t] layout)
template <int N>
DTP_DEV void stage_cols(float* __restrict__ buf, int lane, int c0, const float (&v)[16]) {
  float* p = buf + (lane & 3) * kStgQ + (lane >> 2) + c0 * 16;
#pragma unroll
  for (int c = 0; c < N; ++c) p[c * 16] = v[c];
}

DTP_DEV void stage_one(float* __restrict__ buf, int lane, int col, float v) {
  buf[(lane & 3) * kStgQ + (lane >> 2) + col * 16] = v;
}

// ---- bf16 compute (Stage<..., BF = true>): the dW tiles on v_mfma_f32_16x16x32_bf16 ----
// A staged operand is [column][sample] bf16, column stride kBfStride (64 samples + 8 pad:
// 144 B, so the 16 columns one ds_read_b128 group reads start on distinct banks).  The
// MFMA reader, lane l = (g = l>>4, c = l&15), finds samples 32m + 8g .. +7 of column c
// contiguous: one ds_read_b128 per K-step.  The writer (lane = sample) stores one bf16
// per column; values are already bf16-rounded (Stage::rnd), so the conversion is the
// top half of the float.  A tile over a wave's 64 samples is TWO K = 32 steps (the f32
// path needs 16 K = 4 steps, 32 cycles each: the bf16 instance's dW costs 1/16 of it).
constexpr int kBfStride = 72;
static_assert(16 * kBfStride / 2 <= kStgArr, "a bf16 staged operand fits the f32 staging array");
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

template <int N>
DTP_DEV void stage_cols_bf(float* __restrict__ buf, int lane, int c0, const float (&v)[16]) {
  unsigned short* p = reinterpret_cast<unsigned short*>(buf) + c0 * kBfStride + lane;
#pragma unroll
  for (int c = 0; c < N; ++c) p[c * kBfStride] = (unsigned short)(__float_as_uint(v[c]) >> 16);
}

DTP_DEV void stage_one_bf(float* __restrict__ buf, int lane, int col, float v) {
  reinterpret_cast<unsigned short*>(buf)[col * kBfStride + lane] = (unsigned short)(__float_as_uint(v) >> 16);
}

struct TileOpsBf {
  u32x4_t a[2], b[2];
};
DTP_DEV TileOpsBf tile_ops_bf(const float* __restrict__ dzb, const float* __restrict__ hb, int lane) {
  const int off = (lane & 15) * kBfStride + 8 * (lane >> 4);
  const unsigned short* pa = reinterpret_cast<const unsigned short*>(dzb) + off;
  const unsigned short* pb = reinterpret_cast<const unsigned short*>(hb) + off;
  TileOpsBf t;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    t.a[m] = *reinterpret_cast<const u32x4_t*>(pa + 32 * m);
    t.b[m] = *reinterpret_cast<const u32x4_t*>(pb + 32 * m);
  }
  return t;
}
template <int K>
DTP_DEV void tile_kstep(const TileOpsBf& t, f32x4& acc0, f32x4& acc1) {
  const bf16x8_t a = __builtin_bit_cast(bf16x8_t, t.a[K]), b = __builtin_bit_cast(bf16x8_t, t.b[K]);
  if constexpr (K & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc1, 0, 0, 0);
  else acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc0, 0, 0, 0);
}
DTP_DEV f32x4 wave_outer_acc_bf(const float* __restrict__ dzb, const float* __restrict__ hb, f32x4 acc0, int lane) {
  const TileOpsBf t = tile_ops_bf(dzb, hb, lane);
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
  tile_kstep<0>(t, acc0, acc1);
  tile_kstep<1>(t, acc0, acc1);
  return acc0 + acc1;
}

// the staging / tile-operand flavour of a stage type: f32 (16 K-steps) or bf16 (2)
template <class S>
struct TileKind {
  using Ops = std::conditional_t<S::BF, TileOpsBf, TileOps>;
  static constexpr int NK = S::BF ? 2 : 16;
  template <int N>
  static DTP_DEV void cols(float* buf, int lane, int c0, const float (&v)[16]) {
    if constexpr (S::BF) stage_cols_bf<N>(buf, lane, c0, v);
    else stage_cols<N>(buf, lane, c0, v);
  }
  static DTP_DEV void one(float* buf, int lane, int col, float v) {
    if constexpr (S::BF) stage_one_bf(buf, lane, col, v);
    else stage_one(buf, lane, col, v);
  }
  static DTP_DEV Ops ops(const float* dzb, const float* hb, int lane) {
    if constexpr (S::BF) return tile_ops_bf(dzb, hb, lane);
    else return tile_ops(dzb, hb, lane);
  }
  static DTP_DEV f32x4 outer(const float* dzb, const float* hb, f32x4 acc, int lane) {
    if constexpr (S::BF) return wave_outer_acc_bf(dzb, hb, acc, lane);
    else return wave_outer_acc(dzb, hb, acc, lane);
  }
};

}  // namespace dtp
