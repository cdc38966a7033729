// Software-pipelined forward + backward of the fused train step (v6).
//
// Why: in the v5 step (mlp_scalar.h lds_forward / lds_backward_dx) every layer
// reads its LDS weight block right before the FMAs that consume it.  The
// compiler keeps those reads just ahead of their uses, so a wave -- alone on its
// SIMD, nothing to switch to -- sits on ~90 `s_waitcnt lgkmcnt` per step, each
// exposing most of an LDS round trip (rocprofv3 + ISA listing, docs/perf_notes.md).
//
// Here a layer's block is already in registers when the layer starts: the
// NEXT block's rows are read in small chunks between the current layer's rows
// (one `sched_barrier` region per row), so at most a handful of LDS reads are in
// flight at any wait and every wait finds its data landed.  The forward's last
// layer prefetches the first two backward blocks; each backward layer prefetches
// the block of the layer below.  The MFMA K-steps of a layer's dW tile start a
// few rows into its input-gradient chain, once the tile operands read right
// after the staging writes have landed (LDS executes a wave's ops in order).
//
// Same arithmetic, same order of every floating-point operation as v5: the
// results are bitwise those of mlp_scalar.h's path.
#pragma once
#include <type_traits>

#include "mlp_scalar.h"

#ifndef DTP_PIPE_J0
#define DTP_PIPE_J0 4  // first input-gradient row that carries MFMA K-steps
#endif

namespace dtp {

// forward block of layer l in registers: row 0 = bias, rows 1..I = W^T rows
template <class S, int l>
struct FBlk {
  static constexpr int I = S::din(l), O = S::dout(l), OP = Scal<S>::pad4(O), NQ = OP / 4, NR = I + 1;
  float4 w[NR][NQ];
  template <int R0, int R1>
  DTP_DEV void load(const float* __restrict__ wl) {
    static_for<R0, (R1 < NR ? R1 : NR)>([&](auto RC) {
      constexpr int r = decltype(RC)::value;
      constexpr int off = r == 0 ? Scal<S>::lfb(l) : Scal<S>::lfo(l) + (r - 1) * OP;
      static_for<0, NQ>([&](auto QC) { w[r][decltype(QC)::value] = row_quad<O, decltype(QC)::value>(wl + off); });
    });
  }
};

// backward block of layer l >= 1 in registers: W_l rows (output-major)
template <class S, int l>
struct BBlk {
  static constexpr int I = S::din(l), O = S::dout(l), IP = Scal<S>::pad4(I), NQ = IP / 4, NR = O;
  float4 w[NR][NQ];
  template <int R0, int R1>
  DTP_DEV void load(const float* __restrict__ wl) {
    static_for<R0, (R1 < NR ? R1 : NR)>([&](auto RC) {
      constexpr int r = decltype(RC)::value;
      static_for<0, NQ>([&](auto QC) {
        w[r][decltype(QC)::value] = row_quad<I, decltype(QC)::value>(wl + Scal<S>::lbo(l) + r * IP);
      });
    });
  }
};

struct NoBlk {
  static constexpr int NR = 0;
  template <int, int>
  DTP_DEV void load(const float*) {}
};

// rows [A, B) of the concatenation P1 ++ P2
template <int A, int B, class P1, class P2>
DTP_DEV void load_rows(const float* __restrict__ wl, P1& p1, P2& p2) {
  constexpr int N1 = P1::NR;
  p1.template load<A, (B < N1 ? B : N1)>(wl);
  p2.template load<(A > N1 ? A - N1 : 0), (B > N1 ? B - N1 : 0)>(wl);
}

// the prefetch chunk that rides with compute row j of NJ: the rows of P1 ++ P2 are
// spread over the first NJ - 2 rows (the last two rows give the tail reads time)
template <int j, int NJ, class P1, class P2>
DTP_DEV void prefetch_chunk(const float* __restrict__ wl, P1& p1, P2& p2) {
  constexpr int T = P1::NR + P2::NR;
  constexpr int NP = NJ > 2 ? NJ - 2 : 1;
  if constexpr (j < NP && T > 0) load_rows<j * T / NP, (j + 1) * T / NP>(wl, p1, p2);
}

// the top two backward blocks, prefetched by the forward's last layer
template <class S>
using TopB2 = std::conditional_t<(S::NL >= 3), BBlk<S, (S::NL >= 3 ? S::NL - 2 : 1)>, NoBlk>;

// one forward layer from the register block B, prefetching P1 ++ P2 row by row.
// LM: LeakyReLU as max(z, slope * z), exact (NaN and signed zeros included) for
// 0 <= slope <= 1 and one VALU op shorter than the compare-and-select form
template <class S, int l, bool LM, class P1, class P2>
DTP_DEV void pipe_fwd_layer(const float* __restrict__ wl, const FBlk<S, l>& B, float (&h)[S::NL + 1][16],
                            float slope, P1& p1, P2& p2) {
  constexpr int I = S::din(l), O = S::dout(l), NQ = FBlk<S, l>::NQ;
  f32x2 z[2 * NQ];
  static_for<0, NQ>([&](auto QC) {
    constexpr int q = decltype(QC)::value;
    z[2 * q] = f32x2{B.w[0][q].x, B.w[0][q].y};
    z[2 * q + 1] = f32x2{B.w[0][q].z, B.w[0][q].w};
  });
  static_for<0, I>([&](auto IC) {
    constexpr int i = decltype(IC)::value;
    const f32x2 hi = f32x2{h[l][i], h[l][i]};
    static_for<0, NQ>([&](auto QC) {
      constexpr int q = decltype(QC)::value;
      if constexpr (4 * q < O) z[2 * q] = __builtin_elementwise_fma(f32x2{B.w[i + 1][q].x, B.w[i + 1][q].y}, hi, z[2 * q]);
      if constexpr (4 * q + 2 < O)
        z[2 * q + 1] = __builtin_elementwise_fma(f32x2{B.w[i + 1][q].z, B.w[i + 1][q].w}, hi, z[2 * q + 1]);
    });
    // this row's FMAs need the current block only: issue them before the next
    // block's reads, so their waits never count the fresh reads
    __builtin_amdgcn_sched_barrier(0);
    prefetch_chunk<i, I>(wl, p1, p2);
    __builtin_amdgcn_sched_barrier(0);
  });
  static_for<0, O>([&](auto JC) {
    constexpr int j = decltype(JC)::value;
    const float v = S::rnd((j & 1) ? z[j / 2].y : z[j / 2].x);  // bf16: the Linear output, then the activation
    h[l + 1][j] = S::rnd(S::act(l) ? (LM ? fmaxf(v, v * slope) : leaky(v, slope)) : v);
  });
}

// forward of layers [l, NL) with layer l's block in B; the last layer prefetches
// the backward blocks of layers NL-1 and NL-2 into bt, bt2
template <class S, int l, bool LM = false>
DTP_DEV void pipe_forward(const float* __restrict__ wl, const FBlk<S, l>& B, float (&h)[S::NL + 1][16], float slope,
                          BBlk<S, S::NL - 1>& bt, TopB2<S>& bt2) {
  if constexpr (l + 1 < S::NL) {
    FBlk<S, l + 1> nb;
    NoBlk none;
    pipe_fwd_layer<S, l, LM>(wl, B, h, slope, nb, none);
    pipe_forward<S, l + 1, LM>(wl, nb, h, slope, bt, bt2);
  } else {
    pipe_fwd_layer<S, l, LM>(wl, B, h, slope, bt, bt2);
  }
}

// Backward state shared by the layers of one step.
template <class S>
struct PipeBwdCtx {
  const float* wl;
  float* stg_pack;
  float* stg_hid;
  int lane;
  float slope;
  float lpart;
};

// stage (dz_l, [h_l, 1]) of layer l into its staging area; returns that area
template <class S, int l>
DTP_DEV float* pipe_stage(const PipeBwdCtx<S>& c, const float (&h)[S::NL + 1][16], const float (&dz)[16]) {
  using SC = Scal<S>;
  constexpr int I = S::din(l), O = S::dout(l);
  constexpr bool packed = SC::PACK && (l == 0 || l == S::NL - 1);
  float* stg = packed ? c.stg_pack : c.stg_hid;
  using TK = TileKind<S>;
  TK::template cols<O>(stg, c.lane, SC::rowoff(l), dz);
  // the batch loss rides in a free row of the output tile (f32 only: a bf16 operand
  // would round it; the bf16 instance sums the loss with a wave reduction instead)
  if constexpr (l == S::NL - 1 && !S::BF) stage_one(stg, c.lane, SC::lossrow(), c.lpart);
  TK::template cols<I>(stg + kStgArr, c.lane, SC::coloff(l), h[l]);
  TK::one(stg + kStgArr, c.lane, SC::coloff(l) + I, 1.f);
  return stg;
}

// backward layer l >= 1: stage, read the tile operands (unpacked tiles), then the
// input-gradient chain from the register block B with the tile's 16 MFMA K-steps
// on rows [J0, O) and the prefetch of P (the block of layer l-1) on the first rows
template <class S, int l, class P>
DTP_DEV void pipe_bwd_layer(const PipeBwdCtx<S>& c, const BBlk<S, l>& B, const float (&h)[S::NL + 1][16],
                            float (&dz)[16], f32x4 (&acc)[Scal<S>::NT], P& p) {
  using SC = Scal<S>;
  constexpr int I = S::din(l), O = S::dout(l), NQ = BBlk<S, l>::NQ;
  constexpr bool packed = SC::PACK && (l == 0 || l == S::NL - 1);
  using TK = TileKind<S>;
  constexpr int NK = TK::NK;
  float* stg = pipe_stage<S, l>(c, h, dz);
  typename TK::Ops to;
  if constexpr (!packed) {
    __builtin_amdgcn_wave_barrier();
    to = TK::ops(stg, stg + kStgArr, c.lane);
  }
  f32x4 a1 = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 a0 = acc[SC::tile(l)];
  NoBlk none;
  f32x2 g[2 * NQ];
  static_for<0, 2 * NQ>([&](auto QC) { g[decltype(QC)::value] = f32x2{0.f, 0.f}; });
  constexpr int J0 = O > DTP_PIPE_J0 ? DTP_PIPE_J0 : 0;
  static_for<0, O>([&](auto JC) {
    constexpr int j = decltype(JC)::value;
    if constexpr (!packed && j >= J0) {
      constexpr int k0 = NK * (j - J0) / (O - J0), k1 = NK * (j - J0 + 1) / (O - J0);
      static_for<k0, k1>([&](auto KC) { tile_kstep<decltype(KC)::value>(to, a0, a1); });
    }
    const f32x2 d = f32x2{dz[j], dz[j]};
    static_for<0, NQ>([&](auto QC) {
      constexpr int q = decltype(QC)::value;
      if constexpr (4 * q < I) g[2 * q] = __builtin_elementwise_fma(f32x2{B.w[j][q].x, B.w[j][q].y}, d, g[2 * q]);
      if constexpr (4 * q + 2 < I)
        g[2 * q + 1] = __builtin_elementwise_fma(f32x2{B.w[j][q].z, B.w[j][q].w}, d, g[2 * q + 1]);
    });
    __builtin_amdgcn_sched_barrier(0);
    prefetch_chunk<j, O>(c.wl, p, none);
    __builtin_amdgcn_sched_barrier(0);
  });
  if constexpr (!packed) acc[SC::tile(l)] = a0 + a1;
  static_for<0, I>([&](auto IC) {
    constexpr int i = decltype(IC)::value;
    const float v = (i & 1) ? g[i / 2].y : g[i / 2].x;
    dz[i] = S::rnd(S::rnd(v) * (S::act(l - 1) ? leaky_grad_from_out(h[l][i], c.slope) : 1.f));
  });
}

// backward of layers [1, l] with layer l's block in B (the block of layer l-1
// is prefetched during layer l), then layer 0 (no input gradient)
template <class S, int l>
DTP_DEV void pipe_bwd_rest(const PipeBwdCtx<S>& c, const BBlk<S, l>& B, const float (&h)[S::NL + 1][16],
                           float (&dz)[16], f32x4 (&acc)[Scal<S>::NT]) {
  if constexpr (l > 1) {
    BBlk<S, l - 1> nb;
    pipe_bwd_layer<S, l>(c, B, h, dz, acc, nb);
    pipe_bwd_rest<S, l - 1>(c, nb, h, dz, acc);
  } else {
    NoBlk none;
    pipe_bwd_layer<S, l>(c, B, h, dz, acc, none);
    // layer 0: its dW tile only
    using SC = Scal<S>;
    float* stg = pipe_stage<S, 0>(c, h, dz);
    if constexpr (!SC::PACK) {
      __builtin_amdgcn_wave_barrier();
      acc[SC::tile(0)] = TileKind<S>::outer(stg, stg + kStgArr, acc[SC::tile(0)], c.lane);
    }
  }
}

// whole backward: top layer (block bt, the next block bt2 already prefetched by
// the forward), the hidden layers, layer 0, then the packed first/last tile
template <class S>
DTP_DEV void pipe_backward(const PipeBwdCtx<S>& c, const BBlk<S, S::NL - 1>& bt, const TopB2<S>& bt2,
                           const float (&h)[S::NL + 1][16], float (&dz)[16], f32x4 (&acc)[Scal<S>::NT]) {
  static_assert(S::NL >= 3, "the pipelined step serves networks of >= 3 layers");
  using SC = Scal<S>;
  NoBlk none;
  pipe_bwd_layer<S, S::NL - 1>(c, bt, h, dz, acc, none);
  pipe_bwd_rest<S, S::NL - 2>(c, bt2, h, dz, acc);
  if constexpr (SC::PACK) {
    __builtin_amdgcn_wave_barrier();
    acc[0] = TileKind<S>::outer(c.stg_pack, c.stg_pack + kStgArr, acc[0], c.lane);
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace dtp
