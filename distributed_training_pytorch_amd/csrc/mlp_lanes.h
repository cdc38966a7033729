// Fused train step with SEVERAL LANES PER SAMPLE (mlp_train.hip includes this).
//
// Why: the one-lane-per-sample step (mlp_train_kernel) is latency-bound, so its time
// does not depend on the batch: 4.26 / 4.30 / 4.27 us at B = 64 / 128 / 256
// (docs/perf_notes.md).  The reference's headline workload is strong scaling -- ONE
// 512-sample set split by DistributedSampler, per-rank batch 256 / 256 / 128 / 64 at
// W = 1 / 2 / 4 / 8 (/root/reference/demo.py:141-148) -- so a step that does not get
// shorter with the batch caps the whole node at 512 / (4.3 us + exchange).
//
// Decomposition (L = 2 or 4 lanes per sample, always 256 lanes = one wave per SIMD):
//   * the L lanes of a sample are adjacent inside a DPP quad; lane part p owns outputs
//     [p*NO, p*NO + NO) of every hidden layer (NO = ceil(H / L));
//   * forward of a hidden layer: each lane runs NO output chains over the full input
//     vector (its own slice of W^T read from LDS: L distinct 16-byte chunks per quad,
//     2-3x fewer LDS bytes than the broadcast of the whole block), the activation on its
//     slice, then the slice is broadcast to the sample's other lanes with DPP quad_perm
//     moves (NO * L v_mov_dpp);
//   * the last layer (OUT outputs) is computed whole by every lane of the sample;
//   * input-gradient chain: the output gradient slice is gathered by DPP the same way,
//     each lane forms its own slice of W^T dz (the next-lower layer's slice);
//   * weight gradient: each lane stages its own slices of (dz, h) into the wave's
//     per-tile LDS area; the MFMA K dimension runs over the wave's G = 64 / L samples
//     (G / 4 K-steps of v_mfma_f32_16x16x4_f32 per tile instead of 16); the constant-1
//     bias columns are written once per launch;
//   * cross-wave reduction, Adam, the xGMI exchange and the sampler are those of the
//     one-lane kernel (same per-thread parameter ownership, same granule format).
// Numerics: forward and input-gradient chains run the same fmaf sequence as the
// one-lane kernel (bias first, inputs ascending; outputs ascending from 0), so those
// values are bitwise the same; the dW and loss sums group the batch differently
// (16 or 32 samples per wave), i.e. differ by float reassociation only.
//
// Serves the FAST configuration only (MSE, Adam, SAMPLER_TABLE ring, dataset cached in
// LDS, 0 <= slope <= 1, fp32); the host picks it in resolve_train() when the per-rank
// batch is <= 256 / L.
#pragma once
#include "mlp_scalar.h"

namespace dtp {

// value v of the lane holding part P of this lane's sample (DPP quad_perm broadcast)
template <int L, int P>
DTP_DEV float part_bcast(float v) {
  static_assert(L == 2 || L == 4, "2 or 4 lanes per sample");
  constexpr int ctrl = L == 4 ? P * 0x55 : (P | (P << 2) | ((2 + P) << 4) | ((2 + P) << 6));
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xF, 0xF, false));
}

template <class S, int L_>
struct LaneCfg {
  static constexpr int L = L_, NL = S::NL, H = S::H, IN = S::IN, OUT = S::OUT;
  static_assert(L == 2 || L == 4, "2 or 4 lanes per sample");
  static_assert(NL >= 3, "hidden layers partitioned, last layer whole: NL >= 3");
  static constexpr int G = kWave / L;         // samples per wave
  static constexpr int BMAX = kBlock / L;     // samples per step
  static constexpr int TS = G / 4;            // MFMA K-steps per tile (4 samples each)
  static constexpr int NO = (H + L - 1) / L;  // hidden outputs (and inputs) per part
  static constexpr int NOP = (NO + 3) & ~3;   // a part's slice padded to float4
  static constexpr int NPR = (NO + 1) / 2;    // v_pk_fma pairs per slice
  static constexpr bool EXACT = NO * L == H;  // every slot of every part is a real unit
  static constexpr int pad4(int x) { return (x + 3) & ~3; }
  // bf16 compute (Stage BF): matmul operands and outputs rounded to bf16 (mlp_core.h); the
  // dW tiles stay on the exact fp32 MFMA, whose products of bf16 values are exact
  static DTP_DEV float rnd(float v) { return S::rnd(v); }
  static constexpr int RW = pad4(H + 1);      // last layer's whole block: row o = W[o][0..H-1], b[o]
  // forward block of partitioned layer l (< NL-1): rows r < din(l) = inputs, row din(l) = bias;
  // a row = [part][NOP] (W[p*NO + k][r] at (r*L + p)*NOP + k)
  static constexpr int FR(int l) { return (S::din(l) + 1) * L * NOP; }
  static constexpr int f_off(int l) {
    int o = 0;
    for (int k = 0; k < l && k < NL - 1; ++k) o += FR(k);
    return o;
  }
  static constexpr int f_last() { return f_off(NL - 1); }
  // backward block of layer l >= 1: rows o < dout(l); a row = [part][NOP] (W_l[o][p*NO + k])
  static constexpr int BR(int l) { return S::dout(l) * L * NOP; }
  static constexpr int b_off(int l) {
    int o = f_last() + OUT * RW;
    for (int k = 1; k < l; ++k) o += BR(k);
    return o;
  }
  static constexpr int LW = b_off(NL);
  // per-tile staging of one wave: sample s at [s & 3][col][s >> 2]; reader lane (q, c) finds
  // its TS K-step operands contiguous (TS floats)
  static constexpr int QS = 16 * TS + 4;
  static constexpr int AREA = 4 * QS;  // floats per staged operand (dz or h) of one tile
};

// positions of torch-order parameter p: forward block, backward block (-1: none), dW tile
template <class C, class S>
DTP_DEV void lane_pos(int p, int& pf, int& pb, int& tp) {
  using SC = Scal<S>;
  constexpr int NL = S::NL, L = C::L, NO = C::NO, NOP = C::NOP;
  pf = 0;
  pb = -1;
  tp = 0;
  static_for<0, NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l);
    constexpr int base = SC::tile(l) * SC::TSZ, ro = SC::rowoff(l), co = SC::coloff(l);
    if (p >= S::gw(l) && p < S::gb(l)) {
      const int q = p - S::gw(l), j = q / I, i = q - j * I;
      if constexpr (l < NL - 1) pf = C::f_off(l) + (i * L + j / NO) * NOP + j % NO;
      else pf = C::f_last() + j * C::RW + i;
      if constexpr (l >= 1) pb = C::b_off(l) + (j * L + i / NO) * NOP + i % NO;
      tp = base + SC::tslot(ro + j, co + i);
    } else if (p >= S::gb(l) && p < S::gb(l) + O) {
      const int j = p - S::gb(l);
      if constexpr (l < NL - 1) pf = C::f_off(l) + (I * L + j / NO) * NOP + j % NO;
      else pf = C::f_last() + j * C::RW + I;
      tp = base + SC::tslot(ro + j, co + I);  // bias column = constant-1 input
    }
  });
}

// ---- register blocks (row-chunked loads, so a layer can prefetch the next one) ----
template <class C, int l>
struct LFBlk {  // this lane's slice of partitioned forward layer l: din(l) input rows + bias
  static constexpr int NR = (l == 0 ? C::IN : C::H) + 1, NQ = C::NOP / 4;
  float4 w[NR][NQ];
  template <int R0, int R1>
  DTP_DEV void load(const float* __restrict__ wl, const float* __restrict__ wlp) {
    static_for<R0, (R1 < NR ? R1 : NR)>([&](auto RC) {
      constexpr int r = decltype(RC)::value;
      static_for<0, NQ>([&](auto QC) {
        constexpr int q = decltype(QC)::value;
        w[r][q] = row_quad<C::NO, q>(wlp + C::f_off(l) + r * C::L * C::NOP);
      });
    });
  }
};

template <class C>
struct LLast {  // the last layer whole: OUT rows of [W[o][0..H-1], b[o]]
  static constexpr int NR = C::OUT, NQ = C::RW / 4;
  float4 w[NR][NQ];
  template <int R0, int R1>
  DTP_DEV void load(const float* __restrict__ wl, const float* __restrict__ wlp) {
    static_for<R0, (R1 < NR ? R1 : NR)>([&](auto RC) {
      constexpr int r = decltype(RC)::value;
      static_for<0, NQ>([&](auto QC) {
        constexpr int q = decltype(QC)::value;
        w[r][q] = row_quad<C::H + 1, q>(wl + C::f_last() + r * C::RW);
      });
    });
  }
};

template <class C, int l>
struct LBBlk {  // this lane's slice of backward layer l >= 1: dout(l) rows of W_l[o][p*NO + k]
  static constexpr int NR = (l == C::NL - 1 ? C::OUT : C::H), NQ = C::NOP / 4;
  float4 w[NR][NQ];
  template <int R0, int R1>
  DTP_DEV void load(const float* __restrict__ wl, const float* __restrict__ wlp) {
    static_for<R0, (R1 < NR ? R1 : NR)>([&](auto RC) {
      constexpr int r = decltype(RC)::value;
      static_for<0, NQ>([&](auto QC) {
        constexpr int q = decltype(QC)::value;
        w[r][q] = row_quad<C::NO, q>(wlp + C::b_off(l) + r * C::L * C::NOP);
      });
    });
  }
};

struct LNone {
  static constexpr int NR = 0;
  template <int, int>
  DTP_DEV void load(const float*, const float*) {}
};

// rows [A, B) of the concatenation P1 ++ P2
template <int A, int B, class P1, class P2>
DTP_DEV void lrows(const float* wl, const float* wlp, P1& p1, P2& p2) {
  constexpr int N1 = P1::NR;
  p1.template load<A, (B < N1 ? B : N1)>(wl, wlp);
  p2.template load<(A > N1 ? A - N1 : 0), (B > N1 ? B - N1 : 0)>(wl, wlp);
}

// the prefetch chunk riding with compute row j of NJ (spread over the first NJ - 1 rows)
template <int j, int NJ, class P1, class P2>
DTP_DEV void lchunk(const float* wl, const float* wlp, P1& p1, P2& p2) {
  constexpr int T = P1::NR + P2::NR;
  constexpr int NP = NJ > 1 ? NJ - 1 : 1;
  if constexpr (j < NP && T > 0) lrows<j * T / NP, (j + 1) * T / NP>(wl, wlp, p1, p2);
}

template <int Q>
DTP_DEV f32x2 quad_pair(const float4& v) {
  if constexpr (Q == 0) return f32x2{v.x, v.y};
  else return f32x2{v.z, v.w};
}

// Per-step state of one lane.
template <class C>
struct LaneAct {
  float hin[16];               // full input vector of the layer being computed
  float own[C::NL][C::NOP];    // own slice of every partitioned layer's output (index l + 1 - 1 = l)
};

// forward of partitioned layer l from block B (full input hin -> own slice, full output
// into hin), prefetching P1 ++ P2 row by row
template <class C, int l, class P1, class P2>
DTP_DEV void lane_fwd_layer(const float* wl, const float* wlp, const LFBlk<C, l>& B, LaneAct<C>& st, float slope,
                            P1& p1, P2& p2) {
  constexpr int I = LFBlk<C, l>::NR - 1, NO = C::NO, NPR = C::NPR;
  f32x2 z[NPR];
  static_for<0, NPR>([&](auto RC) {
    constexpr int r = decltype(RC)::value;
    z[r] = quad_pair<r % 2>(B.w[I][r / 2]);
  });
  static_for<0, I>([&](auto IC) {
    constexpr int i = decltype(IC)::value;
    const f32x2 hi = f32x2{st.hin[i], st.hin[i]};
    static_for<0, NPR>([&](auto RC) {
      constexpr int r = decltype(RC)::value;
      z[r] = __builtin_elementwise_fma(quad_pair<r % 2>(B.w[i][r / 2]), hi, z[r]);
    });
    __builtin_amdgcn_sched_barrier(0);
    lchunk<i, I>(wl, wlp, p1, p2);
    __builtin_amdgcn_sched_barrier(0);
  });
  static_for<0, NO>([&](auto KC) {
    constexpr int k = decltype(KC)::value;
    const float v = C::rnd((k & 1) ? z[k / 2].y : z[k / 2].x);  // bf16: the Linear output, then the activation
    st.own[l][k] = C::rnd(fmaxf(v, v * slope));  // LeakyReLU, exact for 0 <= slope <= 1
  });
  // the whole output vector in every lane of the sample
  static_for<0, C::L>([&](auto PC) {
    constexpr int pp = decltype(PC)::value;
    static_for<0, NO>([&](auto KC) {
      constexpr int k = decltype(KC)::value;
      if constexpr (pp * NO + k < C::H) st.hin[pp * NO + k] = part_bcast<C::L, pp>(st.own[l][k]);
    });
  });
}

// forward of layers [l, NL-1) (partitioned) then the whole last layer; the last hidden
// layer prefetches the last layer's block and its backward block, the last layer the
// backward block of layer NL-2
template <class C, int l>
DTP_DEV void lane_forward(const float* wl, const float* wlp, const LFBlk<C, l>& B, LaneAct<C>& st, float slope,
                          LLast<C>& last, LBBlk<C, C::NL - 1>& bt, LBBlk<C, C::NL - 2>& bt2, float (&out)[16]) {
  constexpr int NL = C::NL;
  if constexpr (l + 1 < NL - 1) {
    LFBlk<C, l + 1> nb;
    LNone none;
    lane_fwd_layer<C, l>(wl, wlp, B, st, slope, nb, none);
    lane_forward<C, l + 1>(wl, wlp, nb, st, slope, last, bt, bt2, out);
  } else {
    lane_fwd_layer<C, l>(wl, wlp, B, st, slope, last, bt);
    // last layer, whole, every lane: z_o = b_o + sum_i W[o][i] h_i (inputs ascending)
    constexpr int H = C::H;
    float z[C::OUT];
    static_for<0, C::OUT>([&](auto OC) {
      constexpr int o = decltype(OC)::value;
      const float4& bq = last.w[o][H / 4];
      z[o] = (H % 4 == 0) ? bq.x : (H % 4 == 1) ? bq.y : (H % 4 == 2) ? bq.z : bq.w;
    });
    LNone none;
    static_for<0, H>([&](auto IC) {
      constexpr int i = decltype(IC)::value;
      static_for<0, C::OUT>([&](auto OC) {
        constexpr int o = decltype(OC)::value;
        const float4& wq = last.w[o][i / 4];
        const float w = (i % 4 == 0) ? wq.x : (i % 4 == 1) ? wq.y : (i % 4 == 2) ? wq.z : wq.w;
        z[o] = fmaf(w, st.hin[i], z[o]);
      });
      __builtin_amdgcn_sched_barrier(0);
      lchunk<i, H>(wl, wlp, bt2, none);
      __builtin_amdgcn_sched_barrier(0);
    });
    static_for<0, C::OUT>([&](auto OC) { out[decltype(OC)::value] = C::rnd(z[decltype(OC)::value]); });
  }
}

// Staging pointers of one lane for one tile: writer base (sample slot) and reader base.
struct LaneStg {
  float* wr;        // + col * TS: this lane's sample slot in a staged operand
  const float* rd;  // reader: lane (q, c) -> its TS contiguous K-step operands
};

template <class C, int TSZ>
struct LaneTileOps {
  float4 a[TSZ / 4], b[TSZ / 4];
};

template <class C>
DTP_DEV LaneTileOps<C, C::TS> lane_tile_ops(const float* tile, int rdoff) {
  LaneTileOps<C, C::TS> t;
  static_for<0, C::TS / 4>([&](auto MC) {
    constexpr int m = decltype(MC)::value;
    t.a[m] = *reinterpret_cast<const float4*>(tile + rdoff + 4 * m);
    t.b[m] = *reinterpret_cast<const float4*>(tile + C::AREA + rdoff + 4 * m);
  });
  return t;
}

template <int K, class T>
DTP_DEV void lane_kstep(const T& t, f32x4& acc0, f32x4& acc1) {
  const float4& a = t.a[K / 4];
  const float4& b = t.b[K / 4];
  const float av = (K % 4 == 0) ? a.x : (K % 4 == 1) ? a.y : (K % 4 == 2) ? a.z : a.w;
  const float bv = (K % 4 == 0) ? b.x : (K % 4 == 1) ? b.y : (K % 4 == 2) ? b.z : b.w;
  if constexpr (K & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc1, 0, 0, 0);
  else acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc0, 0, 0, 0);
}

#ifndef DTP_LANES_BFMMA
// 1: bf16 instances run each dW tile as ONE bf16 MFMA over the wave's samples (16x16x16 at
// 4 lanes per sample: 16 samples; 16x16x32 at 2: 32) instead of TS f32 K = 4 steps
#define DTP_LANES_BFMMA 1
#endif

// top halves of two bf16-valued floats as one packed bf16 pair (lo in bits 0..15)
DTP_DEV unsigned bf_pair(float lo, float hi) {
  return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);
}

// bf16 compute: a whole dW tile of the wave on one bf16 MFMA.  The staged operands hold
// bf16-rounded floats (Stage::rnd), so packing their top halves is exact.  Reader lane
// (q, c) holds the K-step operands of samples q, 4 + q, 8 + q, ... (one per f32 K-step);
// they become its 4 (or 8) K values of the bf16 instruction -- the same sample at the same
// position for both operands, so the tile sums the same products.
template <class C, class T>
DTP_DEV f32x4 lane_tile_bf(const T& t, f32x4 acc) {
  static_assert(C::TS == 4 || C::TS == 8, "16 or 32 samples per wave");
  if constexpr (C::TS == 4) {
    typedef short s4 __attribute__((ext_vector_type(4)));
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    const u2 a = {bf_pair(t.a[0].x, t.a[0].y), bf_pair(t.a[0].z, t.a[0].w)};
    const u2 b = {bf_pair(t.b[0].x, t.b[0].y), bf_pair(t.b[0].z, t.b[0].w)};
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s4, a), __builtin_bit_cast(s4, b), acc, 0, 0, 0);
  } else {
    typedef __bf16 b8 __attribute__((ext_vector_type(8)));
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4 a = {bf_pair(t.a[0].x, t.a[0].y), bf_pair(t.a[0].z, t.a[0].w), bf_pair(t.a[1].x, t.a[1].y),
                  bf_pair(t.a[1].z, t.a[1].w)};
    const u4 b = {bf_pair(t.b[0].x, t.b[0].y), bf_pair(t.b[0].z, t.b[0].w), bf_pair(t.b[1].x, t.b[1].y),
                  bf_pair(t.b[1].z, t.b[1].w)};
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), acc, 0, 0, 0);
  }
}

// a whole tile: TS f32 K-steps, or the bf16 instruction (bf16 instances)
template <class C, class S, class T>
DTP_DEV f32x4 lane_tile(const T& t, f32x4 acc) {
  if constexpr (S::BF && DTP_LANES_BFMMA) {
    return lane_tile_bf<C>(t, acc);
  } else {
    f32x4 a1 = f32x4{0.f, 0.f, 0.f, 0.f};
    static_for<0, C::TS>([&](auto KC) { lane_kstep<decltype(KC)::value>(t, acc, a1); });
    return acc + a1;
  }
}

}  // namespace dtp
