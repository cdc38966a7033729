// "Pair" decomposition of the fused train step (v2): TWO lanes per sample.
//
// Why: with one lane per sample a 256-sample batch is 4 waves = one wave per
// SIMD, and a lone wave issues VALU at half the SIMD rate (MI355X_MICROARCH.md,
// v_fma_f32 "one wave alone: 4" cycles).  Splitting every layer's outputs
// between two lanes of the same wave gives 8 waves (two per SIMD) with
// half the FMAs each.  The two lanes of a sample are ADJACENT (2s, 2s+1), so a
// partner's value is one DPP quad_perm[1,0,3,2] move (no LDS, no barrier, no
// select) before the next layer.
//
// Per layer l and half h = lane & 1:
//   * the lane computes outputs [obeg(l,h), obeg(l,h) + ocnt(l,h)) (OH(l) slots,
//     the unused slot of an odd width is a zero row);
//   * its inputs arrive as (own half, partner half) -- the forward weight block
//     FW(l,h) is stored with its columns in exactly that order, the backward block
//     BW(l,h) (input-gradient rows of the lane's half) likewise for dz, so the
//     code is identical for both halves and only the LDS base differs (two
//     broadcast addresses per wave).  Both blocks are stored input-major
//     ([input][output]) so one ds_read_b128 yields four consecutive outputs of
//     one input: two v_pk_fma_f32 with the input broadcast, no register shuffles;
//   * the dW MFMA staging row of a sample is written half by each lane.
// The first and the last layer share one 16x16 MFMA tile when they fit (toy:
// 10x3 and 1x11 blocks + two loss rows), so the toy needs 4 tiles, not 5.
#pragma once
#include "mlp_core.h"

namespace dtp {

template <class S>
struct Pair {
  static constexpr int NL = S::NL;
  static constexpr int IN = S::IN, OUT = S::OUT;
  static constexpr int OH(int l) { return (S::dout(l) + 1) / 2; }
  static constexpr int obeg(int l, int h) { return h == 0 ? 0 : OH(l); }
  static constexpr int ocnt(int l, int h) { return h == 0 ? OH(l) : S::dout(l) - OH(l); }
  // inputs of layer l >= 1 are the outputs of layer l-1, split the same way
  static constexpr int IHM(int l) { return l == 0 ? IN : OH(l - 1); }
  static constexpr int ibeg(int l, int h) { return l == 0 ? 0 : obeg(l - 1, h); }
  static constexpr int icnt(int l, int h) { return l == 0 ? IN : ocnt(l - 1, h); }
  static constexpr int pad4(int x) { return (x + 3) & ~3; }
  // forward block FW(l,h), input-major: NIN rows (inputs: x, or [own half | partner half])
  // x OHP cols (the lane's outputs, padded to 4), then OHP biases
  static constexpr int NIN(int l) { return l == 0 ? IN : 2 * IHM(l); }
  static constexpr int OHP(int l) { return pad4(OH(l)); }
  static constexpr int FB(int l) { return NIN(l) * OHP(l); }  // bias offset inside a half block
  static constexpr int FH(int l) { return FB(l) + OHP(l); }
  static constexpr int fwo(int l) {
    int o = 0;
    for (int k = 0; k < l; ++k) o += 2 * FH(k);
    return o;
  }
  // backward block BW(l,h), l >= 1, dz-major: 2*OH rows ([own dz half | partner dz half])
  // x IHP cols (the lane's input gradients, padded to 4)
  static constexpr int IHP(int l) { return pad4(IHM(l)); }
  static constexpr int BH(int l) { return 2 * OH(l) * IHP(l); }
  static constexpr int bwo(int l) {
    int o = fwo(NL);
    for (int k = 1; k < l; ++k) o += 2 * BH(k);
    return o;
  }
  static constexpr int LW = bwo(NL);
  static constexpr int OHMAX() {
    int m = 1;
    for (int l = 0; l < NL; ++l) m = OH(l) > m ? OH(l) : m;
    return m;
  }
  // ---- MFMA tiles ----
  static constexpr int O0 = S::dout(0);
  static constexpr int IL = S::din(NL - 1);
  // first + last layer (and the two loss rows) packed into one tile when they fit
  static constexpr bool PACK = NL >= 2 && (O0 + OUT + 2 <= 16) && (IN + 1 + IL + 1 <= 16);
  static constexpr int NT = PACK ? NL - 1 : NL;
  static constexpr int tile(int l) { return PACK ? (l == NL - 1 ? 0 : l) : l; }
  static constexpr int rowoff(int l) { return (PACK && l == NL - 1) ? O0 : 0; }
  static constexpr int coloff(int l) { return (PACK && l == NL - 1) ? IN + 1 : 0; }
  static constexpr int lossrow() { return rowoff(NL - 1) + OUT; }          // rows lossrow, lossrow+1
  static constexpr int losscol() { return coloff(NL - 1) + S::din(NL - 1); }  // last layer's bias column
  static_assert(S::OUT + 2 <= 16, "two loss rows must fit under the output rows");
  static_assert(NL >= 2, "pair kernel expects at least two layers");
  static constexpr int NPT = (S::P + 511) / 512;  // params per thread with 512 threads
};

// staging for the wave's 32 samples s = 4t + q: [q][col][t], q stride 136 (= 8 mod 32:
// conflict-free column writes from the 32 lanes of a half; reads are 2 x b128)
constexpr int kQ2 = 136;
constexpr int kStg2 = 4 * kQ2;  // floats per staged operand array

DTP_DEV void stg2_write(float* __restrict__ buf, int sl, int col, float v) {
  buf[(sl & 3) * kQ2 + col * 8 + (sl >> 2)] = v;
}

DTP_DEV f32x4 wave_outer_acc32(const float* __restrict__ dzb, const float* __restrict__ hb, f32x4 acc0, int lane) {
  const int off = (lane >> 4) * kQ2 + (lane & 15) * 8;
  const float4 a0 = *reinterpret_cast<const float4*>(dzb + off);
  const float4 a1 = *reinterpret_cast<const float4*>(dzb + off + 4);
  const float4 b0 = *reinterpret_cast<const float4*>(hb + off);
  const float4 b1 = *reinterpret_cast<const float4*>(hb + off + 4);
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
  acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc0, 0, 0, 0);
  acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc1, 0, 0, 0);
  acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc0, 0, 0, 0);
  acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc1, 0, 0, 0);
  acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1.x, acc0, 0, 0, 0);
  acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1.y, acc1, 0, 0, 0);
  acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1.z, acc0, 0, 0, 0);
  acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1.w, acc1, 0, 0, 0);
  return acc0 + acc1;
}

// value held by the partner lane (lane ^ 1): DPP quad_perm [1,0,3,2]
DTP_DEV float partner(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}

// LDS positions of torch-order parameter p in the forward / backward blocks (-1: none)
template <class S>
DTP_DEV void pair_pos(int p, int& pf, int& pb) {
  using PR = Pair<S>;
  pf = -1;
  pb = -1;
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l);
    if (p >= S::gw(l) && p < S::gb(l)) {
      const int q = p - S::gw(l), j = q / I, i = q % I;
      const int h = j < PR::OH(l) ? 0 : 1;
      const int k = j - PR::obeg(l, h);
      int m;
      if constexpr (l == 0) {
        m = i;
      } else {
        const bool own = i >= PR::ibeg(l, h) && i < PR::ibeg(l, h) + PR::icnt(l, h);
        m = own ? i - PR::ibeg(l, h) : PR::IHM(l) + (i - PR::ibeg(l, 1 - h));
      }
      pf = PR::fwo(l) + h * PR::FH(l) + m * PR::OHP(l) + k;
      if constexpr (l >= 1) {
        const int hi = i < PR::OH(l - 1) ? 0 : 1;  // half owning input i
        const int ki = i - PR::ibeg(l, hi);
        const bool jown = j >= PR::obeg(l, hi) && j < PR::obeg(l, hi) + PR::ocnt(l, hi);
        const int mj = jown ? j - PR::obeg(l, hi) : PR::OH(l) + (j - PR::obeg(l, 1 - hi));
        pb = PR::bwo(l) + hi * PR::BH(l) + mj * PR::IHP(l) + ki;
      }
    } else if (p >= S::gb(l) && p < S::gb(l) + O) {
      const int j = p - S::gb(l);
      const int h = j < PR::OH(l) ? 0 : 1;
      pf = PR::fwo(l) + h * PR::FH(l) + PR::FB(l) + (j - PR::obeg(l, h));
    }
  });
}

// position of parameter p in the reduced tiles: tile*256 + row*16 + col
template <class S>
DTP_DEV int pair_tile_pos(int p) {
  using PR = Pair<S>;
  int r = 0;
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l);
    constexpr int base = PR::tile(l) * 256, ro = PR::rowoff(l), co = PR::coloff(l);
    if (p >= S::gw(l) && p < S::gb(l)) {
      const int q = p - S::gw(l);
      r = base + (ro + q / I) * 16 + co + q % I;
    } else if (p >= S::gb(l) && p < S::gb(l) + O) {
      r = base + (ro + p - S::gb(l)) * 16 + co + I;
    }
  });
  return r;
}

}  // namespace dtp
