// Per-sample MLP building blocks shared by the fused train-step kernel and the
// stage forward/backward kernels.
//
// Work decomposition (MI355X-first):
//   * one lane = one sample: forward and the input-gradient chain are VALU FMA
//     chains over LDS-broadcast weights (widths <= 15, so a 16x16 MFMA tile would
//     waste >60% of its lanes on padding there);
//   * the weight/bias gradient dW_l = sum_s dz_l[s] (x) [h_l[s], 1] is a K = batch
//     reduction, which is exactly what the MFMA K dimension does for free:
//     each wave stages its 64 samples' (dz, h) rows in LDS and runs 16
//     v_mfma_f32_16x16x4_f32 per layer (exact fp32, fmaf-chain numerics).  The
//     bias gradient rides in the same tile through a constant-1 input column.
//   * the four per-wave partial tiles are summed through LDS by the optimizer
//     phase, which owns one parameter per thread.
#pragma once
#include "dtp_common.h"

namespace dtp {

// A stage = NL Linear layers  IN -> H -> ... -> H -> OUT, LeakyReLU after every
// layer but the last (and after the last too when FINAL_ACT, which is how a
// layer-split stage that ends inside the network looks).
template <int IN_, int H_, int NL_, int OUT_, bool FINAL_ACT_>
struct Stage {
  static constexpr int IN = IN_, H = H_, NL = NL_, OUT = OUT_;
  static constexpr bool FINAL_ACT = FINAL_ACT_;
  static constexpr int din(int l) { return l == 0 ? IN : H; }
  static constexpr int dout(int l) { return l == NL - 1 ? OUT : H; }
  static constexpr bool act(int l) { return l < NL - 1 ? true : FINAL_ACT; }
  static constexpr int pad4(int x) { return (x + 3) & ~3; }
  // torch parameter order: W0[out][in], b0[out], W1, b1, ...
  static constexpr int gw(int l) {
    int o = 0;
    for (int k = 0; k < l; ++k) o += dout(k) * (din(k) + 1);
    return o;
  }
  static constexpr int gb(int l) { return gw(l) + dout(l) * din(l); }
  static constexpr int P = gw(NL);
  // LDS layout: rows of W padded to a multiple of 4 floats (ds_read_b128), bias padded
  static constexpr int lw(int l) {
    int o = 0;
    for (int k = 0; k < l; ++k) o += dout(k) * pad4(din(k)) + pad4(dout(k));
    return o;
  }
  static constexpr int lb(int l) { return lw(l) + dout(l) * pad4(din(l)); }
  static constexpr int LP = lw(NL);
  static constexpr int NPT = (P + kBlock - 1) / kBlock;  // params per thread in the optimizer phase
  // saved activations for the stage backward: h_1 .. h_{NL-1} (hidden widths)
  static constexpr int SAVED = (NL - 1) * H;
  static_assert(IN + 1 <= 16 && OUT <= 16 && (NL == 1 || H + 1 <= 16), "fused MLP kernels support widths <= 15");
};

// global parameter index -> LDS (padded) position
template <class S>
DTP_DEV int lds_pos(int p) {
  int r = 0;
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l);
    if (p >= S::gw(l) && p < S::gb(l)) {
      const int q = p - S::gw(l);
      r = S::lw(l) + (q / I) * S::pad4(I) + (q % I);
    } else if (p >= S::gb(l) && p < S::gb(l) + O) {
      r = S::lb(l) + (p - S::gb(l));
    }
  });
  return r;
}

// global parameter index -> (layer, row, col) position in the reduced dW tiles
template <class S>
DTP_DEV int tile_pos(int p) {
  int r = 0;
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l);
    if (p >= S::gw(l) && p < S::gb(l)) {
      const int q = p - S::gw(l);
      r = l * 256 + (q / I) * 16 + (q % I);
    } else if (p >= S::gb(l) && p < S::gb(l) + O) {
      r = l * 256 + (p - S::gb(l)) * 16 + I;  // bias column = I (constant-1 input)
    }
  });
  return r;
}

// forward of one sample: h[0] is the input, h[l+1] the output of layer l
template <class S>
DTP_DEV void mlp_forward(const float* __restrict__ sw, float (&h)[S::NL + 1][16], float slope) {
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l), IP = S::pad4(I);
    static_for<0, O>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      float z = sw[S::lb(l) + j];
      static_for<0, I>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        z = fmaf(sw[S::lw(l) + j * IP + i], h[l][i], z);
      });
      if constexpr (S::act(l)) {
        h[l + 1][j] = leaky(z, slope);
      } else {
        h[l + 1][j] = z;
      }
    });
  });
}

// One wave-local LDS staging area: rows = the wave's 64 samples, 16 floats per
// row; 16-byte chunks XOR-swizzled by ((row >> 1) & 3) so that both the
// row-per-lane ds_write_b128 and the MFMA-operand ds_read_b32 pattern are
// bank-conflict free (8-lane write groups hit 8 distinct 4-bank sets; each
// 32-lane read half covers banks 0..31 once).
DTP_DEV int swz(int row, int chunk) { return row * 16 + ((chunk ^ ((row >> 1) & 3)) << 2); }

template <int N>
DTP_DEV void stage_row(float* __restrict__ buf, int lane, const float (&v)[16]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float4 x;
    x.x = (4 * c + 0 < N) ? v[4 * c + 0] : 0.f;
    x.y = (4 * c + 1 < N) ? v[4 * c + 1] : 0.f;
    x.z = (4 * c + 2 < N) ? v[4 * c + 2] : 0.f;
    x.w = (4 * c + 3 < N) ? v[4 * c + 3] : 0.f;
    *reinterpret_cast<float4*>(buf + swz(lane, c)) = x;
  }
}

// acc += sum over the wave's 64 samples of dz[s] (x) h[s]   (16x16 tile)
DTP_DEV f32x4 wave_outer_acc(const float* __restrict__ dzb, const float* __restrict__ hb, f32x4 acc0, int lane) {
  const int q = lane >> 4, col = lane & 15, c = col >> 2, w = col & 3;
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 16; t += 2) {
    const int s0 = 4 * t + q, s1 = s0 + 4;
    const int o0 = swz(s0, c) + w, o1 = swz(s1, c) + w;
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(dzb[o0], hb[o0], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(dzb[o1], hb[o1], acc1, 0, 0, 0);
  }
  return acc0 + acc1;
}

// Backward of one sample through all layers, starting from dz (gradient w.r.t.
// the pre-activation output of the LAST layer).  Accumulates the wave's dW tiles
// into acc[l]; writes d(input) into dx when WANT_DX.
// stg: this wave's staging area, 2 x 1024 floats (dz rows, then h rows).
template <class S, bool WANT_DX>
DTP_DEV void mlp_backward(const float* __restrict__ sw, const float (&h)[S::NL + 1][16], float (&dz)[16],
                          float* __restrict__ stg, f32x4 (&acc)[S::NL], float slope, int lane, float (&dx)[16]) {
  float* dzb = stg;
  float* hb = stg + 1024;
  static_for<0, S::NL>([&](auto RC) {
    constexpr int l = S::NL - 1 - decltype(RC)::value;
    constexpr int I = S::din(l), O = S::dout(l), IP = S::pad4(I);
    // stage (dz_l, [h_l, 1]) for the K=batch MFMA reduction
    float hr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) hr[i] = (i < I) ? h[l][i] : (i == I ? 1.f : 0.f);
    stage_row<O>(dzb, lane, dz);
    stage_row<I + 1>(hb, lane, hr);
    // input gradient: g = W_l^T dz  (row-major reads of W_l: ds_read_b128 broadcasts)
    if constexpr (l > 0 || WANT_DX) {
      float g[16];
      static_for<0, I>([&](auto IC) { g[decltype(IC)::value] = 0.f; });
      static_for<0, O>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        static_for<0, I>([&](auto IC) {
          constexpr int i = decltype(IC)::value;
          g[i] = fmaf(sw[S::lw(l) + j * IP + i], dz[j], g[i]);
        });
      });
      if constexpr (l > 0) {
        static_for<0, I>([&](auto IC) {
          constexpr int i = decltype(IC)::value;
          dz[i] = g[i] * (S::act(l - 1) ? leaky_grad_from_out(h[l][i], slope) : 1.f);
        });
      } else {
        static_for<0, I>([&](auto IC) { dx[decltype(IC)::value] = g[decltype(IC)::value]; });
      }
    }
    __builtin_amdgcn_wave_barrier();
    acc[l] = wave_outer_acc(dzb, hb, acc[l], lane);
    __builtin_amdgcn_wave_barrier();
  });
}

// write one wave's dW partial tiles into red[wave][l][16*16]
template <class S>
DTP_DEV void store_partial_tiles(float* __restrict__ red, const f32x4 (&acc)[S::NL], int wave, int lane) {
  const int q = lane >> 4, col = lane & 15;
#pragma unroll
  for (int l = 0; l < S::NL; ++l) {
    float* t = red + (wave * S::NL + l) * 256;
#pragma unroll
    for (int r = 0; r < 4; ++r) t[(4 * q + r) * 16 + col] = acc[l][r];
  }
}

template <class S>
DTP_DEV float sum_partial_tiles(const float* __restrict__ red, int tpos, int nwaves) {
  const int l = tpos >> 8, e = tpos & 255;
  float g = 0.f;
  for (int w = 0; w < nwaves; ++w) g += red[(w * S::NL + l) * 256 + e];
  return g;
}

}  // namespace dtp
