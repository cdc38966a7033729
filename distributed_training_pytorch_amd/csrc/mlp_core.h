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
// BF: bf16 compute (the autocast recipe): every matmul operand -- weights,
// activations, backward gradients -- is rounded to bf16 (rnd), products are exact in
// fp32 and accumulate in fp32 (FMA chains and the fp32 MFMA dW tiles: the numerics of
// a bf16 MFMA with fp32 accumulation); master weights, weight gradients and the
// optimizer stay fp32.  BF = false compiles every rnd() away.
template <int IN_, int H_, int NL_, int OUT_, bool FINAL_ACT_, bool BF_ = false>
struct Stage {
  static constexpr int IN = IN_, H = H_, NL = NL_, OUT = OUT_;
  static constexpr bool FINAL_ACT = FINAL_ACT_;
  static constexpr bool BF = BF_;
  static DTP_DEV float rnd(float v) {
    if constexpr (BF) {
      return (float)(__bf16)v;  // v_cvt_pk_bf16_f32: round to nearest even
    } else {
      return v;
    }
  }
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
  static constexpr int LPR = lw(NL);
  // second, transposed copy W^T[in][pad4(out)] for the forward: consecutive
  // outputs j, j+1 of one input i are adjacent -> v_pk_fma_f32 straight from a
  // ds_read_b128, no register shuffles (the backward reads the row-major copy)
  static constexpr int lwt(int l) {
    int o = LPR;
    for (int k = 0; k < l; ++k) o += din(k) * pad4(dout(k));
    return o;
  }
  static constexpr int LP = lwt(NL);
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

// global parameter index -> position in the transposed forward copy (-1 for biases)
template <class S>
DTP_DEV int lds_pos_t(int p) {
  int r = -1;
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l);
    if (p >= S::gw(l) && p < S::gb(l)) {
      const int q = p - S::gw(l);
      r = S::lwt(l) + (q % I) * S::pad4(O) + (q / I);
    }
  });
  return r;
}

// stage parameter p (torch order) into both LDS copies
template <class S>
DTP_DEV void lds_store_param(float* __restrict__ sw, int p, float v) {
  v = S::rnd(v);  // bf16 compute: the matmul operand is the bf16 weight
  sw[lds_pos<S>(p)] = v;
  const int t = lds_pos_t<S>(p);
  if (t >= 0) sw[t] = v;
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

// forward of one sample: h[0] is the input, h[l+1] the output of layer l.
// Each layer first pulls its whole W^T slice out of LDS (broadcast
// ds_read_b128, all issued back to back so their latency overlaps), then runs
// the FMA chains (pairs of outputs per v_pk_fma_f32).
template <class S>
DTP_DEV void mlp_forward(const float* __restrict__ sw, float (&h)[S::NL + 1][16], float slope) {
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l), OP = S::pad4(O);
    float4 wt[I][OP / 4];
    float4 bb[OP / 4];
    static_for<0, OP / 4>([&](auto QC) {
      constexpr int q = decltype(QC)::value;
      bb[q] = *reinterpret_cast<const float4*>(sw + S::lb(l) + 4 * q);
      static_for<0, I>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        wt[i][q] = *reinterpret_cast<const float4*>(sw + S::lwt(l) + i * OP + 4 * q);
      });
    });
    float z[OP];
    static_for<0, OP / 4>([&](auto QC) {
      constexpr int q = decltype(QC)::value;
      z[4 * q + 0] = bb[q].x;
      z[4 * q + 1] = bb[q].y;
      z[4 * q + 2] = bb[q].z;
      z[4 * q + 3] = bb[q].w;
    });
    static_for<0, I>([&](auto IC) {
      constexpr int i = decltype(IC)::value;
      const float hi = h[l][i];
      static_for<0, OP / 4>([&](auto QC) {
        constexpr int q = decltype(QC)::value;
        if constexpr (4 * q + 0 < O) z[4 * q + 0] = fmaf(wt[i][q].x, hi, z[4 * q + 0]);
        if constexpr (4 * q + 1 < O) z[4 * q + 1] = fmaf(wt[i][q].y, hi, z[4 * q + 1]);
        if constexpr (4 * q + 2 < O) z[4 * q + 2] = fmaf(wt[i][q].z, hi, z[4 * q + 2]);
        if constexpr (4 * q + 3 < O) z[4 * q + 3] = fmaf(wt[i][q].w, hi, z[4 * q + 3]);
      });
    });
    static_for<0, O>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      if constexpr (S::act(l)) {
        h[l + 1][j] = S::rnd(leaky(S::rnd(z[j]), slope));  // bf16 Linear output, then bf16 LeakyReLU
      } else {
        h[l + 1][j] = S::rnd(z[j]);
      }
    });
  });
}

// One wave-local LDS staging area per operand (dz rows, h rows): the wave's 64
// samples s = 4t + q are stored as [q][col][t] (q stride kStgQ = 264 floats), so
//   * the writer (lane = sample) issues one ds_write_b32 per used column; for a
//     fixed column the 32 lanes of a half hit 32 distinct banks (264 = 8 mod 32);
//   * the MFMA reader (lane = (q = l>>4, col = l&15)) finds its 16 K-step operands
//     contiguous: 4 ds_read_b128, one wait, then 16 back-to-back MFMAs.
// Unused columns are never written: garbage there only reaches tile rows/cols
// nobody reads (D[i][j] depends on A row i and B column j only).
constexpr int kStgQ = 264;
constexpr int kStgArr = 4 * kStgQ;  // floats per staged operand array

template <int N>
DTP_DEV void stage_row(float* __restrict__ buf, int lane, const float (&v)[16]) {
  float* p = buf + (lane & 3) * kStgQ + (lane >> 2);
#pragma unroll
  for (int c = 0; c < N; ++c) p[c * 16] = v[c];
}

// acc += sum over the wave's 64 samples of dz[s] (x) h[s]   (16x16 tile)
DTP_DEV f32x4 wave_outer_acc(const float* __restrict__ dzb, const float* __restrict__ hb, f32x4 acc0, int lane) {
  const int off = (lane >> 4) * kStgQ + (lane & 15) * 16;
  const float4* a4 = reinterpret_cast<const float4*>(dzb + off);
  const float4* b4 = reinterpret_cast<const float4*>(hb + off);
  float4 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = a4[i];
    b[i] = b4[i];
  }
  // all eight reads in flight before the first MFMA waits (left alone, the
  // scheduler pairs each read with its MFMAs: four LDS round trips in a row)
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, b[i].x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, b[i].y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, b[i].z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, b[i].w, acc1, 0, 0, 0);
  }
  return acc0 + acc1;
}

// Backward of one sample through all layers, starting from dz (gradient w.r.t.
// the pre-activation output of the LAST layer).  Accumulates the wave's dW tiles
// into acc[l]; writes d(input) into dx when WANT_DX.
// stg: this wave's staging area, 2 x kStgArr floats (dz rows, then h rows).
// LOSS_ROW: dz[OUT] carries the sample's loss value into an otherwise unused
// row of the output-layer tile; against the constant-1 bias column it sums the
// batch loss inside the same MFMAs (tile entry (NL-1, OUT, din(NL-1))).
template <class S, bool WANT_DX, bool LOSS_ROW = false>
DTP_DEV void mlp_backward(const float* __restrict__ sw, const float (&h)[S::NL + 1][16], float (&dz)[16],
                          float* __restrict__ stg, f32x4 (&acc)[S::NL], float slope, int lane, float (&dx)[16]) {
  float* dzb = stg;
  float* hb = stg + kStgArr;
  static_for<0, S::NL>([&](auto RC) {
    constexpr int l = S::NL - 1 - decltype(RC)::value;
    constexpr int I = S::din(l), O = S::dout(l), IP = S::pad4(I);
    // stage (dz_l, [h_l, 1]) for the K=batch MFMA reduction
    float hr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) hr[i] = (i < I) ? h[l][i] : (i == I ? 1.f : 0.f);
    if constexpr (LOSS_ROW && l == S::NL - 1) {
      static_assert(S::OUT + 1 <= 16, "loss row needs a free tile row");
      stage_row<O + 1>(dzb, lane, dz);
    } else {
      stage_row<O>(dzb, lane, dz);
    }
    stage_row<I + 1>(hb, lane, hr);
    // input gradient: g = W_l^T dz  (row-major reads of W_l: ds_read_b128 broadcasts)
    if constexpr (l > 0 || WANT_DX) {
      float4 wr[O][IP / 4];
      static_for<0, O>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        static_for<0, IP / 4>([&](auto QC) {
          constexpr int q = decltype(QC)::value;
          wr[j][q] = *reinterpret_cast<const float4*>(sw + S::lw(l) + j * IP + 4 * q);
        });
      });
      float g[IP];
      static_for<0, IP>([&](auto IC) { g[decltype(IC)::value] = 0.f; });
      static_for<0, O>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        const float d = dz[j];
        static_for<0, IP / 4>([&](auto QC) {
          constexpr int q = decltype(QC)::value;
          if constexpr (4 * q + 0 < I) g[4 * q + 0] = fmaf(wr[j][q].x, d, g[4 * q + 0]);
          if constexpr (4 * q + 1 < I) g[4 * q + 1] = fmaf(wr[j][q].y, d, g[4 * q + 1]);
          if constexpr (4 * q + 2 < I) g[4 * q + 2] = fmaf(wr[j][q].z, d, g[4 * q + 2]);
          if constexpr (4 * q + 3 < I) g[4 * q + 3] = fmaf(wr[j][q].w, d, g[4 * q + 3]);
        });
      });
      if constexpr (l > 0) {
        static_for<0, I>([&](auto IC) {
          constexpr int i = decltype(IC)::value;
          dz[i] = S::rnd(S::rnd(g[i]) * (S::act(l - 1) ? leaky_grad_from_out(h[l][i], slope) : 1.f));
        });
      } else {
        static_for<0, I>([&](auto IC) { dx[decltype(IC)::value] = S::rnd(g[decltype(IC)::value]); });
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

// tile position of the loss row entry (see mlp_backward LOSS_ROW)
template <class S>
constexpr int loss_tile_pos() { return (S::NL - 1) * 256 + S::OUT * 16 + S::din(S::NL - 1); }

template <class S>
DTP_DEV float sum_partial_tiles(const float* __restrict__ red, int tpos, int nwaves) {
  const int l = tpos >> 8, e = tpos & 255;
  float g = 0.f;
  for (int w = 0; w < nwaves; ++w) g += red[(w * S::NL + l) * 256 + e];
  return g;
}

}  // namespace dtp
