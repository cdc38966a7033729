// Fused MLP training kernels for gfx950 (MI355X).
//
//   mlp_train_kernel  : one workgroup per model (the reference trains two
//                       independent ToyModels per iteration, demo.py:104-111),
//                       device-side sampler -> gather -> forward -> MSE/CE ->
//                       backward (MFMA weight-gradient reduction) -> optimizer,
//                       optionally for n_steps iterations inside one launch with
//                       weights, dataset and optimizer state resident in LDS /
//                       registers (no launch boundary per step).
//   mlp_stage_fwd/bwd : one stage of a layer-split model (autograd path,
//                       demo_one_model_multi_gpu.py:17-42 equivalent).
#include <cstdio>
#include <string>

#include "dtp_api.h"
#include "mlp_core.h"
#include "mlp_pair.h"
#include "optim_core.h"
#include "xgmi_core.h"

namespace dtp {

constexpr int kDataCache = 4096;  // floats of dataset that may be staged in LDS
constexpr int kPermCap = 2048;    // per-rank epoch permutation kept in LDS
constexpr int kBlock2 = 512;      // 8 waves: two lanes per sample (mlp_pair.h)
constexpr int kWaves2 = kBlock2 / kWave;

template <class S>
struct TrainSmem {
  float w[Pair<S>::pad4(Pair<S>::LW)];
  // per wave: [packed first/last tile | hidden parity 0 | hidden parity 1] x (dz rows, h rows);
  // reused for the cross-wave dW tile reduction
  float stage[kWaves2][3][2 * kStg2];
  float data[kDataCache];
  int perm[kPermCap];
};

// In-kernel phase stamps (diagnostic instantiation only, PROF = true): lane 0 of
// wave 0 records s_memtime at phase boundaries of the first 8 iterations; per-wave
// end-of-backward stamps at [8 + wave].  Never used on timed runs.
#define DTP_STAMP(K)                                                                     \
  do {                                                                                   \
    if constexpr (PROF) {                                                                \
      if (lane == 0 && it < 8 && (((K) >= 8 && (K) < 16) || wave == 0)) {                \
        unsigned long long _t;                                                           \
        __builtin_amdgcn_sched_barrier(0);                                               \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");       \
        __builtin_amdgcn_sched_barrier(0);                                               \
        prof[((size_t)blockIdx.x * 8 + it) * 32 + (K)] = _t;                             \
      }                                                                                  \
    }                                                                                    \
  } while (0)

template <class S, int MODE, bool PROF = false>
__global__ __launch_bounds__(kBlock2) void mlp_train_kernel(DtpTrainArgs a) {
  using PR = Pair<S>;
  constexpr int NL = S::NL, P = S::P, NT = PR::NT, NPT = PR::NPT, OHM = PR::OHMAX();
  static_assert(kWaves2 * NT * 256 <= kWaves2 * 3 * 2 * kStg2, "reduction tiles must fit in the staging area");
  __shared__ __align__(16) TrainSmem<S> sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane & 1, sl = lane >> 1;  // the two lanes of a sample are adjacent
  const bool upper = half != 0;
  const int model = blockIdx.x;
  constexpr bool kUpdate = MODE != DTP_MODE_GRAD;
  constexpr bool kAdam = MODE == DTP_MODE_ADAM || MODE == DTP_MODE_XGMI_ADAM;
  constexpr bool kXgmi = MODE == DTP_MODE_XGMI_ADAM || MODE == DTP_MODE_XGMI_SGD;
  unsigned long long* prof = reinterpret_cast<unsigned long long*>(a.status);
  const bool ce = a.loss == DTP_LOSS_CE;
  const int ydim = ce ? 1 : S::OUT;
  const float slope = a.hp.slope;

  // ---- parameters -> the two LDS layouts (zero padding first)
  float* __restrict__ gp = a.params + (size_t)model * P;
  for (int e = tid; e < PR::LW; e += kBlock2) sm.w[e] = 0.f;
  const SamplerCfg smp = a.smp;
  const bool cached = a.cache_data && smp.n * (S::IN + ydim) <= kDataCache;
  if (cached) {
    for (int e = tid; e < smp.n * S::IN; e += kBlock2) sm.data[e] = a.X[e];
    for (int e = tid; e < smp.n * ydim; e += kBlock2) sm.data[smp.n * S::IN + e] = a.Y[e];
  }
  const float* __restrict__ Xg = a.X;
  const float* __restrict__ Yg = a.Y;
  const int yoff = smp.n * S::IN;
  __syncthreads();
  for (int p = tid; p < P; p += kBlock2) {
    int pf, pb;
    pair_pos<S>(p, pf, pb);
    const float v = gp[p];
    sm.w[pf] = v;
    if (pb >= 0) sm.w[pb] = v;
  }
  // this thread owns parameters tid, tid+512, ... in the optimizer phase
  int lpf[NPT], lpb[NPT], tp[NPT];
  float mr[NPT], vr[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int p = tid + k * kBlock2;
    pair_pos<S>(p < P ? p : 0, lpf[k], lpb[k]);
    tp[k] = pair_tile_pos<S>(p < P ? p : 0);
    mr[k] = 0.f;
    vr[k] = 0.f;
    if (kUpdate && p < P) {
      mr[k] = a.opt_m[(size_t)model * P + p];
      if (kAdam) vr[k] = a.opt_v[(size_t)model * P + p];
    }
  }
  // 32-bit step bookkeeping, advanced incrementally (no 64-bit divisions per step)
  const int t0 = a.step[model];
  const bool explicit_idx = smp.mode == SAMPLER_EXPLICIT;
  int epoch = explicit_idx ? 0 : t0 / smp.steps_per_epoch;
  int bi = explicit_idx ? 0 : t0 - epoch * smp.steps_per_epoch;
  int lslot = a.loss_log ? t0 % a.loss_log_cap : 0;
  uint32_t keys[4];
  epoch_keys(smp, epoch, keys);
  // the shuffled epoch order is computed once per epoch into LDS (cooperatively)
  const bool use_perm = smp.mode == SAMPLER_DIST_SHUFFLE && smp.num_samples <= kPermCap;
  auto fill_perm = [&](int ep) {
    uint32_t kk[4];
    epoch_keys(smp, ep, kk);
    const BatchPos b0{ep, 0, 0};
    for (int pos = tid; pos < smp.num_samples; pos += kBlock2) sm.perm[pos] = sample_index(smp, b0, kk, pos);
  };
  if (use_perm) fill_perm(epoch);
  // Adam bias-correction powers beta^t, carried in double like torch's host math
  double b1t = kAdam ? pow_int(a.hp.beta1, (uint64_t)t0) : 1.0;
  double b2t = kAdam ? pow_int(a.hp.beta2, (uint64_t)t0) : 1.0;
  unsigned xepoch = kXgmi ? a.epoch[model] : 0u;
  float* const stg_pack = &sm.stage[wave][0][0];
  __syncthreads();

  for (int it = 0; it < a.n_steps; ++it) {
    DTP_STAMP(0);
    const int t = t0 + it;
    BatchPos bp;
    bp.epoch = epoch;
    bp.start = bi * smp.batch;
    bp.size = explicit_idx ? smp.batch : min(smp.batch, smp.num_samples - bp.start);
    const int bsz = bp.size;
    const float inv = ce ? 1.f / (float)bsz : 1.f / (float)(bsz * S::OUT);

    f32x4 acc[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int c0 = 0; c0 < bsz; c0 += kWaves2 * 32) {
      const int k = c0 + wave * 32 + sl;
      const bool valid = k < bsz;
      int di = 0;
      if (valid)
        di = explicit_idx ? a.idx[(size_t)it * smp.batch + k]
                          : (use_perm ? sm.perm[bp.start + k] : sample_index(smp, bp, keys, k));
      float x[S::IN];
      if (cached) {
        static_for<0, S::IN>([&](auto IC) {
          constexpr int i = decltype(IC)::value;
          x[i] = valid ? sm.data[di * S::IN + i] : 0.f;
        });
      } else {
        static_for<0, S::IN>([&](auto IC) {
          constexpr int i = decltype(IC)::value;
          x[i] = valid ? Xg[(size_t)di * S::IN + i] : 0.f;
        });
      }
      if (c0 == 0) DTP_STAMP(1);

      // ---------------- forward: this lane computes its half of every layer
      float aown[NL][OHM];  // aown[l] = own half of layer l's output (post-activation for l < NL-1)
      static_for<0, NL>([&](auto LC) {
        constexpr int l = decltype(LC)::value;
        constexpr int OH = PR::OH(l), OHP = PR::OHP(l), NIN = PR::NIN(l), IHM = PR::IHM(l);
        const float* wb = sm.w + PR::fwo(l) + half * PR::FH(l);
        float4 w4[NIN][OHP / 4];
        float4 b4[OHP / 4];
        static_for<0, OHP / 4>([&](auto QC) {
          constexpr int q = decltype(QC)::value;
          b4[q] = *reinterpret_cast<const float4*>(wb + PR::FB(l) + 4 * q);
          static_for<0, NIN>([&](auto MC) {
            constexpr int m = decltype(MC)::value;
            w4[m][q] = *reinterpret_cast<const float4*>(wb + m * OHP + 4 * q);
          });
        });
        float in[NIN];
        if constexpr (l == 0) {
          static_for<0, NIN>([&](auto MC) { in[decltype(MC)::value] = x[decltype(MC)::value]; });
        } else {
          static_for<0, IHM>([&](auto MC) {
            constexpr int m = decltype(MC)::value;
            in[m] = aown[l - 1][m];
            in[IHM + m] = partner(aown[l - 1][m]);
          });
        }
        float z[OHP];
        static_for<0, OHP / 4>([&](auto QC) {
          constexpr int q = decltype(QC)::value;
          z[4 * q + 0] = b4[q].x;
          z[4 * q + 1] = b4[q].y;
          z[4 * q + 2] = b4[q].z;
          z[4 * q + 3] = b4[q].w;
        });
        static_for<0, NIN>([&](auto MC) {
          constexpr int m = decltype(MC)::value;
          const float v = in[m];
          static_for<0, OHP / 4>([&](auto QC) {
            constexpr int q = decltype(QC)::value;
            if constexpr (4 * q + 0 < OH) z[4 * q + 0] = fmaf(w4[m][q].x, v, z[4 * q + 0]);
            if constexpr (4 * q + 1 < OH) z[4 * q + 1] = fmaf(w4[m][q].y, v, z[4 * q + 1]);
            if constexpr (4 * q + 2 < OH) z[4 * q + 2] = fmaf(w4[m][q].z, v, z[4 * q + 2]);
            if constexpr (4 * q + 3 < OH) z[4 * q + 3] = fmaf(w4[m][q].w, v, z[4 * q + 3]);
          });
        });
        static_for<0, OH>([&](auto KC) {
          constexpr int kk = decltype(KC)::value;
          aown[l][kk] = S::act(l) ? leaky(z[kk], slope) : z[kk];
        });
        if (c0 == 0) DTP_STAMP(16 + l);
      });

      // ---------------- loss on the output half (MSE / CE)
      constexpr int L = NL - 1;
      constexpr int OHL = PR::OH(L);
      float dz[OHM];
      float lpart = 0.f;
      const int jbeg = half * OHL;
      const int jcnt = upper ? (S::OUT - OHL) : OHL;
      if (!ce) {
        static_for<0, OHL>([&](auto KC) {
          constexpr int kk = decltype(KC)::value;
          const bool own = kk < jcnt;
          float y = 0.f;
          if (valid && own) y = cached ? sm.data[yoff + di * S::OUT + jbeg + kk] : Yg[(size_t)di * S::OUT + jbeg + kk];
          const float d = aown[L][kk] - y;
          lpart += (valid && own) ? d * d : 0.f;
          dz[kk] = (valid && own) ? 2.f * d * inv : 0.f;
        });
      } else {
        // all logits on both lanes of the pair
        float lg[2 * OHL];
        static_for<0, OHL>([&](auto KC) {
          constexpr int kk = decltype(KC)::value;
          const float o = partner(aown[L][kk]);
          lg[kk] = upper ? o : aown[L][kk];
          lg[OHL + kk] = upper ? aown[L][kk] : o;
        });
        const int cls = valid ? (int)(cached ? sm.data[yoff + di] : Yg[di]) : 0;
        float mx = lg[0];
        static_for<1, S::OUT>([&](auto JC) { mx = fmaxf(mx, lg[decltype(JC)::value]); });
        float se = 0.f, zc = 0.f;
        static_for<0, S::OUT>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          se += __expf(lg[j] - mx);
          zc = (j == cls) ? lg[j] : zc;
        });
        const float lse = mx + __logf(se);
        const float rs = 1.f / se;
        lpart = (valid && !upper) ? lse - zc : 0.f;
        static_for<0, OHL>([&](auto KC) {
          constexpr int kk = decltype(KC)::value;
          const int j = jbeg + kk;
          const float zj = aown[L][kk];
          dz[kk] = (valid && kk < jcnt) ? (__expf(zj - mx) * rs - (j == cls ? 1.f : 0.f)) * inv : 0.f;
        });
      }
      if (c0 == 0) DTP_STAMP(2);

      // ---------------- backward: dX chain (VALU, halves) + dW tiles (MFMA, K = samples)
      static_for<0, NL>([&](auto RC) {
        constexpr int l = NL - 1 - decltype(RC)::value;
        constexpr int OH = PR::OH(l), IHM = PR::IHM(l);
        constexpr bool packed = PR::PACK && (l == 0 || l == NL - 1);
        float* stg = packed ? stg_pack : &sm.stage[wave][1 + (l & 1)][0];
        float* dzb = stg;
        float* hb = stg + kStg2;
        // dz rows of this layer (own half), the loss rows with the last layer
        const int ocnt = upper ? (S::dout(l) - OH) : OH;
        static_for<0, OH>([&](auto KC) {
          constexpr int kk = decltype(KC)::value;
          if (kk < ocnt) stg2_write(dzb, sl, PR::rowoff(l) + half * OH + kk, dz[kk]);
        });
        if constexpr (l == NL - 1) stg2_write(dzb, sl, PR::lossrow() + half, lpart);
        // input columns of this layer (own half) + the constant-1 bias column
        if constexpr (l == 0) {
          if (!upper) {
            static_for<0, S::IN>([&](auto MC) { stg2_write(hb, sl, PR::coloff(0) + decltype(MC)::value, x[decltype(MC)::value]); });
            stg2_write(hb, sl, PR::coloff(0) + S::IN, 1.f);
          }
        } else {
          const int icnt = upper ? (S::din(l) - IHM) : IHM;
          static_for<0, IHM>([&](auto MC) {
            constexpr int m = decltype(MC)::value;
            if (m < icnt) stg2_write(hb, sl, PR::coloff(l) + half * IHM + m, aown[l - 1][m]);
          });
          if (upper) stg2_write(hb, sl, PR::coloff(l) + S::din(l), 1.f);
        }
        if constexpr (!packed) {  // the packed first/last tile runs once, after layer 0's rows
          __builtin_amdgcn_wave_barrier();
          acc[PR::tile(l)] = wave_outer_acc32(dzb, hb, acc[PR::tile(l)], lane);
          __builtin_amdgcn_wave_barrier();
        }
        if constexpr (l > 0) {
          constexpr int IHP = PR::IHP(l);
          const float* wb = sm.w + PR::bwo(l) + half * PR::BH(l);
          float4 bw[2 * OH][IHP / 4];
          static_for<0, 2 * OH>([&](auto MC) {
            static_for<0, IHP / 4>([&](auto QC) {
              bw[decltype(MC)::value][decltype(QC)::value] =
                  *reinterpret_cast<const float4*>(wb + decltype(MC)::value * IHP + 4 * decltype(QC)::value);
            });
          });
          float dfull[2 * OH];
          static_for<0, OH>([&](auto KC) {
            constexpr int kk = decltype(KC)::value;
            dfull[kk] = dz[kk];
            dfull[OH + kk] = partner(dz[kk]);
          });
          float g[IHP];
          static_for<0, IHP>([&](auto KC) { g[decltype(KC)::value] = 0.f; });
          static_for<0, 2 * OH>([&](auto MC) {
            constexpr int m = decltype(MC)::value;
            const float d = dfull[m];
            static_for<0, IHP / 4>([&](auto QC) {
              constexpr int q = decltype(QC)::value;
              if constexpr (4 * q + 0 < IHM) g[4 * q + 0] = fmaf(bw[m][q].x, d, g[4 * q + 0]);
              if constexpr (4 * q + 1 < IHM) g[4 * q + 1] = fmaf(bw[m][q].y, d, g[4 * q + 1]);
              if constexpr (4 * q + 2 < IHM) g[4 * q + 2] = fmaf(bw[m][q].z, d, g[4 * q + 2]);
              if constexpr (4 * q + 3 < IHM) g[4 * q + 3] = fmaf(bw[m][q].w, d, g[4 * q + 3]);
            });
          });
          static_for<0, IHM>([&](auto KC) {
            constexpr int kk = decltype(KC)::value;
            dz[kk] = g[kk] * (S::act(l - 1) ? leaky_grad_from_out(aown[l - 1][kk], slope) : 1.f);
          });
        }
        if (c0 == 0) DTP_STAMP(24 + l);
      });
      if constexpr (PR::PACK) {
        __builtin_amdgcn_wave_barrier();
        acc[0] = wave_outer_acc32(stg_pack, stg_pack + kStg2, acc[0], lane);
      }
    }
    DTP_STAMP(8 + wave);
    DTP_STAMP(3);
    __syncthreads();  // every wave is done with its staging rows
    {
      float* red = &sm.stage[0][0][0];
      const int q = lane >> 4, col = lane & 15;
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        float* tl = red + (wave * NT + tt) * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) tl[(4 * q + r) * 16 + col] = acc[tt][r];
      }
    }
    __syncthreads();
    DTP_STAMP(4);

    const float* red = &sm.stage[0][0][0];
    float g[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int tpos = tp[k];
      const int tt = tpos >> 8, e = tpos & 255;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves2; ++w) s += red[(w * NT + tt) * 256 + e];
      g[k] = s;
    }
    float lsum = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves2; ++w) {
      lsum += red[(w * NT + PR::tile(NL - 1)) * 256 + PR::lossrow() * 16 + PR::losscol()];
      lsum += red[(w * NT + PR::tile(NL - 1)) * 256 + (PR::lossrow() + 1) * 16 + PR::losscol()];
    }
    const float mean_loss = lsum * inv;
    DTP_STAMP(5);

    float gloss = mean_loss;
    if constexpr (kXgmi) {
      // all-reduce (sum) this model's gradient + loss over every rank through
      // the peers' xGMI-mapped receive buffers, inside the step (xgmi_core.h)
      xepoch += 1u;
      gloss = xgmi_allreduce_model<NPT, kBlock2>(a, model, P, g, mean_loss, xepoch, tid);
    }

    if (tid == 0 && a.loss_log) {
      const float lg = kXgmi ? gloss * a.hp.grad_scale : mean_loss;
      a.loss_log[(size_t)lslot * a.n_models + model] = lg;
    }

    if constexpr (MODE == DTP_MODE_GRAD) {
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int p = tid + k * kBlock2;
        if (p < P) a.grad_out[(size_t)model * P + p] = g[k] * a.hp.grad_scale;
      }
      if (tid == 0) a.grad_out[(size_t)a.n_models * P + model] = mean_loss;
    } else if constexpr (kAdam) {
      b1t *= a.hp.beta1;
      b2t *= a.hp.beta2;
      const AdamScalars s = adam_scalars_from_pow(a.hp, b1t, b2t);
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int p = tid + k * kBlock2;
        if (p < P) {
          float w = sm.w[lpf[k]];
          adam_update(w, mr[k], vr[k], g[k] * a.hp.grad_scale, s);
          sm.w[lpf[k]] = w;
          if (lpb[k] >= 0) sm.w[lpb[k]] = w;
        }
      }
    } else {
      const float lr = (float)a.hp.lr, mom = (float)a.hp.momentum, wd = (float)a.hp.weight_decay;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int p = tid + k * kBlock2;
        if (p < P) {
          float w = sm.w[lpf[k]];
          sgd_update(w, mr[k], g[k] * a.hp.grad_scale, lr, mom, wd, t == 0);
          sm.w[lpf[k]] = w;
          if (lpb[k] >= 0) sm.w[lpb[k]] = w;
        }
      }
    }
    DTP_STAMP(6);
    // advance the sampler / loss-ring position
    if (!explicit_idx && ++bi == smp.steps_per_epoch) {
      bi = 0;
      ++epoch;
      epoch_keys(smp, epoch, keys);
      if (use_perm && it + 1 < a.n_steps) fill_perm(epoch);  // ordered by the barrier below
    }
    if (a.loss_log && ++lslot == a.loss_log_cap) lslot = 0;
    __syncthreads();  // updated weights visible; reduction tiles consumed
    DTP_STAMP(7);
  }

  if constexpr (kUpdate) {
    for (int p = tid; p < P; p += kBlock2) {
      int pf, pb;
      pair_pos<S>(p, pf, pb);
      gp[p] = sm.w[pf];
    }
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int p = tid + k * kBlock2;
      if (p < P) {
        a.opt_m[(size_t)model * P + p] = mr[k];
        if (kAdam) a.opt_v[(size_t)model * P + p] = vr[k];
      }
    }
    if (tid == 0) a.step[model] = t0 + a.n_steps;
    if (kXgmi && tid == 0) a.epoch[model] = xepoch;
  }
}

// ------------------------------------------------------------------------------
__global__ void sampler_probe_kernel(SamplerCfg s, long long t0, int n_steps, int* out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int st = blockIdx.y;
  if (k >= s.batch || st >= n_steps) return;
  const BatchPos bp = batch_pos(s, t0 + st);
  uint32_t keys[4];
  epoch_keys(s, bp.epoch, keys);
  out[(size_t)st * s.batch + k] = (k < bp.size) ? sample_index(s, bp, keys, k) : -1;
}

}  // namespace dtp

// ------------------------------------------------------------------------------
// dispatch tables
namespace {
using dtp::check_launch;
using dtp::set_err;

// (IN, H, NL, OUT): shapes the fused train-step kernel is instantiated for
#define DTP_TRAIN_SHAPES(X) \
  X(2, 10, 5, 1)            \
  X(2, 10, 3, 1)            \
  X(2, 10, 5, 4)            \
  X(2, 15, 5, 1)

template <class S>
int launch_train(const DtpTrainArgs* a, int mode, hipStream_t st) {
  dim3 grid(a->n_models), block(dtp::kBlock2);
  switch (mode) {
    case DTP_MODE_GRAD:
      if (a->n_steps != 1) return set_err(-4, "MODE_GRAD requires n_steps == 1");
      hipLaunchKernelGGL((dtp::mlp_train_kernel<S, DTP_MODE_GRAD>), grid, block, 0, st, *a);
      break;
    case DTP_MODE_ADAM:
      hipLaunchKernelGGL((dtp::mlp_train_kernel<S, DTP_MODE_ADAM>), grid, block, 0, st, *a);
      break;
    case DTP_MODE_SGD:
      hipLaunchKernelGGL((dtp::mlp_train_kernel<S, DTP_MODE_SGD>), grid, block, 0, st, *a);
      break;
    case DTP_MODE_XGMI_ADAM:
      hipLaunchKernelGGL((dtp::mlp_train_kernel<S, DTP_MODE_XGMI_ADAM>), grid, block, 0, st, *a);
      break;
    case DTP_MODE_XGMI_SGD:
      hipLaunchKernelGGL((dtp::mlp_train_kernel<S, DTP_MODE_XGMI_SGD>), grid, block, 0, st, *a);
      break;
    default:
      return set_err(-2, "unknown train mode");
  }
  return check_launch("mlp_train_kernel");
}

template <class S>
int launch_train_profile(const DtpTrainArgs* a, hipStream_t st) {
  hipLaunchKernelGGL((dtp::mlp_train_kernel<S, DTP_MODE_ADAM, true>), dim3(a->n_models), dim3(dtp::kBlock2), 0, st, *a);
  return check_launch("mlp_train_kernel<prof>");
}

}  // namespace

extern "C" {


int dtp_mlp_param_count(int in, int h, int nl, int out) {
  int p = 0;
  for (int l = 0; l < nl; ++l) {
    const int di = l == 0 ? in : h, dq = l == nl - 1 ? out : h;
    p += dq * (di + 1);
  }
  return p;
}

int dtp_mlp_train(const DtpTrainArgs* a, int in, int h, int nl, int out, int mode, void* stream) {
  if (!a) return set_err(-1, "null args");
  if (a->n_models <= 0 || a->n_steps <= 0) return set_err(-1, "n_models and n_steps must be positive");
  if (a->smp.batch <= 0 || a->smp.n <= 0) return set_err(-1, "empty dataset or batch");
  if (a->smp.mode != dtp::SAMPLER_EXPLICIT && (a->smp.steps_per_epoch <= 0 || a->smp.num_samples <= 0))
    return set_err(-1, "bad sampler geometry");
  if (a->loss_log && a->loss_log_cap <= 0) return set_err(-1, "loss_log_cap must be positive");
  hipStream_t st = (hipStream_t)stream;
#define X(I, H, N, O) \
  if (in == I && h == H && nl == N && out == O) return launch_train<dtp::Stage<I, H, N, O, false>>(a, mode, st);
  DTP_TRAIN_SHAPES(X)
#undef X
  return set_err(-2, "mlp shape not instantiated for the fused train kernel");
}

// diagnostic: toy shape, Adam, phase stamps into a->status (as u64[n_models][8][16])
int dtp_mlp_train_profile(const DtpTrainArgs* a, void* stream) {
  return launch_train_profile<dtp::Stage<2, 10, 5, 1, false>>(a, (hipStream_t)stream);
}

int dtp_sampler_indices(const dtp::SamplerCfg* s, long long t0, int n_steps, int* out, void* stream) {
  if (!s || !out || s->batch <= 0 || n_steps <= 0) return set_err(-1, "bad sampler probe args");
  dim3 grid((s->batch + 255) / 256, n_steps), block(256);
  hipLaunchKernelGGL(dtp::sampler_probe_kernel, grid, block, 0, (hipStream_t)stream, *s, t0, n_steps, out);
  return check_launch("sampler_probe_kernel");
}

}  // extern "C"
