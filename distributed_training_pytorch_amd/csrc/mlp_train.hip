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
#include <cstdlib>
#include <cstring>
#include <string>

#include "dtp_api.h"
#include "mlp_core.h"
#include "mlp_lanes.h"
#include "mlp_pipe.h"
#include "mlp_scalar.h"
#include "optim_core.h"
#include "xgmi_core.h"
#include "grp_core.h"

namespace dtp {

// floats of dataset staged in LDS: the whole weak-scaling dataset of an 8-GPU
// node (n = 512 x 8 samples x (2 inputs + 1 target)) stays on-chip
constexpr int kDataCache = 12288;
// Adam bias-correction scalars of the next kAdamTab steps, formed cooperatively in
// f64 (torch's host math) once per kAdamTab steps instead of per step
constexpr int kAdamTab = 1024;
#ifndef DTP_PIPE
#define DTP_PIPE 1  // software-pipelined forward/backward (mlp_pipe.h); 0 = the v5 schedule
#endif

constexpr int kWaves = kBlock / kWave;

#ifndef DTP_GRP_SPLIT
#define DTP_GRP_SPLIT 1  // split-batch exchange: publisher / poller waves (grp_allreduce_split); 0: every thread both
#endif
#ifndef DTP_GRP_DIRECT
// 1: the publisher wave sums its granules from the dW tiles itself (no staging, no barrier):
// measured slower (3.70 vs 3.61 us/step: 24 scattered tile reads on the publisher's path
// against one LDS round and a barrier, profiles/r5_exchange/direct_ab/)
#define DTP_GRP_DIRECT 0
#endif

#ifndef DTP_XWAIT
#define DTP_XWAIT 1  // 0 (A/B builds only): no exchange-wait diagnostic (bench exchange_wait_us_per_step)
#endif

// entries base + tid + j * kBlock (j < J) of the host's Adam table for a launch starting
// at step t0: {lr / (1 - b1^t1), sqrt(1 - b2^t1)} with t1 = t0 + e + 1, clamped to the
// table's saturated last row
// (only the rows the launch's n_steps reach: a 20-step launch loads 20 entries, not 1024)
template <int J, int NTH = kBlock>
DTP_DEV void adam_tab_load(const DtpTrainArgs& a, int t0, int base, int tid, float2 (&v)[J]) {
  const float2* __restrict__ tab = reinterpret_cast<const float2*>(a.adam_tab);
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int e = base + tid + j * NTH;
    const long long t1 = (long long)t0 + e + 1;
    v[j] = make_float2(0.f, 1.f);
    if (e < a.n_steps) v[j] = tab[t1 < a.adam_tab_len ? t1 : a.adam_tab_len - 1];
  }
}
template <int J, int NTH = kBlock>
DTP_DEV void adam_tab_store(float2* __restrict__ lds, int n, int tid, const float2 (&v)[J]) {
#pragma unroll
  for (int j = 0; j < J; ++j)
    if (tid + j * NTH < n) lds[tid + j * NTH] = v[j];
}

template <class S, bool XCH = false>
struct TrainSmem {
  float wb[Scal<S>::LW];  // backward + forward weight blocks (mlp_scalar.h)
  float2 adam_tab[kAdamTab];  // per-step Adam scalars {lr / (1 - b1^t), sqrt(1 - b2^t)}
  // per wave: [packed first/last tile | hidden layer] x (dz rows, h rows) -- one hidden
  // buffer suffices: a wave's LDS ops execute in order, so layer l-1's staging
  // writes land after layer l's operand reads were issued; reused for the
  // cross-wave dW tile reduction
  float stage[kWaves][2][2 * kStgArr];
  float data[kDataCache];
  float sink[4];  // target of the optimizer's predicated-off stores (slots past P)
  float lossw[kBlock / kWave];  // bf16 instances: per-wave batch-loss sums (not through a bf16 tile)
  // xGMI instances: the split exchange's payloads (xgmi_allreduce_split)
  alignas(16) float2 xg[XCH ? xgmi_split_lds_f2<S::P, S::NPT>() : 2];
};

// One lane's sample of a step: input, target (class index for CE) and validity.
template <class S>
struct SampleRegs {
  float x[S::IN];
  float y[S::OUT];
  bool valid;
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

// Fused train step(s), one workgroup (4 waves, one lane per sample) per model.
// Weights live in LDS blocks read into registers one layer ahead (mlp_pipe.h),
// activations in VGPRs, the dW reduction
// over the batch runs on MFMA through a per-wave LDS staging area, the optimizer
// owns NPT parameters per thread in registers (params and moments).
#ifndef DTP_TRAIN_WAVES_PER_EU
#define DTP_TRAIN_WAVES_PER_EU 1  // one wave per SIMD: the scheduler may spend registers on latency
#endif
#if DTP_TRAIN_WAVES_PER_EU
#define DTP_TRAIN_ATTR __attribute__((amdgpu_waves_per_eu(DTP_TRAIN_WAVES_PER_EU, DTP_TRAIN_WAVES_PER_EU)))
#else
#define DTP_TRAIN_ATTR
#endif
// FAST: the common configuration fixed at compile time (MSE, batch <= 256, the
// SAMPLER_TABLE sampler -- the epoch permutations in a device ring the host fills
// ahead, torch's exact DistributedSampler order by default --, dataset cached in LDS,
// 0 <= slope <= 1; fast_path_ok() on the host): each lane's dataset index is loaded
// from the ring a whole step before it is used, so the next step's sample gather
// is straight-line LDS code the scheduler interleaves with the optimizer, and
// LeakyReLU is max(z, slope z).
template <class S, int MODE, bool PROF = false, bool FAST = false>
__global__ __launch_bounds__(kBlock) DTP_TRAIN_ATTR void mlp_train_kernel(DtpTrainArgs a) {
  using SC = Scal<S>;
  constexpr int NL = S::NL, P = S::P, NT = SC::NT, NPT = S::NPT;
  static_assert(NT * SC::TSZ <= 2 * 2 * kStgArr, "a wave's reduction tiles must fit in its staging area");
  __shared__ __align__(16) TrainSmem<S, DTP_XGMI_SPLIT && (MODE == DTP_MODE_XGMI_ADAM || MODE == DTP_MODE_XGMI_SGD)> sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int model = blockIdx.x;
  constexpr bool kUpdate = MODE != DTP_MODE_GRAD;
  constexpr bool kPipe = DTP_PIPE && S::NL >= 3;
  constexpr bool kAdam = MODE == DTP_MODE_ADAM || MODE == DTP_MODE_XGMI_ADAM;
  constexpr bool kXgmi = MODE == DTP_MODE_XGMI_ADAM || MODE == DTP_MODE_XGMI_SGD;
  unsigned long long* prof = reinterpret_cast<unsigned long long*>(a.status);
  // PROF: kernel entry and exit stamps of the launch (slots 20 and 21 of iteration 0)
  auto stamp_launch = [&](int slot) {
    if constexpr (PROF) {
      if (tid == 0) {
        unsigned long long t_;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        prof[(size_t)blockIdx.x * 8 * 32 + slot] = t_;
      }
    }
  };
  stamp_launch(20);
  const bool ce = !FAST && a.loss == DTP_LOSS_CE;  // FAST: MSE
  const int ydim = ce ? 1 : S::OUT;
  const float slope = a.hp.slope;

  // ---- setup. Every global read of the prologue (owned params and moments, step
  // and exchange counters, the dataset) is issued before the first wait, so a
  // launch pays ONE memory round trip before its first step, not three.
  float* __restrict__ gp = a.params + (size_t)model * P;
  const SamplerCfg smp = a.smp;
  const bool cached = FAST || (a.cache_data && smp.n * (S::IN + ydim) <= kDataCache);
  int pf[NPT], pb[NPT], tp[NPT], pfl[NPT];
  float pw[NPT], mr[NPT], vr[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int p = NPT * tid + k;  // blocked ownership: thread t holds parameters NPT t .. NPT t + NPT-1
    scal_pos<S>(p < P ? p : 0, pf[k], pb[k], tp[k], pfl[k]);
    const bool own = p < P;
    pw[k] = own ? gp[p] : 0.f;
    mr[k] = (kUpdate && own) ? a.opt_m[(size_t)model * P + p] : 0.f;
    vr[k] = (kAdam && own) ? a.opt_v[(size_t)model * P + p] : 0.f;
  }
  // the step number: from the host when it knows it (the persistent engine), so the
  // first dataset indices can be requested without waiting for the counter's load
  const int t0 = a.host_t0 >= 0 ? a.host_t0 : a.step[model];
  // the host's Adam-scalar table (persistent engine): the first kAdamTab entries are
  // loaded with the prologue's other global reads (one memory round trip for all)
  const bool htab = kAdam && a.adam_tab && a.host_t0 >= 0;
  float2 tabv[kAdamTab / kBlock];
  if (htab) adam_tab_load<kAdamTab / kBlock>(a, t0, 0, tid, tabv);
  // 32-bit step bookkeeping, advanced incrementally (no 64-bit divisions per step)
  const bool explicit_idx = !FAST && smp.mode == SAMPLER_EXPLICIT;
  int epoch = explicit_idx ? 0 : t0 / smp.steps_per_epoch;
  int bi = explicit_idx ? 0 : t0 - epoch * smp.steps_per_epoch;
  // FAST: this lane's dataset index of the step at (ep_, b_): the padded-list position
  // (padding repeats from the start), looked up in the epoch's slot of the ring; -1
  // past the batch.  The load is issued a step ahead of its use (fidx below).
  auto fast_index = [&](int ep_, int b_) -> int {
    const int start = b_ * smp.batch;
    const int size = min(smp.batch, smp.num_samples - start);
    int q = smp.rank + (start + tid) * smp.world;
    q = q >= smp.n ? q - smp.n : q;
    q = q < smp.n ? q : smp.n - 1;  // lanes past the batch: any in-range position
    const int di = table_epoch(smp, ep_)[q];
    return tid < size ? di : -1;
  };
  auto roll = [&](int& ep_, int& b_) {  // advance a (epoch, batch) cursor by one step, branch-free
    const bool r_ = ++b_ == smp.steps_per_epoch;
    b_ = r_ ? 0 : b_;
    ep_ += r_ ? 1 : 0;
  };
  // FAST: the first step's indices and the second step's (in flight across the
  // prologue), and the cursor of the step after the next one to gather
  int e2 = epoch, b2 = bi, fidx0 = 0, fidx = 0;
  if constexpr (FAST) {
    fidx0 = fast_index(epoch, bi);
    roll(e2, b2);
    fidx = fast_index(e2, b2);
  }
  unsigned xepoch = kXgmi ? a.epoch[model] : 0u;
  // the exchanges' sticky timeout flag, read once per launch with the prologue loads
  bool xdead = (kXgmi && a.status) ? (__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
                                   : false;
  unsigned long long xwait[2] = {0ull, 0ull};  // exchange-wait / publish ticks of this thread (xgmi_record_wait)
  for (int e = tid; e < SC::LW; e += kBlock) sm.wb[e] = 0.f;
  if (cached) {
    for (int e = tid; e < smp.n * S::IN; e += kBlock) sm.data[e] = a.X[e];
    for (int e = tid; e < smp.n * ydim; e += kBlock) sm.data[smp.n * S::IN + e] = a.Y[e];
  }
  stamp_launch(18);
  const float* __restrict__ Xg = a.X;
  const float* __restrict__ Yg = a.Y;
  const int yoff = smp.n * S::IN;
  __syncthreads();  // weight blocks zeroed (pads stay 0) before the owners scatter into them
  stamp_launch(19);
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    if (NPT * tid + k < P) {
      const float wv = S::rnd(pw[k]);  // bf16 compute: the matmul operand is the bf16 weight
      sm.wb[pfl[k]] = wv;
      if (pb[k] >= 0) sm.wb[pb[k]] = wv;
    }
  }
  stamp_launch(22);
  int lslot = a.loss_log ? t0 % a.loss_log_cap : 0;
  uint32_t keys[4];
  epoch_keys(smp, epoch, keys);
  // sample k of step it (batch geometry bp): index (explicit list or the in-kernel
  // Feistel shuffle, sampler.h) -> input and target from the LDS-resident dataset.
  // The next step's first chunk is gathered while the current step's optimizer
  // runs (the sampler depends on nothing the update writes), so a step starts
  // with its inputs already in registers.
  auto gather = [&](int it_, const BatchPos& bp_, const uint32_t (&keys_)[4], int k, int bsz_) {
    SampleRegs<S> r;
    r.valid = k < bsz_;
    int di = 0;
    if (r.valid) di = explicit_idx ? a.idx[(size_t)it_ * smp.batch + k] : sample_index(smp, bp_, keys_, k);
    static_for<0, S::IN>([&](auto IC) {
      constexpr int i = decltype(IC)::value;
      r.x[i] = r.valid ? S::rnd(cached ? sm.data[di * S::IN + i] : Xg[(size_t)di * S::IN + i]) : 0.f;
    });
    static_for<0, S::OUT>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      float y = 0.f;
      if (r.valid && j < ydim) y = cached ? sm.data[yoff + di * ydim + j] : Yg[(size_t)di * ydim + j];
      r.y[j] = y;
    });
    return r;
  };
  auto batch_at = [&](int ep, int b) {
    BatchPos bp_;
    bp_.epoch = ep;
    bp_.start = b * smp.batch;
    bp_.size = explicit_idx ? smp.batch : min(smp.batch, smp.num_samples - bp_.start);
    return bp_;
  };
  auto fast_gather = [&](int di) {
    SampleRegs<S> r;
    r.valid = di >= 0;
    di = (unsigned)di < (unsigned)smp.n ? di : 0;  // never index LDS out of range
    static_for<0, S::IN>([&](auto IC) {
      constexpr int i = decltype(IC)::value;
      const float v = S::rnd(sm.data[di * S::IN + i]);
      r.x[i] = r.valid ? v : 0.f;
    });
    static_for<0, S::OUT>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      const float v = j < ydim ? sm.data[yoff + di * ydim + j] : 0.f;
      r.y[j] = r.valid ? v : 0.f;
    });
    return r;
  };
  SampleRegs<S> nxt;
  if constexpr (FAST) {
    nxt = fast_gather(fidx0);  // the first step's samples (the index loads overlapped the prologue)
  } else {
    nxt = gather(0, batch_at(epoch, bi), keys, tid, batch_at(epoch, bi).size);
  }
  // Adam bias-correction powers beta^t, carried in double like torch's host math
  // table entry e holds the scalars of step number t0 + base + e + 1
  auto fill_adam = [&](int base) {
    const int n = min(kAdamTab, a.n_steps - base);  // short launches (eager / graph) fill only what they use
    if (htab) {
      float2 v[kAdamTab / kBlock];
      if (base) adam_tab_load<kAdamTab / kBlock>(a, t0, base, tid, v);
      adam_tab_store<kAdamTab / kBlock>(sm.adam_tab, n, tid, base ? v : tabv);
      return;
    }
    for (int e = tid; e < n; e += kBlock) {
      const uint64_t t1 = (uint64_t)t0 + (uint64_t)base + (uint64_t)e + 1u;
      const double bc1 = 1.0 - pow_int(a.hp.beta1, t1), bc2 = 1.0 - pow_int(a.hp.beta2, t1);
      sm.adam_tab[e] = make_float2((float)(a.hp.lr / bc1), (float)sqrt(bc2));
    }
  };
  if (kAdam) fill_adam(0);
  stamp_launch(23);
  float* const stg_pack = &sm.stage[wave][0][0];
  __syncthreads();  // scattered weight blocks and the Adam table visible to every wave
  stamp_launch(29);

  for (int it = 0; it < a.n_steps; ++it) {
    DTP_STAMP(0);
    const int t = t0 + it;
    const BatchPos bp = batch_at(epoch, bi);
    const int bsz = bp.size;
    const float inv = ce ? 1.f / (float)bsz : 1.f / (float)(bsz * S::OUT);

    f32x4 acc[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    float lacc = 0.f;  // this lane's loss over the step's chunks (bf16 instances)

    // FAST: batch <= kBlock, one chunk (the loop folds away: fwd, loss and bwd are
    // one straight-line region)
    for (int c0 = 0; c0 < (FAST ? kBlock : bsz); c0 += kBlock) {
      const SampleRegs<S> smpl = c0 == 0 ? nxt : gather(it, bp, keys, c0 + tid, bsz);
      const bool valid = smpl.valid;
      float h[NL + 1][16];
      static_for<0, S::IN>([&](auto IC) { h[0][decltype(IC)::value] = smpl.x[decltype(IC)::value]; });
      BBlk<S, NL - 1> pbt;  // backward blocks prefetched by the pipelined forward
      TopB2<S> pbt2;
      if constexpr (kPipe) {
        FBlk<S, 0> pb0;
        pb0.template load<0, FBlk<S, 0>::NR>(sm.wb);
        if (c0 == 0) DTP_STAMP(1);
        pipe_forward<S, 0, FAST>(sm.wb, pb0, h, slope, pbt, pbt2);
      } else {
        if (c0 == 0) DTP_STAMP(1);
        lds_forward<S>(sm.wb, h, slope);
      }

      // ---------------- loss (MSE / CE) -> dz of the last layer
      constexpr int L = NL - 1;
      float dz[16];
      float lpart = 0.f;
      if (!ce) {
        static_for<0, S::OUT>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          const float d = h[L + 1][j] - smpl.y[j];
          lpart = valid ? fmaf(d, d, lpart) : lpart;
          dz[j] = valid ? S::rnd(2.f * d * inv) : 0.f;
        });
      } else {
        const int cls = valid ? (int)smpl.y[0] : 0;
        float mx = h[L + 1][0];
        static_for<1, S::OUT>([&](auto JC) { mx = fmaxf(mx, h[L + 1][decltype(JC)::value]); });
        float se = 0.f, zc = 0.f;
        static_for<0, S::OUT>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          se += __expf(h[L + 1][j] - mx);
          zc = (j == cls) ? h[L + 1][j] : zc;
        });
        const float lse = mx + __logf(se);
        const float rs = 1.f / se;
        lpart = valid ? lse - zc : 0.f;
        static_for<0, S::OUT>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          dz[j] = valid ? S::rnd((__expf(h[L + 1][j] - mx) * rs - (j == cls ? 1.f : 0.f)) * inv) : 0.f;
        });
      }
      if (c0 == 0) DTP_STAMP(2);
      lacc += lpart;

      // ---------------- backward: dX chain (VALU, LDS weight blocks) + dW tiles (MFMA, K = samples)
      if constexpr (kPipe) {
        const PipeBwdCtx<S> pc{sm.wb, stg_pack, &sm.stage[wave][1][0], lane, slope, lpart};
        pipe_backward<S>(pc, pbt, pbt2, h, dz, acc);
      } else {
      static_for<0, NL>([&](auto RC) {
        constexpr int l = NL - 1 - decltype(RC)::value;
        constexpr int I = S::din(l), O = S::dout(l);
        constexpr bool packed = SC::PACK && (l == 0 || l == NL - 1);
        float* stg = packed ? stg_pack : &sm.stage[wave][1][0];
        float* dzb = stg;
        float* hb = stg + kStgArr;
        stage_cols<O>(dzb, lane, SC::rowoff(l), dz);
        if constexpr (l == NL - 1) stage_one(dzb, lane, SC::lossrow(), lpart);
        stage_cols<I>(hb, lane, SC::coloff(l), h[l]);
        stage_one(hb, lane, SC::coloff(l) + I, 1.f);
        if constexpr (l == 2) if (c0 == 0) DTP_STAMP(16);
        if constexpr (!packed) {
          // this layer's 16 MFMA K-steps ride between the dX rows (mlp_scalar.h)
          __builtin_amdgcn_wave_barrier();
          const TileOps to = tile_ops(dzb, hb, lane);
          if constexpr (l == 2 && PROF) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(to.a[0].x), "v"(to.b[3].w));
            if (c0 == 0) DTP_STAMP(17);
          }
          f32x4 a1 = f32x4{0.f, 0.f, 0.f, 0.f};
          f32x4& a0 = acc[SC::tile(l)];
          lds_backward_dx<S, l, 16>(sm.wb, h, dz, slope,
                                    [&](auto KC) { tile_kstep<decltype(KC)::value>(to, a0, a1); });
          a0 += a1;
          __builtin_amdgcn_wave_barrier();
        } else if constexpr (l > 0) {
          lds_backward_dx<S, l, 0>(sm.wb, h, dz, slope, [](auto) {});
        }
        if (c0 == 0) DTP_STAMP(24 + l);
      });
      if constexpr (SC::PACK) {
        __builtin_amdgcn_wave_barrier();
        acc[0] = wave_outer_acc(stg_pack, stg_pack + kStgArr, acc[0], lane);
        __builtin_amdgcn_wave_barrier();
      }
      }
    }
    if constexpr (S::BF) {
      const float wl = wave_sum(lacc);
      if (lane == 0) sm.lossw[wave] = wl;
    }
    DTP_STAMP(8 + wave);
    DTP_STAMP(3);
    // each wave parks its partial dW tiles in its OWN staging area (no other wave
    // touches it, and this wave's staging reads were issued before these writes),
    // so one barrier publishes them
    {
      const int q = lane >> 4, col = lane & 15;
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
        *reinterpret_cast<f32x4*>(&sm.stage[wave][0][0] + tt * SC::TSZ + SC::tslot(4 * q, col)) = acc[tt];
    }
    __syncthreads();
    // this step's Adam scalars: requested now, consumed after the reduction
    float2 adam_sc = make_float2(0.f, 1.f);
    if constexpr (kAdam) adam_sc = sm.adam_tab[it % kAdamTab];
    DTP_STAMP(4);

    float g[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < kWaves; ++ww) s += sm.stage[ww][0][tp[k]];
      g[k] = s;
    }
    float lsum = 0.f;
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww)
      lsum += S::BF ? sm.lossw[ww] : sm.stage[ww][0][SC::losspos()];
    const float mean_loss = lsum * inv;
    DTP_STAMP(5);

    float gloss = mean_loss;
    if constexpr (kXgmi) {
      // all-reduce (sum) this model's gradient + loss over every rank through
      // the peers' xGMI-mapped receive buffers, inside the step (xgmi_core.h)
      xepoch += 1u;
#if DTP_XGMI_SPLIT
      const XgmiCtx xc{a.peers, a.status, a.smp.world, a.smp.rank, a.n_models, a.timeout_us};
      gloss = xgmi_allreduce_split<P, NPT, kBlock>(xc, model, g, mean_loss, xepoch, tid, sm.xg,
                                                   sm.xg + xgmi_slot16(P, NPT), xdead, DTP_XWAIT ? xwait : nullptr);
#else
      gloss = xgmi_allreduce_model<NPT, kBlock>(a, model, P, g, mean_loss, xepoch, tid, DTP_XWAIT ? xwait : nullptr,
                                                1, 0, &xdead);
#endif
    }

    // advance the sampler / loss-ring position and gather the next step's first
    // chunk now: its index hashing and LDS reads overlap the optimizer's latency
    // (FAST: the gather is straight-line code in the optimizer's basic block; the
    // loss-log store, a branch of thread 0, comes after the update)
    const int lslot_now = lslot;
    if constexpr (FAST) {
      roll(epoch, bi);
    } else if (!explicit_idx && ++bi == smp.steps_per_epoch) {
      bi = 0;
      ++epoch;
      epoch_keys(smp, epoch, keys);
    }
    if (a.loss_log && ++lslot == a.loss_log_cap) lslot = 0;
    if constexpr (FAST) {
      // the next step's samples from the index loaded a step ago, then the load for the
      // step after it (past the last step: an in-range table read, never used)
      nxt = fast_gather(fidx);
      roll(e2, b2);
      fidx = fast_index(e2, b2);
    } else if (it + 1 < a.n_steps) {
      const BatchPos bpn = batch_at(epoch, bi);
      nxt = gather(it + 1, bpn, keys, tid, bpn.size);
    }

    if constexpr (MODE == DTP_MODE_GRAD) {
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int p = NPT * tid + k;
        if (p < P) a.grad_out[(size_t)model * P + p] = g[k] * a.hp.grad_scale;
      }
      if (tid == 0) a.grad_out[(size_t)a.n_models * P + model] = mean_loss;
    } else {
      AdamScalars as = adam_consts(a.hp);
      as.step_size = adam_sc.x;
      as.bc2_sqrt = adam_sc.y;
      const float lr = (float)a.hp.lr, mom = (float)a.hp.momentum, wd = (float)a.hp.weight_decay;
      // branch-free over the thread's NPT slots (slots past P hold zeros and store
      // into sm.sink), so the compiler can interleave the slots' dependency chains
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        if constexpr (kAdam) adam_update(pw[k], mr[k], vr[k], g[k] * a.hp.grad_scale, as);
        else sgd_update(pw[k], mr[k], g[k] * a.hp.grad_scale, lr, mom, wd, t == 0);
      }
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const bool own = NPT * tid + k < P;
        const float wv = S::rnd(pw[k]);
        *(own ? &sm.wb[pfl[k]] : &sm.sink[0]) = wv;
        *(own && pb[k] >= 0 ? &sm.wb[pb[k]] : &sm.sink[1]) = wv;
      }
    }
    // the thread that holds the global loss logs it (xgmi_core.h: the loss granule's owner)
    if (tid == (kXgmi ? xgmi_loss_tid<NPT>(P, kBlock) : 0) && a.loss_log) {
      const float lg = kXgmi ? gloss * a.hp.grad_scale : mean_loss;
      a.loss_log[(size_t)lslot_now * a.n_models + model] = lg;
    }
    DTP_STAMP(6);
    __syncthreads();  // updated weights visible; reduction tiles consumed
    // the next kAdamTab steps' Adam scalars, once every kAdamTab steps at a step
    // boundary (every wave read this step's entry before the barrier above)
    if (kAdam && (it + 1) % kAdamTab == 0 && it + 1 < a.n_steps) {
      fill_adam(it + 1);
      __syncthreads();
    }
    DTP_STAMP(7);
  }

  if constexpr (kUpdate) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int p = NPT * tid + k;
      if (p < P) {
        gp[p] = pw[k];
        a.opt_m[(size_t)model * P + p] = mr[k];
        if (kAdam) a.opt_v[(size_t)model * P + p] = vr[k];
      }
    }
    if (tid == 0) a.step[model] = t0 + a.n_steps;
    if (kXgmi && tid == 0) a.epoch[model] = xepoch;
    if (DTP_XWAIT && kXgmi && model == 0 && a.status) xgmi_record_wait(a.status, xwait, (unsigned long long)a.n_steps, tid);
    stamp_launch(21);
  }
}

// ------------------------------------------------------------------------------
// Several lanes per sample (mlp_lanes.h): the step for per-rank batches <= 256 / L.
// floats of dataset staged in LDS by the lanes kernel (strong scaling: n = 512 x 3)
constexpr int kLaneData = 4096;

// staging areas of one wave: the packed first/last tile (or the last layer's and the first
// layer's when they do not pack) and ONE area shared by the hidden layers -- a wave's LDS
// operations execute in order, so layer l-1's staging writes land after layer l's MFMA
// operand reads were issued (the constant-1 bias column, written once, is the same
// column in every hidden tile)
template <class S>
DTP_HD constexpr int lane_areas() { return Scal<S>::PACK ? 2 : 3; }
template <class S>
DTP_HD constexpr int lane_area(int l) {
  return (Scal<S>::PACK && (l == 0 || l == S::NL - 1)) ? 0 : (l == S::NL - 1 ? 0 : (l == 0 ? 2 : 1));
}

#ifndef DTP_LANE_OWN
// 1: the several-lanes kernels' parameter ownership follows the forward blocks' LDS order
// (lane_own_param) instead of torch order: consecutive lanes then write consecutive LDS
// words in the post-Adam weight scatter and read consecutive tile slots in the cross-wave
// gradient sums (torch order puts 5-8 lanes of a 32-lane group on one bank in both).
// Measured SLOWER at batch 256 (split-batch step, K = 2000, 4 interleaved runs each:
// 3.351-3.362 vs 3.320-3.331 us/step, profiles/r6_misc/r6j/): off
#define DTP_LANE_OWN 0
#endif

// the torch-order parameter of ownership slot s (< P): the forward blocks' LDS order -- a
// partitioned layer's block is rows r (inputs, then the bias row) of outputs j, the whole
// last layer's rows j of inputs i (then its bias)
template <class S>
DTP_DEV int lane_own_param(int s) {
  int p = s;
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l), base = S::gw(l), n = O * (I + 1);
    if (s >= base && s < base + n) {
      const int q = s - base;
      int j, r;
      if constexpr (l < S::NL - 1) {
        r = q / O;
        j = q - r * O;
      } else {
        j = q / (I + 1);
        r = q - j * (I + 1);
      }
      p = r < I ? base + j * I + r : S::gb(l) + j;
    }
  });
  return p;
}

template <class S, int L, int NW, bool GRP = false>
struct LaneSmem {
  using C = LaneCfg<S, L>;
  alignas(16) float wb[C::pad4(C::LW)];
  alignas(16) float stg[NW][lane_areas<S>()][2 * C::AREA];  // per wave, per area: dz operand, h operand
  alignas(16) float red[NW][Scal<S>::NT * Scal<S>::TSZ];             // per-wave partial dW tiles
  alignas(16) float2 adam_tab[kAdamTab];
  alignas(16) float data[kLaneData];
  float sink[4];
  // split-batch exchange (grp_allreduce_split): this member's payloads, then every member's
  static constexpr int GSLOT = xgmi_slot16(S::P, (S::P + 64 * NW - 1) / (64 * NW));
  // (the 3-float form, DTP_GRP_G3: (kGrpMax + 1) rows of grp_ps3(P) floats)
  // (the 3-float xGMI form, DTP_XGMI_G3: xgmi_g3_lds_floats(P) floats)
  static constexpr int GX2a = (kGrpMax + 1) * GSLOT > (kGrpMax + 1) * grp_ps3(S::P) / 2
                                  ? (kGrpMax + 1) * GSLOT : (kGrpMax + 1) * grp_ps3(S::P) / 2;
  static constexpr int GX2 = GX2a > xgmi_g3_lds_floats(S::P) / 2 ? GX2a : xgmi_g3_lds_floats(S::P) / 2;
  alignas(16) float2 gx[GRP ? GX2 : 2];
};

// NW waves per workgroup (4: one per SIMD; 8: two per SIMD, for batches of 256 / L < B <= 512 / L)
// GRP: the batch split over a.groups workgroups per model (grp_core.h): member k of model m
// is block m + 8 k (the members of a model share an XCD under round-robin dispatch), runs
// the step on batch positions [k 64 NW / L, (k + 1) 64 NW / L), and the members' partial
// weight gradients and losses are summed on chip before every member's (identical)
// optimizer step.
// CE: softmax cross-entropy head (class ids as floats in Y) instead of MSE; MODE: Adam or
// SGD (momentum, weight decay), local or with the in-kernel xGMI exchange.
template <class S, int L, int MODE, bool PROF = false, int NW = 4, bool GRP = false, bool CE = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4, NW / 4)))
void mlp_train_lanes_kernel(DtpTrainArgs a) {
  using SC = Scal<S>;
  using C = LaneCfg<S, L>;
  constexpr int NTH = 64 * NW;                 // threads of the workgroup
  constexpr int NPT = (S::P + NTH - 1) / NTH;  // parameters owned per thread (optimizer, exchange)
  constexpr int NL = S::NL, P = S::P, NT = SC::NT, NO = C::NO, TS = C::TS, H = S::H;
  constexpr bool kXgmi = MODE == DTP_MODE_XGMI_ADAM || MODE == DTP_MODE_XGMI_SGD;
  constexpr bool kAdam = MODE == DTP_MODE_ADAM || MODE == DTP_MODE_XGMI_ADAM;
  static_assert(MODE != DTP_MODE_GRAD, "the lanes step serves the optimizer modes");
  // GRP with kXgmi: ONE flat exchange over world x groups members (xgmi_core.h)
  static_assert(!CE || S::OUT >= 2, "cross-entropy needs >= 2 classes");
  constexpr int YD = CE ? 1 : S::OUT;  // target floats per sample (a class id for CE)
  // the split exchanges' LDS: the split-batch step, and the xGMI instances of 4 waves (the
  // 8-wave ones keep the single-role exchange: their LDS is full)
  constexpr bool kXsplit = DTP_XGMI_SPLIT && NW == 4 && (MODE == DTP_MODE_XGMI_ADAM || MODE == DTP_MODE_XGMI_SGD);
  // the 3-float cross-GPU exchange (xgmi_core.h:xgmi_allreduce_g3), 4-wave instances
  constexpr bool kXg3 = DTP_XGMI_G3 && !kXsplit && NW == 4 && kXgmi;
  __shared__ __align__(16) LaneSmem<S, L, NW, GRP || kXsplit || kXg3> sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int model = GRP ? (int)(blockIdx.x & 7u) : (int)blockIdx.x;
  const int gk = GRP ? (int)(blockIdx.x >> 3) : 0;  // member of the model's group
  if (GRP && (model >= a.n_models || gk >= a.groups)) return;  // grid = 8 x groups blocks
  const bool lead = gk == 0;                // the member that writes the state back
  const int part = lane & (L - 1);          // this lane's slice of every hidden layer
  const int ws = lane / L;                  // sample slot inside the wave
  const int bk = gk * (NW * C::G) + wave * C::G + ws;  // batch position of this lane's sample
  const GrpCtx gctx{a.grp_buf, a.grp_status, a.groups, gk, a.n_models, a.timeout_us};
  if constexpr (PROF) {  // placement of this block: XCC id (slot 12) and HW_ID (13) of step 0's row
    if (tid == 0) {
      unsigned xcc, hwid;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
      unsigned long long* pr = reinterpret_cast<unsigned long long*>(a.status) + (size_t)blockIdx.x * 8 * 32;
      pr[12] = xcc;
      pr[13] = hwid;
    }
  }
  unsigned long long* prof = reinterpret_cast<unsigned long long*>(a.status);
  const float slope = a.hp.slope;
  // PROF: launch-level stamps in row 0 of this block (thread 0): 20 entry, 18 prologue LDS
  // fills issued, 19 first barrier (global loads consumed), 22 weight scatter, 23 Adam table,
  // 29 loop start, 24 loop end, 21 write-back issued (the lead)
  auto stamp_launch = [&](int slot) {
    if constexpr (PROF) {
      if (tid == 0) {
        unsigned long long t_;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        prof[(size_t)blockIdx.x * 8 * 32 + slot] = t_;
      }
    }
  };
  stamp_launch(20);

  // ---- prologue (all global reads issued before the first wait, as in mlp_train_kernel)
  float* __restrict__ gp = a.params + (size_t)model * P;
  const SamplerCfg smp = a.smp;
  int pf[NPT], pb[NPT], tp[NPT], pown[NPT];
  float pw[NPT], mr[NPT], vr[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int s_ = NPT * tid + k;  // ownership slot (the exchanges' payload index)
    const bool own = s_ < P;
    const int p = DTP_LANE_OWN ? (own ? lane_own_param<S>(s_) : 0) : s_;
    pown[k] = p;
    lane_pos<C, S>(own ? p : 0, pf[k], pb[k], tp[k]);
    pw[k] = own ? gp[p] : 0.f;
    mr[k] = own ? a.opt_m[(size_t)model * P + p] : 0.f;
    vr[k] = (kAdam && own) ? a.opt_v[(size_t)model * P + p] : 0.f;
  }
  // split-batch publisher (wave 0, DTP_GRP_DIRECT): the dW-tile positions of the parameters of
  // its granules q = tid + 64 j (granule q holds parameters NPT (q / GPT) + 2 (q % GPT), + 1;
  // the last granule is the loss), so it sums them straight from the tiles
  constexpr int kGpt = xgmi_gpt<NPT>(), kNg = xgmi_nthr(P, NPT) * kGpt + 1, kPubJ = (kNg + kWave - 1) / kWave;
  int gtp[GRP && DTP_GRP_DIRECT ? kPubJ : 1][2];
  if constexpr (GRP && DTP_GRP_DIRECT) {
#pragma unroll
    for (int j = 0; j < kPubJ; ++j) {
      const int q = tid + j * kWave;
      const int p0 = (q / kGpt) * NPT + 2 * (q % kGpt);
      const bool two = 2 * (q % kGpt) + 1 < NPT;
      int pf_, pb_;
      lane_pos<C, S>(p0 < P ? p0 : 0, pf_, pb_, gtp[j][0]);
      lane_pos<C, S>((two && p0 + 1 < P) ? p0 + 1 : 0, pf_, pb_, gtp[j][1]);
    }
  }
  // split-batch direct publish (DTP_GRP_DIRECT3): the dW-tile positions of the payload floats
  // 3 tid .. 3 tid + 2 of granule tid (a parameter's tile slot, the loss slot, or -1: the XCC
  // id / padding)
  int gt3[GRP && DTP_GRP_DIRECT3 ? 3 : 1];
  if constexpr (GRP && DTP_GRP_DIRECT3) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int f = 3 * tid + i;
      int pf_, pb_, t_;
      lane_pos<C, S>(f < P ? f : 0, pf_, pb_, t_);
      gt3[i] = f < P ? t_ : (f == P ? SC::losspos() : -1);
    }
  }
  const int t0 = a.host_t0 >= 0 ? a.host_t0 : a.step[model];
  const bool htab = kAdam && a.adam_tab && a.host_t0 >= 0;
  float2 tabv[kAdamTab / NTH];
  if (htab) adam_tab_load<kAdamTab / NTH, NTH>(a, t0, 0, tid, tabv);
  int epoch = t0 / smp.steps_per_epoch;
  int bi = t0 - epoch * smp.steps_per_epoch;
  auto fast_index = [&](int ep_, int b_) -> int {
    const int start = b_ * smp.batch;
    const int size = min(smp.batch, smp.num_samples - start);
    int q = smp.rank + (start + bk) * smp.world;
    q = q >= smp.n ? q - smp.n : q;
    q = q < smp.n ? q : smp.n - 1;
    const int di = table_epoch(smp, ep_)[q];
    return bk < size ? di : -1;
  };
  auto roll = [&](int& ep_, int& b_) {
    const bool r_ = ++b_ == smp.steps_per_epoch;
    b_ = r_ ? 0 : b_;
    ep_ += r_ ? 1 : 0;
  };
  int e2 = epoch, b2 = bi;
  const int fidx0 = fast_index(epoch, bi);
  roll(e2, b2);
  int fidx = fast_index(e2, b2);
  unsigned xepoch = kXgmi ? a.epoch[model] : (GRP ? a.grp_epoch[model] : 0u);  // GRP + xGMI: the xGMI epochs
  // the exchanges' sticky timeout flag, read once per launch with the prologue loads
  const int* xst = kXgmi ? a.status : (GRP ? a.grp_status : nullptr);
  bool xdead = xst ? (__hip_atomic_load(xst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) : false;
  const unsigned xcc = GRP ? grp_xcc_id() : 0u;  // split-batch exchange: plain stores once every member shares it
  bool gplain = false;
  unsigned long long xwait[2] = {0ull, 0ull};
  for (int e = tid; e < C::pad4(C::LW); e += NTH) sm.wb[e] = 0.f;
  // the dataset (inputs then targets) straight into LDS (LDS-DMA; the first barrier waits)
  lds_dma_fill2<NTH>(sm.data, a.X, smp.n * S::IN, a.Y, smp.n * YD, tid);
  const int yoff = smp.n * S::IN;
  stamp_launch(18);
  // this wave's staging areas: zero (unwritten rows / columns stay finite), then the
  // constant-1 bias columns of every tile, written once per launch
  {
    float* s0 = &sm.stg[wave][0][0];
    for (int e = lane; e < lane_areas<S>() * 2 * C::AREA; e += kWave) s0[e] = 0.f;
    static_for<0, NL>([&](auto LC) {
      constexpr int l = decltype(LC)::value;
      constexpr int col = SC::coloff(l) + S::din(l);
      float* hb = &sm.stg[wave][lane_area<S>(l)][C::AREA];
      for (int e = lane; e < 4 * TS; e += kWave) hb[(e / TS) * C::QS + col * TS + e % TS] = 1.f;
    });
  }
  __syncthreads();  // weight blocks zeroed (pads stay 0) before the owners scatter into them
  stamp_launch(19);
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    if (NPT * tid + k < P) {
      const float wv = S::rnd(pw[k]);  // bf16 compute: the matmul operand is the bf16 weight
      sm.wb[pf[k]] = wv;
      if (pb[k] >= 0) sm.wb[pb[k]] = wv;
    }
  }
  stamp_launch(22);
  int lslot = a.loss_log ? t0 % a.loss_log_cap : 0;
  auto fast_gather = [&](int di, float (&x)[S::IN], float (&y)[S::OUT]) {
    const bool v = di >= 0;
    di = (unsigned)di < (unsigned)smp.n ? di : 0;
    static_for<0, S::IN>([&](auto IC) {
      constexpr int i = decltype(IC)::value;
      const float t_ = S::rnd(sm.data[di * S::IN + i]);
      x[i] = v ? t_ : 0.f;
    });
    static_for<0, S::OUT>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      const float t_ = j < YD ? sm.data[yoff + di * YD + j] : 0.f;
      y[j] = v ? t_ : 0.f;
    });
    return v;
  };
  float nx[S::IN], ny[S::OUT];
  bool nvalid = fast_gather(fidx0, nx, ny);
  auto fill_adam = [&](int base) {
    const int n = min(kAdamTab, a.n_steps - base);
    if (htab) {
      float2 v[kAdamTab / NTH];
      if (base) adam_tab_load<kAdamTab / NTH, NTH>(a, t0, base, tid, v);
      adam_tab_store<kAdamTab / NTH, NTH>(sm.adam_tab, n, tid, base ? v : tabv);
      return;
    }
    for (int e = tid; e < n; e += NTH) {
      const uint64_t t1 = (uint64_t)t0 + (uint64_t)base + (uint64_t)e + 1u;
      const double bc1 = 1.0 - pow_int(a.hp.beta1, t1), bc2 = 1.0 - pow_int(a.hp.beta2, t1);
      sm.adam_tab[e] = make_float2((float)(a.hp.lr / bc1), (float)sqrt(bc2));
    }
  };
  if (kAdam) fill_adam(0);
  stamp_launch(23);
  // per-lane LDS bases: the part's slice of the partitioned blocks, the sample's slot in a
  // staged operand (+ the part's first column), the MFMA reader's operands
  const float* const wlp = sm.wb + part * C::NOP;
  const int wslot = (ws & 3) * C::QS + (ws >> 2);
  const int wpart = wslot + part * NO * TS;
  const int rdoff = (lane >> 4) * C::QS + (lane & 15) * TS;
  // is slot k of this lane's slice a real unit (k*L + part < H)?
  auto slot_ok = [&](int k) { return C::EXACT || part * NO + k < H; };
  // A staging write of a lane with nothing to stage (a padding slot, a part other than 0
  // for the per-sample rows) goes to row / column 15 of its sample slot when no tile uses
  // it -- D[15][*] and D[*][15] are never read -- so the writes are branch-free
  constexpr bool kSink = H <= 14 && SC::lossrow() <= 14 && (!SC::PACK || S::IN + 1 + H <= 14);
  auto put = [&](float* tl, int area, int off, bool ok, float v) {
    if constexpr (kSink) {
      tl[area + (ok ? off : wslot + 15 * TS)] = v;
    } else {
      if (ok) tl[area + off] = v;
    }
  };
  const bool p0 = part == 0;
  __syncthreads();
  stamp_launch(29);

  for (int it = 0; it < a.n_steps; ++it) {
    DTP_STAMP(0);
    const int bsz = min(smp.batch, smp.num_samples - bi * smp.batch);
    const float inv = CE ? 1.f / (float)bsz : 1.f / (float)(bsz * S::OUT);
    f32x4 acc[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool valid = nvalid;
    LaneAct<C> st;
    static_for<0, S::IN>([&](auto IC) { st.hin[decltype(IC)::value] = nx[decltype(IC)::value]; });
    float x0[S::IN];
    static_for<0, S::IN>([&](auto IC) { x0[decltype(IC)::value] = nx[decltype(IC)::value]; });

    // ---------------- forward
    LLast<C> last;
    LBBlk<C, NL - 1> bt;
    LBBlk<C, NL - 2> bt2;
    float out[16];
    {
      LFBlk<C, 0> b0;
      b0.template load<0, LFBlk<C, 0>::NR>(sm.wb, wlp);
      DTP_STAMP(1);
      lane_forward<C, 0>(sm.wb, wlp, b0, st, slope, last, bt, bt2, out);
    }
    // ---------------- loss (MSE) -> output gradient (every lane of the sample)
    float dzl[S::OUT];
    float lpart = 0.f;
    if constexpr (!CE) {
      static_for<0, S::OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        const float d = out[j] - ny[j];
        lpart = valid ? fmaf(d, d, lpart) : lpart;
        dzl[j] = valid ? S::rnd(2.f * d * inv) : 0.f;
      });
    } else {  // the one-lane kernel's CE arithmetic (mlp_train_kernel), per lane
      const int cls = valid ? (int)ny[0] : 0;
      float mx = out[0];
      static_for<1, S::OUT>([&](auto JC) { mx = fmaxf(mx, out[decltype(JC)::value]); });
      float se = 0.f, zc = 0.f, ex[S::OUT];  // each exponential once (the same bits as twice)
      static_for<0, S::OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        ex[j] = __expf(out[j] - mx);
        se += ex[j];
        zc = (j == cls) ? out[j] : zc;
      });
      const float lse = mx + __logf(se);
      const float rs = 1.f / se;
      lpart = valid ? lse - zc : 0.f;
      static_for<0, S::OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        dzl[j] = valid ? S::rnd((ex[j] * rs - (j == cls ? 1.f : 0.f)) * inv) : 0.f;
      });
    }
    DTP_STAMP(2);

    // ---------------- backward
    float dzp[C::NOP];  // this lane's slice of the current layer's output gradient
    {  // last layer: stage (dz, loss, own slice of its input), input-gradient slice
      constexpr int l = NL - 1;
      float* tl = &sm.stg[wave][lane_area<S>(l)][0];
      static_for<0, S::OUT>([&](auto JC) {
        put(tl, 0, wslot + (SC::rowoff(l) + decltype(JC)::value) * TS, p0, dzl[decltype(JC)::value]);
      });
      put(tl, 0, wslot + SC::lossrow() * TS, p0, lpart);
      static_for<0, NO>([&](auto KC) {
        constexpr int k = decltype(KC)::value;
        put(tl, C::AREA, wpart + (SC::coloff(l) + k) * TS, slot_ok(k), st.own[l - 1][k]);
      });
      f32x2 g[C::NPR];
      static_for<0, C::NPR>([&](auto RC) { g[decltype(RC)::value] = f32x2{0.f, 0.f}; });
      static_for<0, S::OUT>([&](auto OC) {
        constexpr int o = decltype(OC)::value;
        const f32x2 d = f32x2{dzl[o], dzl[o]};
        static_for<0, C::NPR>([&](auto RC) {
          constexpr int r = decltype(RC)::value;
          g[r] = __builtin_elementwise_fma(quad_pair<r % 2>(bt.w[o][r / 2]), d, g[r]);
        });
      });
      static_for<0, NO>([&](auto KC) {
        constexpr int k = decltype(KC)::value;
        const float v = S::rnd((k & 1) ? g[k / 2].y : g[k / 2].x);
        dzp[k] = S::rnd(v * leaky_grad_from_out(st.own[l - 1][k], slope));
      });
      if constexpr (!SC::PACK) {
        __builtin_amdgcn_wave_barrier();
        const auto to = lane_tile_ops<C>(tl, rdoff);
        acc[SC::tile(l)] = lane_tile<C, S>(to, acc[SC::tile(l)]);
      }
    }
    // hidden layers NL-2 .. 1: block B of layer l in registers, block l-1 prefetched
    auto hidden = [&](auto LC, const auto& B, auto& nb) {
      constexpr int l = decltype(LC)::value;
      float* tl = &sm.stg[wave][lane_area<S>(l)][0];
      // the previous layer's MFMA operand reads of this area were issued before these writes
      __builtin_amdgcn_sched_barrier(0);
      static_for<0, NO>([&](auto KC) {
        constexpr int k = decltype(KC)::value;
        put(tl, 0, wpart + (SC::rowoff(l) + k) * TS, slot_ok(k), dzp[k]);
        put(tl, C::AREA, wpart + (SC::coloff(l) + k) * TS, slot_ok(k), st.own[l - 1][k]);
      });
      __builtin_amdgcn_wave_barrier();
      const auto to = lane_tile_ops<C>(tl, rdoff);
      float dzf[16];
      static_for<0, C::L>([&](auto PC) {
        constexpr int pp = decltype(PC)::value;
        static_for<0, NO>([&](auto KC) {
          constexpr int k = decltype(KC)::value;
          if constexpr (pp * NO + k < H) dzf[pp * NO + k] = part_bcast<C::L, pp>(dzp[k]);
        });
      });
      f32x2 g[C::NPR];
      static_for<0, C::NPR>([&](auto RC) { g[decltype(RC)::value] = f32x2{0.f, 0.f}; });
      f32x4 a0 = acc[SC::tile(l)], a1 = f32x4{0.f, 0.f, 0.f, 0.f};
      constexpr int J0 = 2;
      LNone none;
      static_for<0, H>([&](auto OC) {
        constexpr int o = decltype(OC)::value;
        if constexpr (S::BF && DTP_LANES_BFMMA) {  // the whole tile on one bf16 MFMA
          if constexpr (o == J0) a0 = lane_tile_bf<C>(to, a0);
        } else if constexpr (o >= J0) {
          constexpr int k0 = TS * (o - J0) / (H - J0), k1 = TS * (o - J0 + 1) / (H - J0);
          static_for<k0, k1>([&](auto KC) { lane_kstep<decltype(KC)::value>(to, a0, a1); });
        }
        const f32x2 d = f32x2{dzf[o], dzf[o]};
        static_for<0, C::NPR>([&](auto RC) {
          constexpr int r = decltype(RC)::value;
          g[r] = __builtin_elementwise_fma(quad_pair<r % 2>(B.w[o][r / 2]), d, g[r]);
        });
        __builtin_amdgcn_sched_barrier(0);
        lchunk<o, H>(sm.wb, wlp, nb, none);
        __builtin_amdgcn_sched_barrier(0);
      });
      acc[SC::tile(l)] = a0 + a1;
      static_for<0, NO>([&](auto KC) {
        constexpr int k = decltype(KC)::value;
        const float v = S::rnd((k & 1) ? g[k / 2].y : g[k / 2].x);
        dzp[k] = S::rnd(v * leaky_grad_from_out(st.own[l - 1][k], slope));
      });
    };
    auto hidden_rest = [&](auto self, auto LC, const auto& B) -> void {
      constexpr int l = decltype(LC)::value;
      if constexpr (l > 1) {
        LBBlk<C, l - 1> nb;
        hidden(LC, B, nb);
        self(self, std::integral_constant<int, l - 1>{}, nb);
      } else {
        LNone none;
        hidden(LC, B, none);
      }
    };
    hidden_rest(hidden_rest, std::integral_constant<int, NL - 2>{}, bt2);
    {  // layer 0: its dW tile only (packed with the last layer's when they fit)
      float* tl = &sm.stg[wave][lane_area<S>(0)][0];
      static_for<0, NO>([&](auto KC) {
        constexpr int k = decltype(KC)::value;
        put(tl, 0, wpart + (SC::rowoff(0) + k) * TS, slot_ok(k), dzp[k]);
      });
      static_for<0, S::IN>([&](auto IC) {
        put(tl, C::AREA, wslot + (SC::coloff(0) + decltype(IC)::value) * TS, p0, x0[decltype(IC)::value]);
      });
      __builtin_amdgcn_wave_barrier();
      const auto to = lane_tile_ops<C>(tl, rdoff);
      acc[SC::tile(0)] = lane_tile<C, S>(to, acc[SC::tile(0)]);
    }
    DTP_STAMP(8 + wave);
    DTP_STAMP(3);
    {
      const int q = lane >> 4, col = lane & 15;
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
        *reinterpret_cast<f32x4*>(&sm.red[wave][tt * SC::TSZ + SC::tslot(4 * q, col)]) = acc[tt];
      if constexpr (S::BF && DTP_LANES_BFMMA) {
        // the bf16 MFMA saw the loss row's per-sample values truncated to bf16: the wave's
        // loss goes in from a wave sum of the fp32 values instead (same LDS slot, written after)
        const float lw = wave_sum(p0 ? lpart : 0.f);
        if (lane == 0) sm.red[wave][SC::losspos()] = lw;
      }
    }
    __syncthreads();
    const float2 adam_sc = kAdam ? sm.adam_tab[it % kAdamTab] : make_float2(0.f, 1.f);
    DTP_STAMP(4);
    float g[NPT];
    float lsum = 0.f;
    // this thread's parameters summed over the waves (and the loss), in wave order
    auto own_sums = [&]() {
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        float s = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) s += sm.red[ww][tp[k]];
        g[k] = s;
      }
      float ls = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) ls += sm.red[ww][SC::losspos()];
      lsum = ls;
    };
    // the split-batch step's direct publish forms these inside the exchange
    constexpr bool kDefer = GRP && !kXgmi && DTP_GRP_SPLIT && DTP_GRP_G3 && DTP_GRP_DIRECT3;
    if constexpr (!kDefer) own_sums();
    // the next step's sample and the index of the one after it (independent of this step's
    // exchange: the split-batch step runs it inside the exchange's waits)
    const int lslot_now = lslot;
    auto next_sample = [&]() {
      roll(epoch, bi);
      if (a.loss_log && ++lslot == a.loss_log_cap) lslot = 0;
      nvalid = fast_gather(fidx, nx, ny);
      roll(e2, b2);
      fidx = fast_index(e2, b2);
    };
    bool sampled = false;
    if constexpr (GRP && !kXgmi) {  // the members' partial sums, on chip (grp_core.h)
      xepoch += 1u;
      GrpProf gp_;
#if DTP_GRP_SPLIT && DTP_GRP_DIRECT
      auto pubval = [&](int j) -> float2 {  // granule tid + 64 j of this member, from the tiles
        float x = 0.f, y = 0.f;
        if (tid + j * kWave == kNg - 1) {
#pragma unroll
          for (int ww = 0; ww < NW; ++ww) x += sm.red[ww][SC::losspos()];
        } else {
#pragma unroll
          for (int ww = 0; ww < NW; ++ww) {
            x += sm.red[ww][gtp[j][0]];
            y += sm.red[ww][gtp[j][1]];
          }
        }
        return make_float2(x, y);
      };
      lsum = grp_allreduce_split<P, NPT, NTH>(gctx, model, g, lsum, xepoch, tid, xdead, sm.gx,
                                              sm.gx + xgmi_slot16(P, NPT), xcc, gplain, PROF ? &gp_ : nullptr,
                                              pubval);
#elif DTP_GRP_SPLIT && DTP_GRP_G3 && DTP_GRP_DIRECT3
      // granule q = tid: payload floats 3q .. 3q + 2 summed over the waves' parked tiles in
      // wave order (own_sums' order: the published values are the bits this member adds)
      auto pub3 = [&](int q, float (&v)[3]) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int pos = gt3[i] >= 0 ? gt3[i] : 0;
          float s_ = 0.f;
#pragma unroll
          for (int ww = 0; ww < NW; ++ww) s_ += sm.red[ww][pos];
          const int f = 3 * q + i;
          v[i] = f == P + 1 ? __uint_as_float(xcc) : (gt3[i] >= 0 ? s_ : 0.f);
        }
      };
      lsum = grp_allreduce_split3d<P, NPT, NTH>(gctx, model, g, lsum, xepoch, tid, xdead,
                                                reinterpret_cast<float*>(sm.gx), xcc, gplain,
                                                PROF ? &gp_ : nullptr, pub3, own_sums);
#elif DTP_GRP_SPLIT && DTP_GRP_G3
      lsum = grp_allreduce_split3<P, NPT, NTH>(gctx, model, g, lsum, xepoch, tid, xdead, reinterpret_cast<float*>(sm.gx),
                                               xcc, gplain, PROF ? &gp_ : nullptr, next_sample);
      sampled = DTP_GRP_OVERLAP;
#elif DTP_GRP_SPLIT
      lsum = grp_allreduce_split<P, NPT, NTH>(gctx, model, g, lsum, xepoch, tid, xdead, sm.gx,
                                              sm.gx + xgmi_slot16(P, NPT), xcc, gplain, PROF ? &gp_ : nullptr);
#else
      lsum = grp_allreduce<NPT, NTH>(gctx, model, P, g, lsum, xepoch, tid, xdead, PROF ? &gp_ : nullptr);
#endif
      if constexpr (PROF) {  // thread 0 (split: thread 64, a poller): publish issued (16), first poll consumed
                             // (17), last granule (31), polls (30)
        if (tid == (DTP_GRP_SPLIT ? 64 : 0) && it < 8) {
          unsigned long long* pr = prof + ((size_t)blockIdx.x * 8 + it) * 32;
          pr[16] = gp_.t_pub;
          pr[17] = gp_.t_first;
          pr[31] = gp_.t_end;
          pr[30] = gp_.polls;
          pr[15] = gp_.rt_end;  // chip-wide clock: this member's last granule
        }
        if (DTP_GRP_SPLIT && tid == 0 && it < 8)  // the publisher: chip-wide clock when its stores were issued
          prof[((size_t)blockIdx.x * 8 + it) * 32 + 14] = gp_.rt_pub;
      }
    }
    const float mean_loss = lsum * inv;  // GRP + xGMI: this member's share of the rank's mean
    DTP_STAMP(5);
    float gloss = mean_loss;
    if constexpr (kXgmi) {
      xepoch += 1u;
      if constexpr (kXg3) {
        const XgmiCtx xc{a.peers, a.status, a.smp.world, a.smp.rank, a.n_models, a.timeout_us};
        gloss = xgmi_allreduce_g3<P, NPT, NTH>(xc, model, g, mean_loss, xepoch, tid, reinterpret_cast<float*>(sm.gx),
                                               xdead, DTP_XWAIT ? xwait : nullptr, GRP ? a.groups : 1, gk);
      } else if constexpr (kXsplit) {
        const XgmiCtx xc{a.peers, a.status, a.smp.world, a.smp.rank, a.n_models, a.timeout_us};
        gloss = xgmi_allreduce_split<P, NPT, NTH>(xc, model, g, mean_loss, xepoch, tid, sm.gx,
                                                  sm.gx + xgmi_slot16(P, NPT), xdead, DTP_XWAIT ? xwait : nullptr,
                                                  GRP ? a.groups : 1, gk);
      } else {
        gloss = xgmi_allreduce_model<NPT, NTH>(a, model, P, g, mean_loss, xepoch, tid, DTP_XWAIT ? xwait : nullptr,
                                               GRP ? a.groups : 1, gk, &xdead);
      }
    }
    if (!sampled) next_sample();
    {
      AdamScalars as = adam_consts(a.hp);
      as.step_size = adam_sc.x;
      as.bc2_sqrt = adam_sc.y;
      const float lr = (float)a.hp.lr, mom = (float)a.hp.momentum, wd = (float)a.hp.weight_decay;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        if constexpr (kAdam) adam_update(pw[k], mr[k], vr[k], g[k] * a.hp.grad_scale, as);
        else sgd_update(pw[k], mr[k], g[k] * a.hp.grad_scale, lr, mom, wd, t0 + it == 0);
      }
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const bool own = NPT * tid + k < P;
        const float wv = S::rnd(pw[k]);
        *(own ? &sm.wb[pf[k]] : &sm.sink[0]) = wv;
        *(own && pb[k] >= 0 ? &sm.wb[pb[k]] : &sm.sink[1]) = wv;
      }
    }
    // the thread that holds the summed loss logs it (the loss granule's owner: every other
    // thread of a split-batch member only has its own member's share)
    if (tid == ((kXgmi || GRP) ? xgmi_loss_tid<NPT>(P, NTH) : 0) && a.loss_log && lead) {
      const float lg = kXgmi ? gloss * a.hp.grad_scale : mean_loss;
      a.loss_log[(size_t)lslot_now * a.n_models + model] = lg;
    }
    DTP_STAMP(6);
    __syncthreads();
    if (kAdam && (it + 1) % kAdamTab == 0 && it + 1 < a.n_steps) {
      fill_adam(it + 1);
      __syncthreads();
    }
    DTP_STAMP(7);
  }

  stamp_launch(24);
  if constexpr (GRP || kXgmi) {
    // a launch whose exchange timed out on any thread keeps the state from before it (what
    // it summed is incomplete; check_comm raises on the status word), so a checkpoint or a
    // resume never sees it -- one barrier per launch
    if (__syncthreads_or(xdead ? 1 : 0)) return;
  }
  if (!lead) return;  // every member holds the same state: the first writes it back
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int p = pown[k];
    if (NPT * tid + k < P) {
      gp[p] = pw[k];
      a.opt_m[(size_t)model * P + p] = mr[k];
      if (kAdam) a.opt_v[(size_t)model * P + p] = vr[k];
    }
  }
  if (tid == 0) a.step[model] = t0 + a.n_steps;
  if (kXgmi && tid == 0) a.epoch[model] = xepoch;
  if (GRP && !kXgmi && tid == 0) a.grp_epoch[model] = xepoch;
  if (DTP_XWAIT && kXgmi && model == 0 && a.status) xgmi_record_wait(a.status, xwait, (unsigned long long)a.n_steps, tid);
  stamp_launch(21);
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

using TrainLaunchFn = void (*)(const DtpTrainArgs&, hipStream_t);

template <class S, int MODE, bool FAST = false>
void launch_mode(const DtpTrainArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((dtp::mlp_train_kernel<S, MODE, false, FAST>), dim3(a.n_models), dim3(dtp::kBlock), 0, st, a);
}

// the kernel instance of (shape S, mode, fast path), resolved once (the native
// engine keeps it); the FAST instances exist for the Adam modes (the training
// configurations of the demos and bench.py)
template <class S>
TrainLaunchFn train_fn(int mode, bool fast) {
  switch (mode) {
    case DTP_MODE_GRAD: return &launch_mode<S, DTP_MODE_GRAD>;
    case DTP_MODE_ADAM: return fast ? &launch_mode<S, DTP_MODE_ADAM, true> : &launch_mode<S, DTP_MODE_ADAM>;
    case DTP_MODE_SGD: return &launch_mode<S, DTP_MODE_SGD>;
    case DTP_MODE_XGMI_ADAM:
      return fast ? &launch_mode<S, DTP_MODE_XGMI_ADAM, true> : &launch_mode<S, DTP_MODE_XGMI_ADAM>;
    case DTP_MODE_XGMI_SGD: return &launch_mode<S, DTP_MODE_XGMI_SGD>;
    default: return nullptr;
  }
}

// the FAST preconditions on the data path (the kernels' compile-time configuration): the
// SAMPLER_TABLE ring, the dataset cached in LDS, 0 <= slope <= 1, batch <= kBlock.  The
// several-lanes and split-batch steps need these, for every loss and optimizer they serve.
bool fast_base_ok(const DtpTrainArgs& a, int in, int out) {
  static const bool disabled = [] {
    const char* e = getenv("DTP_FAST");
    return e && e[0] == '0';
  }();
  if (disabled) return false;
  const dtp::SamplerCfg& s = a.smp;
  const int ydim = a.loss == DTP_LOSS_CE ? 1 : out;
  // n >= world: the FAST gather wraps a padded-list position with ONE subtraction of n
  // (positions stay below n + world - 1), where the generic sampler takes q % n
  const bool ring = s.perm && s.perm_epochs > 0 && (s.perm_epochs & (s.perm_epochs - 1)) == 0;
  return a.cache_data && min(s.batch, s.num_samples) <= dtp::kBlock && s.mode == dtp::SAMPLER_TABLE && ring &&
         s.n >= s.world && s.n * (in + ydim) <= dtp::kDataCache && a.hp.slope >= 0.f && a.hp.slope <= 1.f;
}

// may this launch take the one-lane FAST instance?  (the data-path preconditions, Adam, MSE)
bool fast_path_ok(const DtpTrainArgs& a, int in, int out, int mode) {
  return fast_base_ok(a, in, out) && (mode == DTP_MODE_ADAM || mode == DTP_MODE_XGMI_ADAM) &&
         a.loss == DTP_LOSS_MSE;
}

// shapes with a bf16-compute instance (the toy model: MSE and CE heads)
#define DTP_TRAIN_BF16_SHAPES(X) \
  X(2, 10, 5, 1)                 \
  X(2, 10, 5, 4)

template <class S, int L, int MODE, int NW, bool CE = false>
void launch_lanes(const DtpTrainArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((dtp::mlp_train_lanes_kernel<S, L, MODE, false, NW, false, CE>), dim3(a.n_models),
                     dim3(64 * NW), 0, st, a);
}

// split-batch step: member k of model m is block m + 8 k (blocks of absent models exit)
template <class S, int L, int NW, bool PROF = false, int MODE = DTP_MODE_ADAM, bool CE = false>
void launch_lanes_grp(const DtpTrainArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((dtp::mlp_train_lanes_kernel<S, L, MODE, PROF, NW, true, CE>), dim3(8 * a.groups),
                     dim3(64 * NW), 0, st, a);
}

// the lanes instances of one (shape, L, NW, loss, optimizer family)
template <class S, int L, int NW, bool CE, bool SGD>
TrainLaunchFn lanes_modes(int mode) {
  if constexpr (!SGD) {
    if (mode == DTP_MODE_ADAM) return &launch_lanes<S, L, DTP_MODE_ADAM, NW, CE>;
    if (mode == DTP_MODE_XGMI_ADAM) return &launch_lanes<S, L, DTP_MODE_XGMI_ADAM, NW, CE>;
  } else {
    if (mode == DTP_MODE_SGD) return &launch_lanes<S, L, DTP_MODE_SGD, NW, CE>;
    if (mode == DTP_MODE_XGMI_SGD) return &launch_lanes<S, L, DTP_MODE_XGMI_SGD, NW, CE>;
  }
  return nullptr;
}
template <class S, int NW, bool CE, bool SGD>
TrainLaunchFn lanes_by_l(int L, int mode) {
  return L == 4 ? lanes_modes<S, 4, NW, CE, SGD>(mode) : lanes_modes<S, 2, NW, CE, SGD>(mode);
}

// Instances of the several-lanes step (nullptr: none -> the one-lane kernel).  Adam + MSE
// for every DTP_TRAIN_SHAPES shape; SGD + MSE for the toy shape; the CE head (2,10,5,4) with
// Adam and SGD; bf16: the toy shape, Adam + MSE; two waves per SIMD: toy, Adam + MSE.
TrainLaunchFn lanes_inst(int in, int h, int nl, int out, int L, int NW, int mode, bool ce, bool bf16) {
  const bool sgd = mode == DTP_MODE_SGD || mode == DTP_MODE_XGMI_SGD;
  const bool toy = in == 2 && h == 10 && nl == 5 && out == 1;
  const bool ce4 = in == 2 && h == 10 && nl == 5 && out == 4;
  if (L != 2 && L != 4) return nullptr;
  if (NW == 8) {
    if (!toy || ce || sgd || bf16) return nullptr;
    return lanes_by_l<dtp::Stage<2, 10, 5, 1, false>, 8, false, false>(L, mode);
  }
  if (NW != 4) return nullptr;
  if (bf16) return (toy && !ce && !sgd) ? lanes_by_l<dtp::Stage<2, 10, 5, 1, false, true>, 4, false, false>(L, mode)
                                        : nullptr;
  if (ce) {
    if (!ce4) return nullptr;
    using T = dtp::Stage<2, 10, 5, 4, false>;
    return sgd ? lanes_by_l<T, 4, true, true>(L, mode) : lanes_by_l<T, 4, true, false>(L, mode);
  }
  if (sgd) return toy ? lanes_by_l<dtp::Stage<2, 10, 5, 1, false>, 4, false, true>(L, mode) : nullptr;
#define X(I, H, N, O) \
  if (in == I && h == H && nl == N && out == O) return lanes_by_l<dtp::Stage<I, H, N, O, false>, 4, false, false>(L, mode);
  DTP_TRAIN_SHAPES(X)
#undef X
  return nullptr;
}

// Instances of the split-batch step (4-lanes members; one rank, or several with the flat
// xGMI exchange): toy fp32 with Adam or SGD, toy bf16 with Adam, the CE head with Adam or SGD
TrainLaunchFn grp_inst(int in, int h, int nl, int out, int mode, bool ce, bool bf16) {
  const bool toy = in == 2 && h == 10 && nl == 5 && out == 1;
  const bool ce4 = in == 2 && h == 10 && nl == 5 && out == 4;
  using T = dtp::Stage<2, 10, 5, 1, false>;
  using C4 = dtp::Stage<2, 10, 5, 4, false>;
  using B = dtp::Stage<2, 10, 5, 1, false, true>;
  if (mode == DTP_MODE_GRAD) return nullptr;
  const bool sgd = mode == DTP_MODE_SGD || mode == DTP_MODE_XGMI_SGD;
  const bool xg = mode == DTP_MODE_XGMI_ADAM || mode == DTP_MODE_XGMI_SGD;
  if (bf16) {
    if (!toy || ce || sgd) return nullptr;
    return xg ? &launch_lanes_grp<B, 4, 4, false, DTP_MODE_XGMI_ADAM> : &launch_lanes_grp<B, 4, 4>;
  }
  if (ce) {
    if (!ce4) return nullptr;
    switch (mode) {
      case DTP_MODE_ADAM: return &launch_lanes_grp<C4, 4, 4, false, DTP_MODE_ADAM, true>;
      case DTP_MODE_SGD: return &launch_lanes_grp<C4, 4, 4, false, DTP_MODE_SGD, true>;
      case DTP_MODE_XGMI_ADAM: return &launch_lanes_grp<C4, 4, 4, false, DTP_MODE_XGMI_ADAM, true>;
      default: return &launch_lanes_grp<C4, 4, 4, false, DTP_MODE_XGMI_SGD, true>;
    }
  }
  if (!toy) return nullptr;
  switch (mode) {
    case DTP_MODE_ADAM: return &launch_lanes_grp<T, 4, 4>;
    case DTP_MODE_SGD: return &launch_lanes_grp<T, 4, 4, false, DTP_MODE_SGD>;
    case DTP_MODE_XGMI_ADAM: return &launch_lanes_grp<T, 4, 4, false, DTP_MODE_XGMI_ADAM>;
    default: return &launch_lanes_grp<T, 4, 4, false, DTP_MODE_XGMI_SGD>;
  }
}

// the step instance of a launch: lanes per sample and waves per workgroup
struct LanePick {
  int L = 1, NW = 4;
  int GR = 1;  // workgroups per model (split-batch step, grp_core.h)
};

// threads of the workgroups the fused step instances launch (one-lane: kBlock; lanes:
// 64 NW, NW = 4 or 8)
constexpr int kStepThreads[] = {dtp::kBlock, 4 * 64, 8 * 64};

long long xgmi_bytes_for(int P, int n_models, int world, int slot16) {
  return 2ll * n_models * world * slot16 * 16ll;
}
int xgmi_slot16_threads(int P, int nth) { return dtp::xgmi_slot16(P, (P + nth - 1) / nth); }
int xgmi_max_slot16(int P) {
  int m = 0;
  for (int nth : kStepThreads) m = max(m, xgmi_slot16_threads(P, nth));
  return m;
}

// 4 lanes per sample for per-rank batches <= 64, 2 for <= 128, else the one-lane kernel
// (L = 1).  DTP_LANES=<L>[x<NW>] forces a choice (A/B runs; NW = 8 runs two waves per
// SIMD, 512 / L samples); a forced pick whose batch bound does not hold falls back to 1.
// Split-batch step (engine launches only: it owns the exchange buffer): a per-rank batch
// above 64 on one rank runs on ceil(batch / 64) workgroups per model, each the 4-lanes step
// on 64 samples, their gradients summed on chip.  DTP_GROUPS=1 turns it off (A/B runs).
// DTP_GROUPS: unset = the measured policy below, "on" = wherever an instance exists,
// "off" / "0" / "1" = never (A/B runs)
int pick_groups(const DtpTrainArgs& a, int in, int out, bool allow, bool fast1) {
  static const int env = [] {  // -1 policy, 0 off, 1 on
    const char* e = getenv("DTP_GROUPS");
    if (!e) return -1;
    return strcmp(e, "on") == 0 ? 1 : 0;
  }();
  static const bool forced_lanes = getenv("DTP_LANES") != nullptr;  // a forced lanes instance runs as asked
  // the caller's request (DtpTrainArgs.groups before the engine fills it in): 0 policy,
  // 1 on, -1 off; the environment wins (A/B runs)
  const int want = env >= 0 ? env : (a.groups > 0 ? 1 : (a.groups < 0 ? 0 : -1));
  if (!allow || want == 0 || forced_lanes || a.n_models > 8) return 1;
  if (a.smp.n * (in + out) > dtp::kLaneData) return 1;
  const int b = min(a.smp.batch, a.smp.num_samples);
  if (b <= 64) return 1;
  const int gr = (b + 63) / 64;
  // several ranks: one flat exchange over world x groups virtual members (xgmi_core.h)
  const int cap = a.smp.world == 1 ? dtp::kGrpMax : dtp::kXgmiMaxWorld / a.smp.world;
  if (gr > cap) return 1;
  if (want == 1) return gr;
  // the policy (docs/perf_notes.md "Round 5: the split-batch step"): on for 4 members per
  // model (per-rank batch 256 -- one rank: 3.35-3.40 vs 4.11 us/step, two ranks: 5.6 vs 6.2-6.6 in
  // the rehearsal); 2 members (batch 128) measured no better than the 2-lanes step
  (void)fast1;
  return gr >= 4 ? gr : 1;
}

LanePick pick_lanes(const DtpTrainArgs& a, int in, int out, bool fast) {
  static const LanePick forced = [] {
    LanePick f{0, 4};
    const char* e = getenv("DTP_LANES");
    if (e) {
      f.L = atoi(e);
      const char* x = strchr(e, 'x');
      if (x) f.NW = atoi(x + 1);
    }
    return f;
  }();
  LanePick r;
  if (!fast || a.smp.n * (in + out) > dtp::kLaneData) return r;
  // the largest batch a step sees: a rank's share of the epoch can be smaller than the
  // configured batch (strong scaling: 512 samples over 8 ranks -> 64 of batch 256)
  const int b = min(a.smp.batch, a.smp.num_samples);
  r.L = b <= dtp::kBlock / 4 ? 4 : (b <= dtp::kBlock / 2 ? 2 : 1);
  if ((forced.L == 1 || forced.L == 2 || forced.L == 4) && (forced.NW == 4 || forced.NW == 8)) {
    r.L = forced.L;
    r.NW = forced.L == 1 ? 4 : forced.NW;
  }
  if (b > 64 * r.NW / r.L) r = LanePick{};
  return r;
}

TrainLaunchFn resolve_train(const DtpTrainArgs& a, int in, int h, int nl, int out, int mode,
                            LanePick* pick = nullptr, bool allow_groups = false) {
  const bool base = fast_base_ok(a, in, out);
  const bool fast = fast_path_ok(a, in, out, mode);
  const bool ce = a.loss == DTP_LOSS_CE;
  LanePick lp = pick_lanes(a, in, out, base);
  if (base) {
    const int gr = pick_groups(a, in, out, allow_groups, fast);
    // A/B only (DTP_GRP_NW=8): the split-batch step on members of 128 samples, each the
    // two-waves-per-SIMD 4-lanes step (8 waves), half the members of the default -- toy
    // fp32 Adam + MSE at one rank (docs/perf_notes.md "Round 6: two members")
    static const bool nw8 = getenv("DTP_GRP_NW") && atoi(getenv("DTP_GRP_NW")) == 8;
    if (nw8 && gr > 1 && mode == DTP_MODE_ADAM && !ce && !a.bf16 && in == 2 && h == 10 && nl == 5 && out == 1) {
      const int b = min(a.smp.batch, a.smp.num_samples);
      const int gr8 = (b + 127) / 128;
      if (gr8 > 1 && a.smp.n * (in + out) <= dtp::kLaneData) {
        if (pick) *pick = LanePick{4, 8, gr8};
        return &launch_lanes_grp<dtp::Stage<2, 10, 5, 1, false>, 4, 8>;
      }
    }
    if (gr > 1) {
      if (TrainLaunchFn f = grp_inst(in, h, nl, out, mode, ce, a.bf16)) {
        if (pick) *pick = LanePick{4, 4, gr};
        return f;
      }
    }
    if (lp.L > 1) {
      if (TrainLaunchFn f = lanes_inst(in, h, nl, out, lp.L, lp.NW, mode, ce, a.bf16)) {
        if (pick) *pick = lp;
        return f;
      }
    }
  }
  if (pick) *pick = LanePick{};
  if (a.bf16) {
#define X(I, H, N, O) \
  if (in == I && h == H && nl == N && out == O) return train_fn<dtp::Stage<I, H, N, O, false, true>>(mode, fast);
    DTP_TRAIN_BF16_SHAPES(X)
#undef X
    return nullptr;
  }
#define X(I, H, N, O) \
  if (in == I && h == H && nl == N && out == O) return train_fn<dtp::Stage<I, H, N, O, false>>(mode, fast);
  DTP_TRAIN_SHAPES(X)
#undef X
  return nullptr;
}

// the xGMI receive buffer covers the picked instance's granule layout (peers' stores
// through a buffer resource are not bounds-checked: an undersized buffer is corrupted)
int check_xbuf(const DtpTrainArgs& a, int in, int h, int nl, int out, int mode, const LanePick& lp) {
  if ((mode != DTP_MODE_XGMI_ADAM && mode != DTP_MODE_XGMI_SGD) || a.xbuf_bytes <= 0) return 0;
  int P = 0;
  for (int l = 0; l < nl; ++l) P += (l == nl - 1 ? out : h) * ((l == 0 ? in : h) + 1);
  const int nth = lp.L > 1 ? 64 * lp.NW : dtp::kBlock;
  const long long need = xgmi_bytes_for(P, a.n_models, a.smp.world * lp.GR, xgmi_slot16_threads(P, nth));
  if (need > a.xbuf_bytes) {
    char m[160];
    snprintf(m, sizeof m, "xGMI receive buffer too small: %lld bytes needed, %d allocated", need, a.xbuf_bytes);
    return set_err(-5, m);
  }
  return 0;
}

int validate_train(const DtpTrainArgs* a, int mode) {
  if (!a) return set_err(-1, "null args");
  if (a->n_models <= 0 || a->n_steps <= 0) return set_err(-1, "n_models and n_steps must be positive");
  if (a->smp.batch <= 0 || a->smp.n <= 0) return set_err(-1, "empty dataset or batch");
  if (a->smp.mode != dtp::SAMPLER_EXPLICIT && (a->smp.steps_per_epoch <= 0 || a->smp.num_samples <= 0))
    return set_err(-1, "bad sampler geometry");
  if (a->smp.mode == dtp::SAMPLER_EXPLICIT && !a->idx) return set_err(-1, "explicit sampler without indices");
  if (a->smp.mode == dtp::SAMPLER_TABLE &&
      (!a->smp.perm || a->smp.perm_epochs <= 0 || (a->smp.perm_epochs & (a->smp.perm_epochs - 1))))
    return set_err(-1, "table sampler needs a power-of-two permutation ring");
  if (a->loss_log && a->loss_log_cap <= 0) return set_err(-1, "loss_log_cap must be positive");
  if (!a->params || !a->X || !a->Y || !a->step) return set_err(-1, "params, X, Y and step are required");
  if (mode == DTP_MODE_GRAD && !a->grad_out) return set_err(-1, "MODE_GRAD needs grad_out");
  if (mode != DTP_MODE_GRAD && !a->opt_m) return set_err(-1, "optimizer modes need opt_m");
  if ((mode == DTP_MODE_ADAM || mode == DTP_MODE_XGMI_ADAM) && !a->opt_v) return set_err(-1, "Adam needs opt_v");
  if (mode == DTP_MODE_XGMI_ADAM || mode == DTP_MODE_XGMI_SGD) {
    if (!a->peers || !a->epoch) return set_err(-1, "xGMI modes need the peer table and epoch counters");
    if (a->smp.world < 1 || a->smp.world > dtp::kXgmiMaxWorld || a->smp.rank < 0 || a->smp.rank >= a->smp.world)
      return set_err(-1, "xGMI modes serve 1..8 ranks");
  }
  return 0;
}

// Native step executor: the argument block and the kernel instance are fixed at
// creation, so a call costs one kernel launch (no per-call marshalling or
// dispatch on the host; the Python side calls it with (handle, n_steps, stream)).
struct TrainEngine {
  DtpTrainArgs a;
  TrainLaunchFn fn;
  int mode;
  LanePick pick;  // lanes per sample / waves of the chosen instance (L = 1: mlp_train_kernel)
  void* grp_mem = nullptr;  // split-batch step: [status 16 ints | epochs | granule buffer]
  ~TrainEngine() {
    if (grp_mem) (void)hipFree(grp_mem);
  }
};

// the split-batch step's device state, zeroed: 64 B of timeout words, the per-model epoch
// counters (64 B aligned), then the [2][n_models][GR][slot16] granule buffer
int grp_alloc(TrainEngine* e, int P) {
  const int nth = 64 * e->pick.NW;
  const long long slot = dtp::grp_slot16(P, (P + nth - 1) / nth);
  const long long gbytes = 2ll * e->a.n_models * e->pick.GR * slot * 16;
  const long long ebytes = ((long long)e->a.n_models * 4 + 63) & ~63ll;
  const long long total = 64 + ebytes + gbytes;
  if (hipMalloc(&e->grp_mem, total) != hipSuccess) {
    e->grp_mem = nullptr;
    return set_err(-3, "hipMalloc of the split-batch exchange buffer failed");
  }
  if (hipMemset(e->grp_mem, 0, total) != hipSuccess) return set_err(-3, "hipMemset of the exchange buffer failed");
  char* b = static_cast<char*>(e->grp_mem);
  e->a.grp_status = reinterpret_cast<int*>(b);
  e->a.grp_epoch = reinterpret_cast<unsigned*>(b + 64);
  e->a.grp_buf = b + 64 + ebytes;
  e->a.groups = e->pick.GR;
  return 0;
}

template <class S>
int launch_train_profile(const DtpTrainArgs* a, hipStream_t st) {
  if (!fast_path_ok(*a, S::IN, S::OUT, DTP_MODE_ADAM))
    return set_err(-2, "the profile instance is the FAST one: cached dataset, SAMPLER_TABLE sampler");
  hipLaunchKernelGGL((dtp::mlp_train_kernel<S, DTP_MODE_ADAM, true, true>), dim3(a->n_models), dim3(dtp::kBlock), 0,
                     st, *a);
  return check_launch("mlp_train_kernel<prof>");
}

template <class S, int L, int NW = 4>
int launch_lanes_profile(const DtpTrainArgs* a, hipStream_t st) {
  if (!fast_path_ok(*a, S::IN, S::OUT, DTP_MODE_ADAM) || min(a->smp.batch, a->smp.num_samples) > 64 * NW / L ||
      a->smp.n * (S::IN + S::OUT) > dtp::kLaneData)
    return set_err(-2, "the lanes profile instance needs the FAST configuration and batch <= 64 NW / L");
  hipLaunchKernelGGL((dtp::mlp_train_lanes_kernel<S, L, DTP_MODE_ADAM, true, NW>), dim3(a->n_models), dim3(64 * NW),
                     0, st, *a);
  return check_launch("mlp_train_lanes_kernel<prof>");
}

}  // namespace

extern "C" {


int dtp_mlp_train_bf16_supported(int in, int h, int nl, int out) {
#define X(I, H, N, O) \
  if (in == I && h == H && nl == N && out == O) return 1;
  DTP_TRAIN_BF16_SHAPES(X)
#undef X
  return 0;
}

int dtp_mlp_workspace_floats(int in, int h, int nl, int out) {
#define X(I, H, N, O) \
  if (in == I && h == H && nl == N && out == O) return dtp::Scal<dtp::Stage<I, H, N, O, false>>::WS;
  DTP_TRAIN_SHAPES(X)
#undef X
  return 0;
}

// bytes of one rank's receive buffer of the fused step's xGMI exchange
// ([parity 2][model][src rank][slot] of 16-byte granules, xgmi_core.h)
long long dtp_xgmi_fused_buffer_bytes(int P, int n_models, int world) {
  // sized for the instance with the most granules: xgmi_slot16 is not monotone in the
  // parameters per thread, so take the max over every instantiated thread count; and for
  // the split-batch step's virtual members (world x groups <= kXgmiMaxWorld slots)
  const int slots = world <= dtp::kXgmiMaxWorld ? dtp::kXgmiMaxWorld : world;
  return xgmi_bytes_for(P, n_models, slots, xgmi_max_slot16(P));
}

int dtp_mlp_param_count(int in, int h, int nl, int out) {
  int p = 0;
  for (int l = 0; l < nl; ++l) {
    const int di = l == 0 ? in : h, dq = l == nl - 1 ? out : h;
    p += dq * (di + 1);
  }
  return p;
}

int dtp_mlp_train(const DtpTrainArgs* a, int in, int h, int nl, int out, int mode, void* stream) {
  if (int rc = validate_train(a, mode)) return rc;
  if (mode == DTP_MODE_GRAD && a->n_steps != 1) return set_err(-4, "MODE_GRAD requires n_steps == 1");
  LanePick lp;
  TrainLaunchFn fn = resolve_train(*a, in, h, nl, out, mode, &lp);
  if (!fn) return set_err(-2, "mlp shape / mode not instantiated for the fused train kernel");
  if (int rc = check_xbuf(*a, in, h, nl, out, mode, lp)) return rc;
  fn(*a, (hipStream_t)stream);
  return check_launch("mlp_train_kernel");
}

void* dtp_train_engine_create(const DtpTrainArgs* a, int in, int h, int nl, int out, int mode) {
  if (validate_train(a, mode)) return nullptr;
  LanePick lp;
  TrainLaunchFn fn = resolve_train(*a, in, h, nl, out, mode, &lp, true);
  if (!fn) {
    set_err(-2, "mlp shape / mode not instantiated for the fused train kernel");
    return nullptr;
  }
  if (check_xbuf(*a, in, h, nl, out, mode, lp)) return nullptr;
  auto* e = new TrainEngine();
  e->a = *a;
  e->fn = fn;
  e->mode = mode;
  e->pick = lp;
  if (lp.GR > 1 && grp_alloc(e, dtp_mlp_param_count(in, h, nl, out))) {
    delete e;
    return nullptr;
  }
  return e;
}

// diagnostic: the engine's split-batch step (fp32 toy shape) as its PROF instance, phase
// stamps into prof (u64[8 * groups blocks][8][32], block b = model b % 8, member b / 8)
int dtp_train_engine_profile(void* h, int n_steps, int t0, void* prof, void* stream) {
  auto* e = static_cast<TrainEngine*>(h);
  if (!e || !prof || n_steps <= 0) return set_err(-1, "bad engine profile args");
  if (e->pick.GR <= 1 || e->a.bf16 || e->mode != DTP_MODE_ADAM)
    return set_err(-2, "the engine profile instance is the fp32 split-batch step");
  DtpTrainArgs a = e->a;
  a.n_steps = n_steps;
  a.host_t0 = t0;
  a.status = static_cast<int*>(prof);
  launch_lanes_grp<dtp::Stage<2, 10, 5, 1, false>, 4, 4, true>(a, (hipStream_t)stream);
  return check_launch("mlp_train_lanes_kernel<grp, prof>");
}

// workgroups per model of the engine's step (1, or the split-batch step's group size)
int dtp_train_engine_groups(void* h) {
  auto* e = static_cast<TrainEngine*>(h);
  return e ? e->pick.GR : set_err(-1, "null engine");
}

// the split-batch exchange's sticky timeout words {flag, epoch} (synchronous copy; 0/0
// when the engine has no split-batch step)
int dtp_train_engine_status(void* h, int* out2) {
  auto* e = static_cast<TrainEngine*>(h);
  if (!e || !out2) return set_err(-1, "null engine");
  out2[0] = out2[1] = 0;
  if (!e->a.grp_status) return 0;
  if (hipMemcpy(out2, e->a.grp_status, 2 * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return set_err(-3, "status copy failed");
  return 0;
}

// test hook: mark the split-batch exchange as timed out at `epoch` (sticky, as a real
// timeout would), so the next launch runs dead -- and must leave the state untouched
int dtp_train_engine_poison(void* h, int epoch) {
  auto* e = static_cast<TrainEngine*>(h);
  if (!e || !e->a.grp_status) return set_err(-1, "no split-batch exchange");
  const int w[2] = {1, epoch};
  if (hipMemcpy(e->a.grp_status, w, sizeof w, hipMemcpyHostToDevice) != hipSuccess)
    return set_err(-3, "status write failed");
  return 0;
}

// lanes per sample of the engine's kernel instance (1 = one lane per sample)
int dtp_train_engine_lanes(void* h) {
  auto* e = static_cast<TrainEngine*>(h);
  return e ? e->pick.L : set_err(-1, "null engine");
}

// lanes per sample (low byte), waves per workgroup (<< 8) and workgroups per model (<< 16)
// of the step a train engine would launch for these arguments (0: no fused instance)
int dtp_mlp_train_lanes(const DtpTrainArgs* a, int in, int h, int nl, int out, int mode) {
  if (validate_train(a, mode)) return 0;
  LanePick lp;
  return resolve_train(*a, in, h, nl, out, mode, &lp, true) ? (lp.L | (lp.NW << 8) | (lp.GR << 16)) : 0;
}

// n_steps iterations in ONE persistent launch on `stream`, starting at step t0 (the
// host's mirror of the device step counters; -1: read them on the device)
int dtp_train_engine_run(void* h, int n_steps, int t0, void* stream) {
  auto* e = static_cast<TrainEngine*>(h);
  if (!e) return set_err(-1, "null engine");
  if (n_steps <= 0) return set_err(-1, "n_steps must be positive");
  if (e->mode == DTP_MODE_GRAD && n_steps != 1) return set_err(-4, "MODE_GRAD requires n_steps == 1");
  e->a.n_steps = n_steps;
  e->a.host_t0 = t0;
  e->fn(e->a, (hipStream_t)stream);
  return check_launch("mlp_train_kernel");
}

void dtp_train_engine_destroy(void* h) { delete static_cast<TrainEngine*>(h); }

// diagnostic: toy shape, Adam, phase stamps into a->status (as u64[n_models][8][16])
int dtp_mlp_train_profile(const DtpTrainArgs* a, void* stream) {
  return launch_train_profile<dtp::Stage<2, 10, 5, 1, false>>(a, (hipStream_t)stream);
}

// same for the lanes step (toy shape), L = 2 or 4
int dtp_mlp_train_profile_lanes(const DtpTrainArgs* a, int lanes, void* stream) {
  using T = dtp::Stage<2, 10, 5, 1, false>;
  const int L = lanes & 0xff, NW = lanes >> 8 ? lanes >> 8 : 4;
  if (L == 2 && NW == 4) return launch_lanes_profile<T, 2>(a, (hipStream_t)stream);
  if (L == 4 && NW == 4) return launch_lanes_profile<T, 4>(a, (hipStream_t)stream);
  if (L == 2 && NW == 8) return launch_lanes_profile<T, 2, 8>(a, (hipStream_t)stream);
  if (L == 4 && NW == 8) return launch_lanes_profile<T, 4, 8>(a, (hipStream_t)stream);
  return set_err(-1, "lanes must be 2 or 4 (| waves << 8, waves 4 or 8)");
}

int dtp_sampler_indices(const dtp::SamplerCfg* s, long long t0, int n_steps, int* out, void* stream) {
  if (!s || !out || s->batch <= 0 || n_steps <= 0) return set_err(-1, "bad sampler probe args");
  dim3 grid((s->batch + 255) / 256, n_steps), block(256);
  hipLaunchKernelGGL(dtp::sampler_probe_kernel, grid, block, 0, (hipStream_t)stream, *s, t0, n_steps, out);
  return check_launch("sampler_probe_kernel");
}

}  // extern "C"
