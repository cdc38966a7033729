// Persistent layer-split (inter-layer model parallel) training step for gfx950.
//
// Reference: MultiGPUModel (demo_one_model_multi_gpu.py:17-42) puts layers 0-1 on
// dev0 and layers 2-4 on dev1, moves the [B,10] activation with .to(dev1) and lets
// autograd copy the gradient back; DDP(device_ids=None) all-reduces per-device
// buckets (:96-98); one Adam steps both stages (:107,128).  Host-driven, that is
// ~10 launches, two peer copies and a bucketed all-reduce per iteration.
//
// Here every stage is ONE workgroup resident on its own GPU for n_steps
// iterations (one lane per sample, batch <= 256), and the stages talk directly:
//   * forward: the stage's output activation [B, OUT] is stored into the next
//     stage's receive buffer as 16-byte granules {epoch, v0, v1, check} (one
//     system-scope store each, peer-mapped over xGMI: posted writes, no copy
//     engine, no host); the next stage's lanes poll their own granules;
//   * backward: the input gradient [B, IN] goes back the same way;
//   * the stage's weight gradient (MFMA dW tiles, mlp_core.h) is all-reduced over
//     the data-parallel ranks INSIDE the step (xgmi_core.h; per-device buckets,
//     overlapped for free: the last stage reduces while the first is still in its
//     backward), then Adam / SGD updates the stage's weights in LDS and registers.
// Epoch = global step + 1: a link buffer needs no parity -- stage s writes the
// activation of step t+1 only after it received the gradient of step t, which the
// next stage sends only after it consumed activation t (and symmetrically for the
// gradient), so a granule is never overwritten while it is still unread.
// Every spin is bounded (status word, then the step continues): a wedged
// neighbour can never hang the GPU.
#include "dtp_api.h"
#include "mlp_core.h"
#include "mlp_pipe.h"
#include "optim_core.h"
#include "xgmi_core.h"

namespace dtp {

constexpr int kSplitCache = 8192;  // floats of dataset staged in LDS (first / last stage)

// cache policy of a link: sc1 = device scope (both stages on one GPU: the granules meet in
// the device's last-level cache, no round trip to HBM), sc0 | sc1 = system scope
// (neighbour on another GPU, uncached fine-grained buffer written over xGMI)
constexpr int kDevCoherent = 16;

// one lane's message: N floats as ceil(N/2) granules at granule index slot * G
template <int N>
DTP_DEV void link_send(void* buf, int slot, unsigned ep, const float (&v)[16], bool valid, bool local) {
  constexpr int G = (N + 1) / 2;
  if (!valid) return;
  const __amdgpu_buffer_rsrc_t rs = xgmi_rsrc(buf);
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint32_t x0 = __float_as_uint(v[2 * g]), x1 = 2 * g + 1 < N ? __float_as_uint(v[2 * g + 1]) : 0u;
    const u32x4 q = {ep, x0, x1, xgmi_check(ep, x0, x1)};
    if (local) __builtin_amdgcn_raw_buffer_store_b128(q, rs, (slot * G + g) * 16, 0, kDevCoherent);
    else __builtin_amdgcn_raw_buffer_store_b128(q, rs, (slot * G + g) * 16, 0, kSysCoherent);
  }
}

// poll this lane's granules of epoch ep in the local receive buffer (bounded)
template <int N>
DTP_DEV void link_recv(const void* buf, int slot, unsigned ep, float (&v)[16], bool valid, int* status,
                       int timeout_us, bool& dead, bool local) {
  constexpr int G = (N + 1) / 2;
  static_assert(G <= 16, "message too wide");
  const __amdgpu_buffer_rsrc_t ms = xgmi_rsrc(buf);
  uint32_t pend = valid ? ((1u << G) - 1u) : 0u;
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = 0.f;
  const unsigned long long deadline =
      __builtin_amdgcn_s_memrealtime() + (unsigned long long)(timeout_us > 0 ? timeout_us : 2000000) * 100ull;
  while (pend && !dead) {
    asm volatile("" ::: "memory");  // a poll is never merged with or hoisted above the previous one
    u32x4 x[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      x[g] = u32x4{0u, 0u, 0u, 0u};
      if ((pend >> g) & 1u)
        x[g] = local ? __builtin_amdgcn_raw_buffer_load_b128(ms, (slot * G + g) * 16, 0, kDevCoherent)
                     : __builtin_amdgcn_raw_buffer_load_b128(ms, (slot * G + g) * 16, 0, kSysCoherent);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (((pend >> g) & 1u) && x[g].x == ep && x[g].w == xgmi_check(ep, x[g].y, x[g].z)) {
        v[2 * g] = __uint_as_float(x[g].y);
        if (2 * g + 1 < N) v[2 * g + 1] = __uint_as_float(x[g].z);
        pend &= ~(1u << g);
      }
    }
    if (!pend) break;
    if (__builtin_amdgcn_s_memrealtime() > deadline) {
      dead = true;
      if (status) {
        atomicExch(&status[0], 1);
        atomicExch(&status[1], (int)ep);
      }
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Adam bias-correction scalars of the next kSplitAdamTab steps, formed once per that
// many steps in f64 (torch's host math) -- not per step
constexpr int kSplitAdamTab = 1024;

template <class S>
struct SplitSmem {
  float w[S::pad4(S::LP)];        // weights, row-major + transposed copies (mlp_core.h)
  float stage[kBlock / kWave][2 * kStgArr];  // per-wave dW staging, reused for the cross-wave reduction
  float data[kSplitCache];
  float2 adam_tab[kSplitAdamTab];  // {lr / (1 - b1^t), sqrt(1 - b2^t)} of steps t0 + base + e + 1
};

// stages of >= 2 layers: the fused step's software-pipelined schedule (mlp_pipe.h)
// with its LDS blocks (mlp_scalar.h), plus layer 0 row-major for the input gradient
// a non-first stage sends back; one staging area per wave (two when the first and last
// layer tiles pack), reused for the cross-wave reduction
template <class S>
struct SplitPipeSmem {
  static constexpr int AREAS = Scal<S>::PACK ? 2 : 1;
  // one float past each block: the sink the non-owning slots' scatter stores land in
  static constexpr int WB_SINK = Scal<S>::LW, W0R_SINK = S::dout(0) * S::pad4(S::IN);
  alignas(16) float wb[WB_SINK + 4];
  alignas(16) float w0r[W0R_SINK + 4];
  alignas(16) float stage[kBlock / kWave][AREAS][2 * kStgArr];
  float data[kSplitCache];
  float2 adam_tab[kSplitAdamTab];
};

constexpr int kSplitSmemBytes = 120 * 1024;  // the largest stage's SplitSmem / SplitPipeSmem

// One pipeline stage, n_steps iterations.  FIRST: gathers the batch inputs from the
// dataset; LAST: gathers the targets and computes the MSE loss; otherwise the
// activation / gradient arrive over the links.  Runs as one workgroup of
// split_multi_kernel (all the stages that share a GPU are one launch, so they are
// co-resident by construction: no reliance on separate hardware queues).
template <class S, bool FIRST, bool LAST>
DTP_DEV void split_stage_body_v1(const DtpSplitStageArgs& a, unsigned char* smem) {
  constexpr int NL = S::NL, P = S::P, NPT = S::NPT;
  static_assert(kBlock / kWave * NL * 256 <= kBlock / kWave * 2 * kStgArr, "reduction tiles fit the staging area");
  static_assert(sizeof(SplitSmem<S>) <= kSplitSmemBytes, "stage LDS exceeds the shared block");
  SplitSmem<S>& sm = *reinterpret_cast<SplitSmem<S>*>(smem);
  const bool adam = a.optim == DTP_MODE_ADAM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const SamplerCfg smp = a.smp;
  const float slope = a.hp.slope;
  constexpr int XW = FIRST ? S::IN : 0;   // dataset columns this stage reads
  constexpr int YW = LAST ? S::OUT : 0;

  // ---- prologue: owned parameters + moments in registers, weights and dataset in LDS
  float pw[NPT], mr[NPT], vr[NPT];
  int tp[NPT], lp[NPT], lpt[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int p = NPT * tid + k;
    const bool own = p < P;
    pw[k] = own ? a.params[p] : 0.f;
    mr[k] = own ? a.opt_m[p] : 0.f;
    vr[k] = (own && adam) ? a.opt_v[p] : 0.f;
    tp[k] = tile_pos<S>(own ? p : 0);
    lp[k] = own ? lds_pos<S>(p) : -1;
    lpt[k] = own ? lds_pos_t<S>(p) : -1;
  }
  for (int e = tid; e < S::pad4(S::LP); e += kBlock) sm.w[e] = 0.f;
  const bool cached = a.cache_data && smp.n * (XW + YW) <= kSplitCache;
  if (cached) {
    if constexpr (FIRST)
      for (int e = tid; e < smp.n * S::IN; e += kBlock) sm.data[e] = a.X[e];
    if constexpr (LAST)
      for (int e = tid; e < smp.n * S::OUT; e += kBlock) sm.data[smp.n * XW + e] = a.Y[e];
  }
  const int t0 = a.step[0];
  // sampler cursor (epoch, batch of the epoch), advanced incrementally: no 64-bit
  // division per step
  int epoch = t0 / smp.steps_per_epoch;
  int bi = t0 - epoch * smp.steps_per_epoch;
  // the dataset index of this lane's sample at cursor (ep, b) -- requested a step ahead
  // (the ring / Feistel lookup overlaps the previous step's reduction and optimizer)
  auto index_at = [&](int ep, int b) -> int {
    if constexpr (!(FIRST || LAST)) {
      return 0;
    } else {
      BatchPos bp;
      bp.epoch = ep;
      bp.start = b * smp.batch;
      bp.size = min(smp.batch, smp.num_samples - bp.start);
      uint32_t keys[4];
      epoch_keys(smp, ep, keys);
      return tid < bp.size ? sample_index(smp, bp, keys, tid) : 0;
    }
  };
  // the sample pipeline (as the fused step's FAST instance): step t's inputs / targets are
  // gathered from LDS at the end of step t-1, from a dataset index loaded a whole step
  // before that -- so no step waits on a global load (a wait at the loop head would also
  // wait out the previous step's loss-log store)
  int e2 = epoch, b2 = bi;
  auto roll2 = [&]() {
    if (++b2 == smp.steps_per_epoch) {
      b2 = 0;
      ++e2;
    }
  };
  float nx[S::IN], ny[S::OUT];
  auto gather = [&](int di_) {
    di_ = (unsigned)di_ < (unsigned)smp.n ? di_ : 0;  // never index out of range
    if constexpr (FIRST)
      static_for<0, S::IN>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        nx[i] = cached ? sm.data[di_ * S::IN + i] : a.X[(size_t)di_ * S::IN + i];
      });
    if constexpr (LAST)
      static_for<0, S::OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        ny[j] = cached ? sm.data[smp.n * XW + di_ * S::OUT + j] : a.Y[(size_t)di_ * S::OUT + j];
      });
  };
  int di_next = 0;
  if constexpr (FIRST || LAST) {
    const int d0 = index_at(e2, b2);
    roll2();
    di_next = index_at(e2, b2);  // step t0 + 1
    roll2();
    gather(d0);
  }
  auto fill_adam = [&](int base) {
    const int n = min(kSplitAdamTab, a.n_steps - base);
    for (int e = tid; e < n; e += kBlock) {
      const uint64_t t1 = (uint64_t)t0 + (uint64_t)base + (uint64_t)e + 1u;
      const double bc1 = 1.0 - pow_int(a.hp.beta1, t1), bc2 = 1.0 - pow_int(a.hp.beta2, t1);
      sm.adam_tab[e] = make_float2((float)(a.hp.lr / bc1), (float)sqrt(bc2));
    }
  };
  if (adam) fill_adam(0);
  __syncthreads();  // pads zeroed before the owners scatter
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    if (lp[k] >= 0) sm.w[lp[k]] = pw[k];
    if (lpt[k] >= 0) sm.w[lpt[k]] = pw[k];
  }
  __syncthreads();

  bool link_dead = __hip_atomic_load(&a.status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  const bool prev_local = a.link_local & 1, next_local = (a.link_local >> 1) & 1;
  const XgmiCtx dp{a.dp_peers, a.status + 2, a.dp_world, a.dp_rank, 1, a.timeout_us};
  const bool use_dp = a.dp_world > 1;
  float* red = &sm.stage[0][0];

  for (int it = 0; it < a.n_steps; ++it) {
    const int t = t0 + it;
    const unsigned ep = (unsigned)t + 1u;
    const int bsz = min(smp.batch, smp.num_samples - bi * smp.batch);
    const bool valid = tid < bsz;
    if (++bi == smp.steps_per_epoch) {
      bi = 0;
      ++epoch;
    }
    // ---- forward
    float h[NL + 1][16];
    if constexpr (FIRST) {
      static_for<0, S::IN>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        h[0][i] = valid ? nx[i] : 0.f;
      });
    } else {
      link_recv<S::IN>(a.act_in, tid, ep, h[0], valid, a.status, a.timeout_us, link_dead, prev_local);
    }
    mlp_forward<S>(sm.w, h, slope);

    // ---- output gradient: from the next stage, or the MSE loss (last stage)
    float dz[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) dz[j] = 0.f;
    const float inv = 1.f / (float)(bsz * S::OUT);
    if constexpr (!LAST) {
      link_send<S::OUT>(a.act_out, tid, ep, h[NL], valid, next_local);
      float go[16];
      link_recv<S::OUT>(a.grad_in, tid, ep, go, valid, a.status, a.timeout_us, link_dead, next_local);
      static_for<0, S::OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        const float d = S::FINAL_ACT ? go[j] * leaky_grad_from_out(h[NL][j], slope) : go[j];
        dz[j] = valid ? d : 0.f;
      });
    } else {
      float lpart = 0.f;
      static_for<0, S::OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        const float y = valid ? ny[j] : 0.f;
        const float d = h[NL][j] - y;
        lpart = valid ? fmaf(d, d, lpart) : lpart;
        dz[j] = valid ? 2.f * d * inv : 0.f;
      });
      dz[S::OUT] = lpart;  // loss row of the output tile (mlp_backward LOSS_ROW)
    }

    // ---- backward: input-gradient chain (VALU) + dW tiles (MFMA, K = samples)
    f32x4 acc[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) acc[l] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dx[16];
    mlp_backward<S, !FIRST, LAST>(sm.w, h, dz, &sm.stage[wave][0], acc, slope, lane, dx);
    if constexpr (!FIRST) link_send<S::IN>(a.grad_out, tid, ep, dx, valid, prev_local);

    // ---- reduce the per-wave tiles (staging area reused once every wave is done)
    __syncthreads();
    store_partial_tiles<S>(red, acc, wave, lane);
    __syncthreads();
    float g[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) g[k] = sum_partial_tiles<S>(red, tp[k], kBlock / kWave);
    float loss = 0.f;
    if constexpr (LAST) {
      loss = sum_partial_tiles<S>(red, loss_tile_pos<S>(), kBlock / kWave) * inv;
    }
    // ---- data parallel: this stage's gradient (+ loss) summed over the ranks
    float gloss = loss;
    if (use_dp) gloss = xgmi_allreduce_slots<NPT>(dp, 0, P, g, loss, ep, tid);
    if constexpr (FIRST || LAST) {  // the next step's sample, and the index of the one after it
      gather(di_next);
      di_next = index_at(e2, b2);
      roll2();
    }

    // ---- optimizer (registers) + weight refresh (LDS)
    const float gs = a.hp.grad_scale;
    if (adam) {
      AdamScalars as = adam_consts(a.hp);
      const float2 sc = sm.adam_tab[it % kSplitAdamTab];
      as.step_size = sc.x;
      as.bc2_sqrt = sc.y;
#pragma unroll
      for (int k = 0; k < NPT; ++k)
        if (lp[k] >= 0) adam_update(pw[k], mr[k], vr[k], g[k] * gs, as);
    } else {
      const float lr = (float)a.hp.lr, mom = (float)a.hp.momentum, wd = (float)a.hp.weight_decay;
#pragma unroll
      for (int k = 0; k < NPT; ++k)
        if (lp[k] >= 0) sgd_update(pw[k], mr[k], g[k] * gs, lr, mom, wd, t == 0);
    }
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      if (lp[k] >= 0) sm.w[lp[k]] = pw[k];
      if (lpt[k] >= 0) sm.w[lpt[k]] = pw[k];
    }
    if constexpr (LAST) {
      const int owner = use_dp ? xgmi_loss_tid<NPT>(P, kBlock) : 0;
      if (tid == owner && a.loss_log) a.loss_log[t % a.loss_log_cap] = use_dp ? gloss * gs : loss;
    }
    __syncthreads();  // new weights visible; reduction tiles consumed before the next staging writes
    if (adam && (it + 1) % kSplitAdamTab == 0 && it + 1 < a.n_steps) {
      fill_adam(it + 1);  // every thread read this step's entry before the barrier above
      __syncthreads();
    }
  }

#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int p = NPT * tid + k;
    if (p < P) {
      a.params[p] = pw[k];
      a.opt_m[p] = mr[k];
      if (adam) a.opt_v[p] = vr[k];
    }
  }
  if (tid == 0) a.step[0] = t0 + a.n_steps;
}

// One pipeline stage of >= 2 layers on the fused step's pipelined schedule: the next
// layer's weight block streams in during the current layer, the dW MFMA K-steps ride
// between the input-gradient rows (mlp_pipe.h).  Same protocol, sampler, exchange and
// optimizer as split_stage_body_v1 (the one-layer stages keep that one).
#ifndef DTP_SPLIT_PROF
#define DTP_SPLIT_PROF 0  // 1 (diagnostic builds only): s_memtime phase stamps of the first 8 steps, lane 0 of
                          // wave 0 of the LAST stage, as u64 at float offset 32768 of its loss log
#endif
#define SPLIT_STAMP(K)                                                                            \
  do {                                                                                            \
    if constexpr (DTP_SPLIT_PROF && LAST) {                                                       \
      if (tid == 0 && it < 8 && a.loss_log) {                                                     \
        unsigned long long _t;                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");             \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        reinterpret_cast<unsigned long long*>(a.loss_log + 32768)[it * 16 + (K)] = _t;           \
      }                                                                                           \
    }                                                                                             \
  } while (0)

template <class S, bool FIRST, bool LAST>
DTP_DEV void split_stage_body_pipe(const DtpSplitStageArgs& a, unsigned char* smem) {
  using SC = Scal<S>;
  constexpr int NL = S::NL, P = S::P, NPT = S::NPT, NT = SC::NT;
  static_assert(NL >= 2, "one-layer stages run split_stage_body_v1");
  static_assert(NT * SC::TSZ <= 2 * kStgArr, "a wave's reduction tiles fit its staging area");
  static_assert(sizeof(SplitPipeSmem<S>) <= kSplitSmemBytes, "stage LDS exceeds the shared block");
  SplitPipeSmem<S>& sm = *reinterpret_cast<SplitPipeSmem<S>*>(smem);
  const bool adam = a.optim == DTP_MODE_ADAM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const SamplerCfg smp = a.smp;
  const float slope = a.hp.slope;
  constexpr int XW = FIRST ? S::IN : 0;
  constexpr int YW = LAST ? S::OUT : 0;
  constexpr int IP0 = S::pad4(S::IN);

  // ---- prologue: owned parameters + moments in registers, weight blocks and dataset in LDS
  float pw[NPT], mr[NPT], vr[NPT];
  int pfl[NPT], pb[NPT], tp[NPT], p0r[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int p = NPT * tid + k;
    const bool own = p < P;
    pw[k] = own ? a.params[p] : 0.f;
    mr[k] = own ? a.opt_m[p] : 0.f;
    vr[k] = (own && adam) ? a.opt_v[p] : 0.f;
    int pf_;
    scal_pos<S>(own ? p : 0, pf_, pb[k], tp[k], pfl[k]);
    if (!own) pfl[k] = pb[k] = -1;
    // layer-0 weights, row-major: the input gradient of a non-first stage
    const int q = p - S::gw(0);
    p0r[k] = (!FIRST && own && q >= 0 && q < S::gb(0)) ? (q / S::IN) * IP0 + q % S::IN : -1;
    // branch-free weight refresh: a slot without a copy in a block stores to its sink
    // (the fused step's idiom; the optimizer also runs on the non-owned slots: their
    // state is zeros / never stored)
    pfl[k] = pfl[k] >= 0 ? pfl[k] : SplitPipeSmem<S>::WB_SINK;
    pb[k] = pb[k] >= 0 ? pb[k] : SplitPipeSmem<S>::WB_SINK;
    p0r[k] = p0r[k] >= 0 ? p0r[k] : SplitPipeSmem<S>::W0R_SINK;
  }
  for (int e = tid; e < SC::LW; e += kBlock) sm.wb[e] = 0.f;
  for (int e = tid; e < S::dout(0) * IP0; e += kBlock) sm.w0r[e] = 0.f;
  // the dataset is in LDS (split_stage_body sends uncached runs to the round-3 body): the
  // sample gather is straight-line LDS code -- a global-load path beside it made the
  // compiler wait out every outstanding store (links, loss log) before each gather
  if constexpr (FIRST)
    for (int e = tid; e < smp.n * S::IN; e += kBlock) sm.data[e] = a.X[e];
  if constexpr (LAST)
    for (int e = tid; e < smp.n * S::OUT; e += kBlock) sm.data[smp.n * XW + e] = a.Y[e];
  const int t0 = a.step[0];
  int epoch = t0 / smp.steps_per_epoch;
  int bi = t0 - epoch * smp.steps_per_epoch;
  auto index_at = [&](int ep, int b) -> int {
    if constexpr (!(FIRST || LAST)) {
      return 0;
    } else {
      BatchPos bp;
      bp.epoch = ep;
      bp.start = b * smp.batch;
      bp.size = min(smp.batch, smp.num_samples - bp.start);
      uint32_t keys[4];
      epoch_keys(smp, ep, keys);
      return tid < bp.size ? sample_index(smp, bp, keys, tid) : 0;
    }
  };
  // the sample pipeline (as the fused step's FAST instance): step t's inputs / targets are
  // gathered from LDS at the end of step t-1, from a dataset index loaded a whole step
  // before that -- so no step waits on a global load (a wait at the loop head would also
  // wait out the previous step's loss-log store)
  int e2 = epoch, b2 = bi;
  auto roll2 = [&]() {
    if (++b2 == smp.steps_per_epoch) {
      b2 = 0;
      ++e2;
    }
  };
  float nx[S::IN], ny[S::OUT];
  auto gather = [&](int di_) {
    di_ = (unsigned)di_ < (unsigned)smp.n ? di_ : 0;  // never index out of range
    if constexpr (FIRST)
      static_for<0, S::IN>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        nx[i] = sm.data[di_ * S::IN + i];
      });
    if constexpr (LAST)
      static_for<0, S::OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        ny[j] = sm.data[smp.n * XW + di_ * S::OUT + j];
      });
  };
  int di_next = 0;
  if constexpr (FIRST || LAST) {
    const int d0 = index_at(e2, b2);
    roll2();
    di_next = index_at(e2, b2);  // step t0 + 1
    roll2();
    gather(d0);
  }
  auto fill_adam = [&](int base) {
    const int n = min(kSplitAdamTab, a.n_steps - base);
    for (int e = tid; e < n; e += kBlock) {
      const uint64_t t1 = (uint64_t)t0 + (uint64_t)base + (uint64_t)e + 1u;
      const double bc1 = 1.0 - pow_int(a.hp.beta1, t1), bc2 = 1.0 - pow_int(a.hp.beta2, t1);
      sm.adam_tab[e] = make_float2((float)(a.hp.lr / bc1), (float)sqrt(bc2));
    }
  };
  if (adam) fill_adam(0);
  auto scatter = [&]() {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      sm.wb[pfl[k]] = pw[k];
      sm.wb[pb[k]] = pw[k];
      if constexpr (!FIRST) sm.w0r[p0r[k]] = pw[k];
    }
  };
  __syncthreads();  // pads zeroed before the owners scatter
  scatter();
  __syncthreads();

  bool link_dead = __hip_atomic_load(&a.status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  const bool prev_local = a.link_local & 1, next_local = (a.link_local >> 1) & 1;
  const XgmiCtx dp{a.dp_peers, a.status + 2, a.dp_world, a.dp_rank, 1, a.timeout_us};
  const bool use_dp = a.dp_world > 1;
  float* const stg_pack = &sm.stage[wave][0][0];
  float* const stg_hid = &sm.stage[wave][SplitPipeSmem<S>::AREAS - 1][0];

  for (int it = 0; it < a.n_steps; ++it) {
    SPLIT_STAMP(0);
    const int t = t0 + it;
    const unsigned ep = (unsigned)t + 1u;
    const int bsz = min(smp.batch, smp.num_samples - bi * smp.batch);
    const bool valid = tid < bsz;
    if (++bi == smp.steps_per_epoch) {
      bi = 0;
      ++epoch;
    }
    const float inv = 1.f / (float)(bsz * S::OUT);
    // ---- forward (the first block is read here; the others stream in layer by layer)
    float h[NL + 1][16];
    if constexpr (FIRST) {
      static_for<0, S::IN>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        h[0][i] = valid ? nx[i] : 0.f;
      });
    } else {
      link_recv<S::IN>(a.act_in, tid, ep, h[0], valid, a.status, a.timeout_us, link_dead, prev_local);
    }
    SPLIT_STAMP(1);
    BBlk<S, NL - 1> pbt;
    TopB2<S> pbt2;
    {
      FBlk<S, 0> pb0;
      pb0.template load<0, FBlk<S, 0>::NR>(sm.wb);
      pipe_forward<S, 0>(sm.wb, pb0, h, slope, pbt, pbt2);
    }
    // ---- output gradient: from the next stage, or the MSE loss (last stage)
    SPLIT_STAMP(2);
    float dz[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) dz[j] = 0.f;
    float lpart = 0.f;
    if constexpr (!LAST) {
      link_send<S::OUT>(a.act_out, tid, ep, h[NL], valid, next_local);
      float go[16];
      link_recv<S::OUT>(a.grad_in, tid, ep, go, valid, a.status, a.timeout_us, link_dead, next_local);
      static_for<0, S::OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        const float d = S::FINAL_ACT ? go[j] * leaky_grad_from_out(h[NL][j], slope) : go[j];
        dz[j] = valid ? d : 0.f;
      });
    } else {
      static_for<0, S::OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        const float y = valid ? ny[j] : 0.f;
        const float d = h[NL][j] - y;
        lpart = valid ? fmaf(d, d, lpart) : lpart;
        dz[j] = valid ? 2.f * d * inv : 0.f;
      });
    }
    // ---- backward: input-gradient chain (VALU) + dW tiles (MFMA, K = samples)
    f32x4 acc[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    SPLIT_STAMP(3);
    const PipeBwdCtx<S> pc{sm.wb, stg_pack, stg_hid, lane, slope, lpart};
    if constexpr (NL >= 3) {
      pipe_backward<S>(pc, pbt, pbt2, h, dz, acc);
    } else {  // two layers: the top layer, then layer 0's tile
      NoBlk none;
      pipe_bwd_layer<S, 1>(pc, pbt, h, dz, acc, none);
      float* stg = pipe_stage<S, 0>(pc, h, dz);
      __builtin_amdgcn_wave_barrier();
      acc[SC::tile(0)] = TileKind<S>::outer(stg, stg + kStgArr, acc[SC::tile(0)], lane);
      __builtin_amdgcn_wave_barrier();
    }
    if constexpr (!FIRST) {  // dz now holds layer 0's output gradient: dx = W_0^T dz
      // the whole row-major block in flight at once (broadcast ds_read_b128; LDS returns in
      // order), then output-major pair FMAs: the order of every sum is j ascending
      constexpr int NQ = IP0 / 4, O0 = S::dout(0);
      float4 w4[O0][NQ];
      static_for<0, O0>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        static_for<0, NQ>([&](auto QC) {
          constexpr int q = decltype(QC)::value;
          w4[j][q] = row_quad<S::IN, q>(sm.w0r + j * IP0);
        });
      });
      f32x2 gx[2 * NQ];
      static_for<0, 2 * NQ>([&](auto QC) { gx[decltype(QC)::value] = f32x2{0.f, 0.f}; });
      static_for<0, O0>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        const f32x2 d = f32x2{dz[j], dz[j]};
        static_for<0, NQ>([&](auto QC) {
          constexpr int q = decltype(QC)::value;
          if constexpr (4 * q < S::IN) gx[2 * q] = __builtin_elementwise_fma(f32x2{w4[j][q].x, w4[j][q].y}, d, gx[2 * q]);
          if constexpr (4 * q + 2 < S::IN)
            gx[2 * q + 1] = __builtin_elementwise_fma(f32x2{w4[j][q].z, w4[j][q].w}, d, gx[2 * q + 1]);
        });
      });
      float dx[16];
      static_for<0, S::IN>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        dx[i] = (i & 1) ? gx[i / 2].y : gx[i / 2].x;
      });
      link_send<S::IN>(a.grad_out, tid, ep, dx, valid, prev_local);
    }
    SPLIT_STAMP(4);
    // ---- each wave parks its partial tiles in its own staging area (its staging reads
    // were issued before these writes); one barrier publishes them
    {
      const int q = lane >> 4, col = lane & 15;
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
        *reinterpret_cast<f32x4*>(stg_pack + tt * SC::TSZ + SC::tslot(4 * q, col)) = acc[tt];
    }
    __syncthreads();
    SPLIT_STAMP(5);
    float g[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < kBlock / kWave; ++ww) v += sm.stage[ww][0][tp[k]];
      g[k] = v;
    }
    float loss = 0.f;
    if constexpr (LAST) {
      float ls = 0.f;
#pragma unroll
      for (int ww = 0; ww < kBlock / kWave; ++ww)
        ls += sm.stage[ww][0][SC::losspos()];
      loss = ls * inv;
    }
    SPLIT_STAMP(6);
    float gloss = loss;
    if (use_dp) gloss = xgmi_allreduce_slots<NPT>(dp, 0, P, g, loss, ep, tid);
    if constexpr (FIRST || LAST) {  // the next step's sample, and the index of the one after it
      gather(di_next);
      di_next = index_at(e2, b2);
      roll2();
    }
    SPLIT_STAMP(7);
    // ---- optimizer (registers) + weight refresh (LDS)
    const float gs = a.hp.grad_scale;
    if (adam) {
      AdamScalars as = adam_consts(a.hp);
      const float2 sc = sm.adam_tab[it % kSplitAdamTab];
      as.step_size = sc.x;
      as.bc2_sqrt = sc.y;
#pragma unroll
      for (int k = 0; k < NPT; ++k) adam_update(pw[k], mr[k], vr[k], g[k] * gs, as);
    } else {
      const float lr = (float)a.hp.lr, mom = (float)a.hp.momentum, wd = (float)a.hp.weight_decay;
#pragma unroll
      for (int k = 0; k < NPT; ++k) sgd_update(pw[k], mr[k], g[k] * gs, lr, mom, wd, t == 0);
    }
    scatter();
    if constexpr (LAST) {
      const int owner = use_dp ? xgmi_loss_tid<NPT>(P, kBlock) : 0;
      if (tid == owner && a.loss_log) a.loss_log[t % a.loss_log_cap] = use_dp ? gloss * gs : loss;
    }
    SPLIT_STAMP(8);
    __syncthreads();  // new weights visible; reduction tiles consumed before the next staging writes
    SPLIT_STAMP(9);
    if (adam && (it + 1) % kSplitAdamTab == 0 && it + 1 < a.n_steps) {
      fill_adam(it + 1);
      __syncthreads();
    }
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int p = NPT * tid + k;
    if (p < P) {
      a.params[p] = pw[k];
      a.opt_m[p] = mr[k];
      if (adam) a.opt_v[p] = vr[k];
    }
  }
  if (tid == 0) a.step[0] = t0 + a.n_steps;
}

#ifndef DTP_SPLIT_PIPE
#define DTP_SPLIT_PIPE 1  // 0: every stage on the round-3 body (A/B builds, build.variant)
#endif

template <class S, bool FIRST, bool LAST>
DTP_DEV void split_stage_body(const DtpSplitStageArgs& a, unsigned char* smem) {
  constexpr int XW = FIRST ? S::IN : 0, YW = LAST ? S::OUT : 0;
  const bool cached = a.cache_data && a.smp.n * (XW + YW) <= kSplitCache;
  if constexpr (DTP_SPLIT_PIPE && S::NL >= 2) {
    if (cached) {
      split_stage_body_pipe<S, FIRST, LAST>(a, smem);
      return;
    }
  }
  split_stage_body_v1<S, FIRST, LAST>(a, smem);
}

// (IN, H, NL, OUT, FINAL_ACT, FIRST): the contiguous layer ranges of the toy model
// as pipeline stages (the first entry: the whole model as ONE stage -- the split code's
// baseline with no links, scripts/split_cost.py) (first stages read the 2-feature input; stages that end inside
// the network carry the LeakyReLU of their last layer and are not last); the shape
// id of a stage is its position in this list
#define DTP_SPLIT_SHAPES(X)   \
  X(2, 10, 5, 1, false, 1)    \
  X(2, 10, 1, 10, true, 1)    \
  X(2, 10, 2, 10, true, 1)    \
  X(2, 10, 3, 10, true, 1)    \
  X(2, 10, 4, 10, true, 1)    \
  X(10, 10, 1, 10, true, 0)   \
  X(10, 10, 2, 10, true, 0)   \
  X(10, 10, 3, 10, true, 0)   \
  X(10, 10, 1, 1, false, 0)   \
  X(10, 10, 2, 1, false, 0)   \
  X(10, 10, 3, 1, false, 0)   \
  X(10, 10, 4, 1, false, 0)

// every stage placed on one GPU, one workgroup each (blockIdx.x = local stage).  One
// kernel holds the bodies of every stage shape of at most MAXNL layers: its registers are
// allocated for the largest of them, so the 4- and 5-layer bodies (which need all 512
// and spill) get their own instance and a launch of shorter stages never pays for them.
template <int MAXNL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1))) void split_multi_kernel(DtpSplitLaunch) {
  __shared__ __align__(16) unsigned char smem[kSplitSmemBytes];
  const int b = blockIdx.x;
  // this workgroup's stage arguments straight from the kernarg segment (uniform
  // loads): indexing the by-value parameter with blockIdx would copy all of it to scratch
  const DtpSplitLaunch* L = (const DtpSplitLaunch*)__builtin_amdgcn_kernarg_segment_ptr();
  const int shape = L->shape_id[b];
  const DtpSplitStageArgs a = L->stage[b];
  int id = 0;
#define X(I, H, N, O, F, FI)                                                                        \
  if constexpr (N <= MAXNL) {                                                                       \
    if (shape == id) split_stage_body<Stage<I, H, N, O, F>, (bool)FI, !F>(a, smem);                 \
  }                                                                                                 \
  ++id;
  DTP_SPLIT_SHAPES(X)
#undef X
}

}  // namespace dtp

extern "C" {

long long dtp_split_link_bytes(int width, int batch) { return (long long)batch * ((width + 1) / 2) * 16ll; }

// shape id of a stage (its position in DTP_SPLIT_SHAPES), -1 if not instantiated
int dtp_split_shape_id(int in, int h, int nl, int out, int final_act, int first) {
  int id = 0;
#define X(I, H, N, O, F, FI)                                                                        \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F && (bool)first == (bool)FI) \
    return id;                                                                                      \
  ++id;
  DTP_SPLIT_SHAPES(X)
#undef X
  return -1;
}

int dtp_split_stage_supported(int in, int h, int nl, int out, int final_act, int first) {
  return dtp_split_shape_id(in, h, nl, out, final_act, first) >= 0;
}

static int validate_stage(const DtpSplitStageArgs* a, int first, int last) {
  using dtp::set_err;
  if (!a || !a->params || !a->opt_m || !a->step || !a->status) return set_err(-1, "split stage: missing buffers");
  if (a->n_steps <= 0) return set_err(-1, "split stage: n_steps must be positive");
  if (a->smp.batch <= 0 || a->smp.batch > dtp::kBlock || a->smp.mode == dtp::SAMPLER_EXPLICIT)
    return set_err(-1, "split stage: batch must be 1..256 samples (one lane each) with a device sampler");
  if (a->optim != DTP_MODE_ADAM && a->optim != DTP_MODE_SGD) return set_err(-1, "split stage: adam or sgd");
  if (a->optim == DTP_MODE_ADAM && !a->opt_v) return set_err(-1, "split stage: Adam needs opt_v");
  if (first && !a->X) return set_err(-1, "split stage: the first stage needs the inputs");
  if (last && !a->Y) return set_err(-1, "split stage: the last stage needs the targets");
  if (!first && (!a->act_in || !a->grad_out)) return set_err(-1, "split stage: missing links to the previous stage");
  if (!last && (!a->act_out || !a->grad_in)) return set_err(-1, "split stage: missing links to the next stage");
  if (last && a->loss_log && a->loss_log_cap <= 0) return set_err(-1, "split stage: loss_log_cap");
  if (a->dp_world > 1 && (!a->dp_peers || a->dp_world > dtp::kXgmiMaxWorld || a->dp_rank < 0 ||
                          a->dp_rank >= a->dp_world))
    return set_err(-1, "split stage: data-parallel exchange serves 1..8 ranks with a peer table");
  return 0;
}

// the stages of one GPU as ONE launch (co-resident workgroups)
int dtp_split_launch(const DtpSplitLaunch* L, void* stream) {
  using dtp::set_err;
  if (!L || L->n < 1 || L->n > DTP_SPLIT_MAX_LOCAL) return set_err(-1, "split launch: 1..8 stages per GPU");
  static const int first_of[] = {
#define X(I, H, N, O, F, FI) FI,
      DTP_SPLIT_SHAPES(X)
#undef X
  };
  static const int last_of[] = {
#define X(I, H, N, O, F, FI) !F,
      DTP_SPLIT_SHAPES(X)
#undef X
  };
  static const int layers_of[] = {
#define X(I, H, N, O, F, FI) N,
      DTP_SPLIT_SHAPES(X)
#undef X
  };
  int maxnl = 0;
  constexpr int nshapes = sizeof(first_of) / sizeof(first_of[0]);
  for (int i = 0; i < L->n; ++i) {
    const int id = L->shape_id[i];
    if (id < 0 || id >= nshapes) return set_err(-2, "split launch: stage shape not instantiated");
    if (int rc = validate_stage(&L->stage[i], first_of[id], last_of[id])) return rc;
    if (L->stage[i].n_steps != L->stage[0].n_steps) return set_err(-1, "split launch: stages disagree on n_steps");
    maxnl = layers_of[id] > maxnl ? layers_of[id] : maxnl;
  }
  if (maxnl <= 3) hipLaunchKernelGGL(dtp::split_multi_kernel<3>, dim3(L->n), dim3(dtp::kBlock), 0, (hipStream_t)stream, *L);
  else hipLaunchKernelGGL(dtp::split_multi_kernel<5>, dim3(L->n), dim3(dtp::kBlock), 0, (hipStream_t)stream, *L);
  return dtp::check_launch("split_multi_kernel");
}

}  // extern "C"
