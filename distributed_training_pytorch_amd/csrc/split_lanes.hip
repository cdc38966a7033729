// Split-batch layer-split stages (round 6): GPipe in space.
//
// Reference: MultiGPUModel (demo_one_model_multi_gpu.py:17-42) splits the model by layers
// over two GPUs and moves the whole [B, 10] activation forward / its gradient back every
// iteration (:39-42, :122-128); no micro-batches.  split_train.hip runs each stage as ONE
// workgroup (one lane per sample): the iteration's critical path is stage 0's forward, a
// hand-off, stage 1's forward + backward, a hand-off and stage 0's backward + Adam, all on
// single-CU latency chains (9.9-10.3 us per iteration, docs/perf_notes.md).
//
// Here a stage's batch is split over M member workgroups ("micro-batches" of batch / M
// <= 64 samples), each running the 4-lanes schedule of mlp_lanes.h (4 lanes per sample,
// every hidden layer partitioned over the lanes of a DPP quad, dW tiles on MFMA):
//   * member k of stage s hands the activations of ITS samples to member k of stage s+1
//     and gets their gradients back -- each member pair is an independent 64-sample
//     pipeline, so the hand-off chains of the M micro-batches run side by side;
//   * a hand-off is one 16-byte granule per lane {ep ^ h(v), v0, v1, v2}: the lane's slice
//     of the sample's activation (3 of the 10 units), stored into the neighbour member's
//     receive buffer (sc1 on one GPU, system scope over xGMI) and polled there;
//   * the members' partial weight gradients (and loss) are summed on chip before every
//     member's identical optimizer step (grp_core.h: grp_allreduce_split3), or with
//     several data-parallel ranks in ONE flat cross-GPU exchange over ranks x members
//     (xgmi_core.h: xgmi_allreduce_g3) -- the hybrid split + DDP of the reference
//     (demo_one_model_multi_gpu.py:96-98).
// Placement: member k of local stage s is block 8 (s M + k); the other blocks of the grid
// exit at once.  Under the round-robin dispatch every member of the launch lands on ONE
// XCD, so the links and the member exchange meet in that XCD's L2 (speed only: the
// protocols are correct under any placement).
// Epoch of step t = t + 1; a link buffer needs no parity (split_train.hip's argument: the
// activation of step t + 1 is sent only after the gradient of step t was received).
#include <type_traits>

#include "dtp_api.h"
#include "grp_core.h"
#include "mlp_lanes.h"
#include "optim_core.h"
#include "sampler.h"
#include "xgmi_core.h"

namespace dtp {

constexpr int kSLData = 4096;     // floats of dataset staged in LDS (first: inputs, last: targets)
constexpr int kSLAdamTab = 1024;  // Adam bias-correction scalars formed per this many steps
constexpr int kSLMaxM = 8;        // members per stage

// 4 lanes per sample, 4 waves of 16 samples: 64 samples per member
template <class S, bool FIRST, bool LAST>
struct SLCfg {
  static constexpr int L = 4, NW = 4, NTH = 64 * NW, G = kWave / L, TS = G / 4;
  static constexpr int NL = S::NL, H = S::H, IN = S::IN, OUT = S::OUT;
  static constexpr int NO = (H + L - 1) / L;  // units of a hidden layer per lane (part)
  static constexpr int NOP = (NO + 3) & ~3;   // a part's slice padded to a float4
  static constexpr int NPR = (NO + 1) / 2;    // v_pk_fma pairs per slice
  static constexpr bool EXACT = NO * L == H;
  static constexpr int PL = LAST ? NL - 1 : NL;  // partitioned layers 0 .. PL-1 (LAST: the last one whole)
  static_assert(FIRST || S::IN == H, "a stage fed over a link takes the hidden width");
  static_assert(LAST || (S::OUT == H && S::FINAL_ACT), "a stage that feeds a link emits the activated hidden width");
  static_assert(!(LAST && FIRST && NL == 1), "a one-layer whole model has no partitioned layer");
  static_assert(NO <= 3, "a lane's slice is one 3-float granule");
  static_assert(H + 1 <= 15 && S::IN + 1 <= 15 && S::OUT + 1 <= 15, "tile row / column 15 is the staging sink");
  static constexpr int pad4(int x) { return (x + 3) & ~3; }
  static constexpr int din(int l) { return S::din(l); }
  static constexpr int dout(int l) { return S::dout(l); }
  // forward block of partitioned layer l: rows r <= din(l) (row din(l) = bias), a row =
  // [part][NOP] (W[p NO + k][r] at (r L + p) NOP + k)
  static constexpr int FR(int l) { return (din(l) + 1) * L * NOP; }
  static constexpr int f_off(int l) {
    int o = 0;
    for (int k = 0; k < l && k < PL; ++k) o += FR(k);
    return o;
  }
  static constexpr int RW = pad4(H + 1);  // the whole last layer: row o = W[o][0 .. H-1], b[o]
  static constexpr int f_last() { return f_off(PL); }
  static constexpr int LF = f_last() + (LAST ? OUT * RW : 0);
  // backward block of layer l (its input gradient): rows o < dout(l) of W_l[o][p NO + k]
  static constexpr bool has_b(int l) { return l >= 1 || !FIRST; }
  static constexpr int BR(int l) { return dout(l) * L * NOP; }
  static constexpr int b_off(int l) {
    int o = LF;
    for (int k = 0; k < l; ++k) o += has_b(k) ? BR(k) : 0;
    return o;
  }
  static constexpr int LW = b_off(NL);
  // per-layer staging (one area per layer, so no layer waits on another's operand reads):
  // sample s of the wave at [s & 3][row or col][s >> 2]; the MFMA reader lane (q, c) finds
  // its TS K-step operands contiguous
  static constexpr int QS = 16 * TS + 4;
  static constexpr int AREA = 4 * QS;
  // parked dW tiles: one per layer, column-major with a 20-float column stride (Scal)
  static constexpr int TSZ = 16 * 20;
  static constexpr int tslot(int row, int col) { return col * 20 + row; }
  static constexpr int losspos() { return (NL - 1) * TSZ + tslot(OUT, din(NL - 1)); }
  static constexpr int NPT = (S::P + NTH - 1) / NTH;
};

template <class S, bool FIRST, bool LAST>
struct SLSmem {
  using C = SLCfg<S, FIRST, LAST>;
  alignas(16) float wb[C::pad4(C::LW) + 4];          // weight blocks, then 4 sink floats
  alignas(16) float stg[C::NW][S::NL][2 * C::AREA];  // per wave, per layer: dz operand, h operand
  alignas(16) float red[C::NW][S::NL * C::TSZ];      // per-wave parked dW tiles
  alignas(16) float2 adam_tab[kSLAdamTab];
  alignas(16) float data[kSLData];
  // member exchange (grp_allreduce_split3) or the cross-rank one (xgmi_allreduce_g3)
  static constexpr int XF = (kGrpMax + 1) * grp_ps3(S::P) > xgmi_g3_lds_floats(S::P)
                                ? (kGrpMax + 1) * grp_ps3(S::P) : xgmi_g3_lds_floats(S::P);
  alignas(16) float xg[XF];
};

constexpr int kSLSmemBytes = 150 * 1024;  // the largest stage's SLSmem (the 5-layer whole model: ~111 KB)

// positions of stage parameter p (torch order): forward block, backward block (sink: none),
// parked dW tile
template <class S, bool FIRST, bool LAST>
DTP_DEV void sl_pos(int p, int& pf, int& pb, int& tp) {
  using C = SLCfg<S, FIRST, LAST>;
  constexpr int L = C::L, NO = C::NO, NOP = C::NOP;
  constexpr int SINK = C::pad4(C::LW);
  pf = SINK;
  pb = SINK;
  tp = 0;
  static_for<0, S::NL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    constexpr int I = S::din(l), O = S::dout(l);
    constexpr bool part = l < C::PL;
    if (p >= S::gw(l) && p < S::gb(l)) {
      const int q = p - S::gw(l), j = q / I, i = q - j * I;
      pf = part ? C::f_off(l) + (i * L + j / NO) * NOP + j % NO : C::f_last() + j * C::RW + i;
      if constexpr (C::has_b(l)) pb = C::b_off(l) + (j * L + i / NO) * NOP + i % NO;
      tp = l * C::TSZ + C::tslot(j, i);
    } else if (p >= S::gb(l) && p < S::gb(l) + O) {
      const int j = p - S::gb(l);
      pf = part ? C::f_off(l) + (I * L + j / NO) * NOP + j % NO : C::f_last() + j * C::RW + I;
      tp = l * C::TSZ + C::tslot(j, I);  // bias column = constant-1 input
    }
  });
}

// one lane's slice of a sample's activation / gradient: {ep ^ h(v), v0, v1, v2}.  local:
// the reader is on this GPU (sc1 write-through stores; plain: the reader is on this
// member's XCD, so a plain store that stays in the XCD's L2 is what its sc1 polls read
// fastest); else system scope (the reader's GPU over xGMI)
DTP_DEV void sl_send(void* buf, int idx, unsigned ep, const float (&v)[3], bool local, bool plain = false) {
  const uint32_t x0 = __float_as_uint(v[0]), x1 = __float_as_uint(v[1]), x2 = __float_as_uint(v[2]);
  const u32x4 q = {ep ^ xgmi_hash3(x0, x1, x2), x0, x1, x2};
  const __amdgpu_buffer_rsrc_t rs = xgmi_rsrc(buf);
  if (local && plain) __builtin_amdgcn_raw_buffer_store_b128(q, rs, idx * 16, 0, 0);
  else if (local) __builtin_amdgcn_raw_buffer_store_b128(q, rs, idx * 16, 0, 16);  // sc1: device scope
  else __builtin_amdgcn_raw_buffer_store_b128(q, rs, idx * 16, 0, kSysCoherent);
}

#ifndef DTP_SL_PLAIN_LINKS
#define DTP_SL_PLAIN_LINKS 1  // 0: every on-GPU link store write-through (A/B)
#endif

// poll this lane's granule of epoch ep (bounded; a timeout sets status[0..1])
DTP_DEV void sl_recv(const void* buf, int idx, unsigned ep, float (&v)[3], bool valid, int* status, int timeout_us,
                     bool& dead, bool local) {
  v[0] = v[1] = v[2] = 0.f;
  if (!valid || dead) return;
  const __amdgpu_buffer_rsrc_t ms = xgmi_rsrc(buf);
  unsigned long long deadline = 0;
  unsigned spins = 0;
  while (true) {
    asm volatile("" ::: "memory");  // a poll is never merged with or hoisted above the previous one
    const u32x4 x = local ? __builtin_amdgcn_raw_buffer_load_b128(ms, idx * 16, 0, 16)
                          : __builtin_amdgcn_raw_buffer_load_b128(ms, idx * 16, 0, kSysCoherent);
    if ((x.x ^ xgmi_hash3(x.y, x.z, x.w)) == ep) {
      v[0] = __uint_as_float(x.y);
      v[1] = __uint_as_float(x.z);
      v[2] = __uint_as_float(x.w);
      return;
    }
    if ((++spins & 63u) == 0u) {
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      if (!deadline) {
        deadline = now + (unsigned long long)(timeout_us > 0 ? timeout_us : 2000000) * 100ull;
      } else if (now > deadline) {
        if (status) {
          atomicExch(&status[0], 1);
          atomicExch(&status[1], (int)ep);
        }
        dead = true;
        return;
      }
    }
  }
}

template <class S, bool FIRST, bool LAST>
DTP_DEV void split_lanes_body(const DtpSplitStageArgs& a, unsigned char* smem, int M, int gk) {
  using C = SLCfg<S, FIRST, LAST>;
  using Sm = SLSmem<S, FIRST, LAST>;
  static_assert(sizeof(Sm) <= kSLSmemBytes, "stage LDS exceeds the shared block");
  constexpr int NL = S::NL, P = S::P, NPT = C::NPT, NTH = C::NTH, NO = C::NO, NOP = C::NOP, NPR = C::NPR;
  constexpr int TS = C::TS, H = S::H, PL = C::PL;
  Sm& sm = *reinterpret_cast<Sm*>(smem);
  const bool adam = a.optim == DTP_MODE_ADAM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int part = lane & (C::L - 1), ws = lane / C::L;
  const SamplerCfg smp = a.smp;
  const float slope = a.hp.slope;
  const bool lead = gk == 0;
  // this lane's sample: position loc of the member's slice of spm samples, batch position bk
  const int spm = (smp.batch + M - 1) / M;
  const int loc = wave * C::G + ws;
  const int bk = gk * spm + loc;
  const bool in_slice = loc < spm;
  const int lidx = bk * C::L + part;  // this lane's granule in a link buffer

  // ---- prologue: owned parameters / moments, step counter, dataset -> LDS
  float pw[NPT], mr[NPT], vr[NPT];
  int pf[NPT], pb[NPT], tp[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int p = NPT * tid + k;
    const bool own = p < P;
    pw[k] = own ? a.params[p] : 0.f;
    mr[k] = own ? a.opt_m[p] : 0.f;
    vr[k] = (own && adam) ? a.opt_v[p] : 0.f;
    sl_pos<S, FIRST, LAST>(own ? p : 0, pf[k], pb[k], tp[k]);
    if (!own) pf[k] = pb[k] = C::pad4(C::LW);  // the sink
  }
  const int t0 = a.step[0];
  for (int e = tid; e < C::pad4(C::LW) + 4; e += NTH) sm.wb[e] = 0.f;
  constexpr int XW = FIRST ? S::IN : 0;
  // inputs (first stage) then targets (last stage), LDS-DMA (the barrier below waits)
  if constexpr (FIRST || LAST)
    lds_dma_fill2<NTH>(sm.data, a.X, FIRST ? smp.n * S::IN : 0, a.Y, LAST ? smp.n * S::OUT : 0, tid);
  {  // this wave's staging areas: zero, then the constant-1 bias column of every layer
    float* s0 = &sm.stg[wave][0][0];
    for (int e = lane; e < NL * 2 * C::AREA; e += kWave) s0[e] = 0.f;
    static_for<0, NL>([&](auto LC) {
      constexpr int l = decltype(LC)::value;
      float* hb = &sm.stg[wave][l][C::AREA];
      for (int e = lane; e < 4 * TS; e += kWave) hb[(e / TS) * C::QS + C::din(l) * TS + e % TS] = 1.f;
    });
  }
  int epoch = t0 / smp.steps_per_epoch;
  int bi = t0 - epoch * smp.steps_per_epoch;
  auto fast_index = [&](int ep_, int b_) -> int {
    if constexpr (!(FIRST || LAST)) {
      return 0;
    } else {
      const int start = b_ * smp.batch;
      const int size = min(smp.batch, smp.num_samples - start);
      int q = smp.rank + (start + bk) * smp.world;
      q = q >= smp.n ? q - smp.n : q;
      q = q < smp.n ? q : smp.n - 1;
      const int di = table_epoch(smp, ep_)[q];
      return (in_slice && bk < size) ? di : -1;
    }
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
  __syncthreads();  // blocks zeroed, dataset in LDS
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const float wv = S::rnd(pw[k]);
    sm.wb[pf[k]] = wv;
    sm.wb[pb[k]] = wv;
  }
  auto gather = [&](int di, float (&x)[S::IN], float (&y)[S::OUT]) {
    const bool v = di >= 0;
    di = (unsigned)di < (unsigned)smp.n ? di : 0;
    if constexpr (FIRST)
      static_for<0, S::IN>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        x[i] = v ? sm.data[di * S::IN + i] : 0.f;
      });
    if constexpr (LAST)
      static_for<0, S::OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        y[j] = v ? sm.data[smp.n * XW + di * S::OUT + j] : 0.f;
      });
  };
  float nx[S::IN], ny[S::OUT];
  static_for<0, S::IN>([&](auto IC) { nx[decltype(IC)::value] = 0.f; });
  static_for<0, S::OUT>([&](auto JC) { ny[decltype(JC)::value] = 0.f; });
  auto fill_adam = [&](int base) {
    const int n = min(kSLAdamTab, a.n_steps - base);
    for (int e = tid; e < n; e += NTH) {
      const uint64_t t1 = (uint64_t)t0 + (uint64_t)base + (uint64_t)e + 1u;
      const double bc1 = 1.0 - pow_int(a.hp.beta1, t1), bc2 = 1.0 - pow_int(a.hp.beta2, t1);
      sm.adam_tab[e] = make_float2((float)(a.hp.lr / bc1), (float)sqrt(bc2));
    }
  };
  if (adam) fill_adam(0);
  __syncthreads();  // weights scattered, Adam table formed
  if constexpr (FIRST || LAST) gather(fidx0, nx, ny);

  const bool prev_local = a.link_local & 1, next_local = (a.link_local >> 1) & 1;
  bool link_dead = __hip_atomic_load(&a.status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  const bool use_dp = a.dp_world > 1;
  int* const xst = use_dp ? a.status + 2 : a.status + 4;  // the gradient exchange's timeout words
  bool xdead = __hip_atomic_load(xst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  const GrpCtx gctx{a.grp_buf, xst, M, gk, 1, a.timeout_us};
  const XgmiCtx xc{a.dp_peers, xst, a.dp_world, a.dp_rank, 1, a.timeout_us};
  const unsigned xcc = grp_xcc_id();
  bool gplain = false;
  // link hello: in its prologue every member stores its XCC id to each on-GPU neighbour
  // member (one granule past the batch's link granules, tagged with this launch's first
  // epoch); at the end of step 0 a member reads its readers' ids and, for a reader on its
  // own XCD, publishes its link granules with plain stores from step 1 on (the line stays
  // in the shared L2 where the reader's sc1 polls find it; a write-through store drops it
  // from L2).  Only the writer decides, readers always poll sc1: correct under any
  // placement, and a hello that has not arrived keeps the write-through form.
  const int hidx = smp.batch * C::L + gk;
  const unsigned htag = (unsigned)t0 + 1u;
  const bool plain_ok = DTP_SL_PLAIN_LINKS && (a.link_local & 4);  // neighbours in this launch
  if (plain_ok && tid == 0) {
    const float hv[3] = {__uint_as_float(xcc), 0.f, 0.f};
    if constexpr (!FIRST)
      if (prev_local) sl_send(a.grad_out, hidx, htag, hv, true);
    if constexpr (!LAST)
      if (next_local) sl_send(a.act_out, hidx, htag, hv, true);
  }
  bool plain_next = false, plain_prev = false;
  // per-lane LDS bases (mlp_train.hip's lanes kernel): the part's slice of the blocks, the
  // sample's slot in a staged operand (+ the part's first row / column), the MFMA reader's
  const float* const wlp = sm.wb + part * NOP;
  const int wslot = (ws & 3) * C::QS + (ws >> 2);
  const int wpart = wslot + part * NO * TS;
  const int rdoff = (lane >> 4) * C::QS + (lane & 15) * TS;
  auto slot_ok = [&](int k) { return C::EXACT || part * NO + k < H; };
  const bool p0 = part == 0;
  // a staging write with nothing to stage goes to row / column 15 of its sample slot (never
  // read): branch-free writes
  auto put = [&](float* tl, int off, bool ok, float v) { tl[ok ? off : wslot + 15 * TS] = v; };
  float* const sink = sm.wb + C::pad4(C::LW);

  for (int it = 0; it < a.n_steps; ++it) {
    const int t = t0 + it;
    const unsigned ep = (unsigned)t + 1u;
    const int bsz = min(smp.batch, smp.num_samples - bi * smp.batch);
    const bool valid = in_slice && bk < bsz;
    const float inv = 1.f / (float)(bsz * S::OUT);
    f32x4 acc[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) acc[l] = f32x4{0.f, 0.f, 0.f, 0.f};
    // ---------------- forward
    float hin[16];
    float own[NL][NOP];   // own slice of every partitioned layer's output
    float inown[NOP];     // !FIRST: own slice of the stage input (from the link)
    float x0[S::IN];
    if constexpr (FIRST) {
      static_for<0, S::IN>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        x0[i] = valid ? S::rnd(nx[i]) : 0.f;
        hin[i] = x0[i];
      });
    } else {
      float r3[3];
      sl_recv(a.act_in, lidx, ep, r3, valid, a.status, a.timeout_us, link_dead, prev_local);
#pragma unroll
      for (int k = 0; k < NOP; ++k) inown[k] = k < 3 ? r3[k < 3 ? k : 0] : 0.f;
      static_for<0, C::L>([&](auto PC) {
        constexpr int pp = decltype(PC)::value;
        static_for<0, NO>([&](auto KC) {
          constexpr int k = decltype(KC)::value;
          if constexpr (pp * NO + k < H) hin[pp * NO + k] = part_bcast<C::L, pp>(inown[k]);
        });
      });
    }
    static_for<0, PL>([&](auto LC) {
      constexpr int l = decltype(LC)::value;
      constexpr int I = C::din(l);
      float4 w[I + 1];
      static_for<0, I + 1>([&](auto RC) {
        constexpr int r = decltype(RC)::value;
        w[r] = row_quad<NO, 0>(wlp + C::f_off(l) + r * C::L * NOP);
      });
      f32x2 z[NPR];
      static_for<0, NPR>([&](auto RC) {
        constexpr int r = decltype(RC)::value;
        z[r] = quad_pair<r % 2>(w[I]);
      });
      static_for<0, I>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        const f32x2 hi = f32x2{hin[i], hin[i]};
        static_for<0, NPR>([&](auto RC) {
          constexpr int r = decltype(RC)::value;
          z[r] = __builtin_elementwise_fma(quad_pair<r % 2>(w[i]), hi, z[r]);
        });
      });
      static_for<0, NOP>([&](auto KC) {
        constexpr int k = decltype(KC)::value;
        if constexpr (k < NO) {
          const float v = S::rnd((k & 1) ? z[k / 2].y : z[k / 2].x);
          own[l][k] = S::rnd(fmaxf(v, v * slope));  // LeakyReLU, exact for 0 <= slope <= 1
        } else {
          own[l][k] = 0.f;
        }
      });
      static_for<0, C::L>([&](auto PC) {
        constexpr int pp = decltype(PC)::value;
        static_for<0, NO>([&](auto KC) {
          constexpr int k = decltype(KC)::value;
          if constexpr (pp * NO + k < H) hin[pp * NO + k] = part_bcast<C::L, pp>(own[l][k]);
        });
      });
    });
    float dzp[NOP];  // this lane's slice of the current layer's output gradient
#pragma unroll
    for (int k = 0; k < NOP; ++k) dzp[k] = 0.f;
    float lpart = 0.f;
    if constexpr (LAST) {
      // the whole last layer, every lane: z_o = b_o + sum_i W[o][i] h_i
      constexpr int OUT = S::OUT, I = C::din(NL - 1);
      float out[OUT];
      static_for<0, OUT>([&](auto OC) {
        constexpr int o = decltype(OC)::value;
        const float* row = sm.wb + C::f_last() + o * C::RW;
        float z = row[I];
        static_for<0, I>([&](auto IC) { z = fmaf(row[decltype(IC)::value], hin[decltype(IC)::value], z); });
        out[o] = S::rnd(z);
      });
      float dzl[OUT];
      static_for<0, OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        const float d = out[j] - ny[j];
        lpart = valid ? fmaf(d, d, lpart) : lpart;
        dzl[j] = valid ? S::rnd(2.f * d * inv) : 0.f;
      });
      // last layer's tile: (dz, loss) rows from part 0, its input's columns from every part
      constexpr int l = NL - 1;
      float* tl = &sm.stg[wave][l][0];
      static_for<0, OUT>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        put(tl, wslot + j * TS, p0, dzl[j]);
      });
      put(tl, wslot + OUT * TS, p0, lpart);
      static_for<0, NO>([&](auto KC) {
        constexpr int k = decltype(KC)::value;
        const float hv = l >= 1 ? own[l >= 1 ? l - 1 : 0][k] : inown[k];
        put(tl + C::AREA, wpart + k * TS, slot_ok(k), hv);
      });
      __builtin_amdgcn_wave_barrier();
      acc[l] = lane_tile<C, S>(lane_tile_ops<C>(tl, rdoff), acc[l]);
      if constexpr (C::has_b(l)) {
        // input-gradient slice: g_k = sum_o W[o][p NO + k] dz_o
        f32x2 g[NPR];
        static_for<0, NPR>([&](auto RC) { g[decltype(RC)::value] = f32x2{0.f, 0.f}; });
        static_for<0, OUT>([&](auto OC) {
          constexpr int o = decltype(OC)::value;
          const float4 wq = row_quad<NO, 0>(wlp + C::b_off(l) + o * C::L * NOP);
          const f32x2 d = f32x2{dzl[o], dzl[o]};
          static_for<0, NPR>([&](auto RC) {
            constexpr int r = decltype(RC)::value;
            g[r] = __builtin_elementwise_fma(quad_pair<r % 2>(wq), d, g[r]);
          });
        });
        static_for<0, NO>([&](auto KC) {
          constexpr int k = decltype(KC)::value;
          const float v = S::rnd((k & 1) ? g[k / 2].y : g[k / 2].x);
          if constexpr (l >= 1) dzp[k] = S::rnd(v * leaky_grad_from_out(own[l >= 1 ? l - 1 : 0][k], slope));
          else dzp[k] = v;  // a one-layer non-first last stage: this is the gradient it sends back
        });
      }
    } else {
      // the activation of this member's samples to the next stage, its gradient back
      float s3[3] = {own[NL - 1][0], NO > 1 ? own[NL - 1][NO > 1 ? 1 : 0] : 0.f,
                     NO > 2 ? own[NL - 1][NO > 2 ? 2 : 0] : 0.f};
      if (valid) sl_send(a.act_out, lidx, ep, s3, next_local, plain_next);
      float go[3];
      sl_recv(a.grad_in, lidx, ep, go, valid, a.status, a.timeout_us, link_dead, next_local);
      static_for<0, NO>([&](auto KC) {
        constexpr int k = decltype(KC)::value;
        dzp[k] = valid ? S::rnd(go[k] * leaky_grad_from_out(own[NL - 1][k], slope)) : 0.f;
      });
    }
    // partitioned layers, top down: tile (dz rows, input columns), then the input-gradient slice
    static_for<0, PL>([&](auto RC) {
      constexpr int l = PL - 1 - decltype(RC)::value;
      float* tl = &sm.stg[wave][l][0];
      static_for<0, NO>([&](auto KC) {
        constexpr int k = decltype(KC)::value;
        put(tl, wpart + k * TS, slot_ok(k), dzp[k]);
      });
      if constexpr (l >= 1) {
        static_for<0, NO>([&](auto KC) {
          constexpr int k = decltype(KC)::value;
          put(tl + C::AREA, wpart + k * TS, slot_ok(k), own[l >= 1 ? l - 1 : 0][k]);
        });
      } else if constexpr (FIRST) {
        static_for<0, S::IN>([&](auto IC) {
          constexpr int i = decltype(IC)::value;
          put(tl + C::AREA, wslot + i * TS, p0, x0[i]);
        });
      } else {
        static_for<0, NO>([&](auto KC) {
          constexpr int k = decltype(KC)::value;
          put(tl + C::AREA, wpart + k * TS, slot_ok(k), inown[k]);
        });
      }
      __builtin_amdgcn_wave_barrier();
      const auto to = lane_tile_ops<C>(tl, rdoff);
      if constexpr (C::has_b(l)) {
        float dzf[16];
        static_for<0, C::L>([&](auto PC) {
          constexpr int pp = decltype(PC)::value;
          static_for<0, NO>([&](auto KC) {
            constexpr int k = decltype(KC)::value;
            if constexpr (pp * NO + k < H) dzf[pp * NO + k] = part_bcast<C::L, pp>(dzp[k]);
          });
        });
        f32x2 g[NPR];
        static_for<0, NPR>([&](auto RC2) { g[decltype(RC2)::value] = f32x2{0.f, 0.f}; });
        static_for<0, H>([&](auto OC) {
          constexpr int o = decltype(OC)::value;
          const float4 wq = row_quad<NO, 0>(wlp + C::b_off(l) + o * C::L * NOP);
          const f32x2 d = f32x2{dzf[o], dzf[o]};
          static_for<0, NPR>([&](auto RC2) {
            constexpr int r = decltype(RC2)::value;
            g[r] = __builtin_elementwise_fma(quad_pair<r % 2>(wq), d, g[r]);
          });
        });
        acc[l] = lane_tile<C, S>(to, acc[l]);
        static_for<0, NO>([&](auto KC) {
          constexpr int k = decltype(KC)::value;
          const float v = S::rnd((k & 1) ? g[k / 2].y : g[k / 2].x);
          if constexpr (l >= 1) dzp[k] = S::rnd(v * leaky_grad_from_out(own[l >= 1 ? l - 1 : 0][k], slope));
          else dzp[k] = v;  // layer 0 of a non-first stage: the input gradient to send back
        });
      } else {
        acc[l] = lane_tile<C, S>(to, acc[l]);
      }
    });
    if constexpr (!FIRST) {  // the stage input's gradient back to the previous stage
      float s3[3] = {dzp[0], NO > 1 ? dzp[NO > 1 ? 1 : 0] : 0.f, NO > 2 ? dzp[NO > 2 ? 2 : 0] : 0.f};
      if (valid) sl_send(a.grad_out, lidx, ep, s3, prev_local, plain_prev);
    }
    // ---------------- the waves' partial tiles -> this member's gradient
    {
      const int q = lane >> 4, col = lane & 15;
#pragma unroll
      for (int l = 0; l < NL; ++l)
        *reinterpret_cast<f32x4*>(&sm.red[wave][l * C::TSZ + C::tslot(4 * q, col)]) = acc[l];
    }
    __syncthreads();
    const float2 adam_sc = adam ? sm.adam_tab[it % kSLAdamTab] : make_float2(0.f, 1.f);
    float g[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      float s_ = 0.f;
#pragma unroll
      for (int ww = 0; ww < C::NW; ++ww) s_ += sm.red[ww][tp[k]];
      g[k] = s_;
    }
    float lsum = 0.f;
    if constexpr (LAST) {
#pragma unroll
      for (int ww = 0; ww < C::NW; ++ww) lsum += sm.red[ww][C::losspos()];
    }
    // ---------------- the members' (and ranks') sums
    float gloss = lsum * inv;  // this member's share of the rank's mean loss
    if (use_dp) {
      gloss = xgmi_allreduce_g3<P, NPT, NTH>(xc, 0, g, gloss, ep, tid, sm.xg, xdead, nullptr, M, gk);
    } else if (M > 1) {
      lsum = grp_allreduce_split3<P, NPT, NTH>(gctx, 0, g, lsum, ep, tid, xdead, sm.xg, xcc, gplain, nullptr,
                                               [] {});
      gloss = lsum * inv;
    }
    if (plain_ok && it == 0) {  // the readers' hello granules (sent in their prologues)
      auto hello = [&](const void* buf) -> bool {
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(xgmi_rsrc(buf), hidx * 16, 0, 16);
        return (x.x ^ xgmi_hash3(x.y, x.z, x.w)) == htag && x.y == xcc;
      };
      if constexpr (!LAST) plain_next = next_local && hello(a.grad_in);
      if constexpr (!FIRST) plain_prev = prev_local && hello(a.act_in);
    }
    // the next step's sample and the index of the one after it
    roll(epoch, bi);
    if constexpr (FIRST || LAST) {
      gather(fidx, nx, ny);
      roll(e2, b2);
      fidx = fast_index(e2, b2);
    }
    // ---------------- optimizer (registers) + weight refresh (LDS)
    const float gs = a.hp.grad_scale;
    if (adam) {
      AdamScalars as = adam_consts(a.hp);
      as.step_size = adam_sc.x;
      as.bc2_sqrt = adam_sc.y;
#pragma unroll
      for (int k = 0; k < NPT; ++k) adam_update(pw[k], mr[k], vr[k], g[k] * gs, as);
    } else {
      const float lr = (float)a.hp.lr, mom = (float)a.hp.momentum, wd = (float)a.hp.weight_decay;
#pragma unroll
      for (int k = 0; k < NPT; ++k) sgd_update(pw[k], mr[k], g[k] * gs, lr, mom, wd, t == 0);
    }
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const float wv = S::rnd(pw[k]);
      sm.wb[pf[k]] = wv;
      sm.wb[pb[k]] = wv;
    }
    (void)sink;
    if constexpr (LAST) {
      if (tid == 0 && lead && a.loss_log) a.loss_log[t % a.loss_log_cap] = use_dp ? gloss * gs : gloss;
    }
    __syncthreads();  // new weights visible; parked tiles consumed before the next park
    if (adam && (it + 1) % kSLAdamTab == 0 && it + 1 < a.n_steps) {
      fill_adam(it + 1);
      __syncthreads();
    }
  }
  // a launch whose link or gradient exchange timed out keeps the state from before it
  if (__syncthreads_or((link_dead || xdead) ? 1 : 0)) return;
  if (!lead) return;  // every member holds the same state: the first writes it back
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

// (IN, H, NL, OUT, FINAL_ACT, FIRST) of the split-batch stages: every DTP_SPLIT_SHAPES
// stage (split_train.hip) -- the toy model's contiguous layer ranges
#define DTP_SPLIT_LANES_SHAPES(X) \
  X(2, 10, 5, 1, false, 1)        \
  X(2, 10, 1, 10, true, 1)        \
  X(2, 10, 2, 10, true, 1)        \
  X(2, 10, 3, 10, true, 1)        \
  X(2, 10, 4, 10, true, 1)        \
  X(10, 10, 1, 10, true, 0)       \
  X(10, 10, 2, 10, true, 0)       \
  X(10, 10, 3, 10, true, 0)       \
  X(10, 10, 1, 1, false, 0)       \
  X(10, 10, 2, 1, false, 0)       \
  X(10, 10, 3, 1, false, 0)       \
  X(10, 10, 4, 1, false, 0)

// every local stage's M members in one launch (co-resident by construction: 8 x n x M
// blocks, the members at blocks 8 (s M + k)); shape ids are those of dtp_split_shape_id
template <int MAXNL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void split_lanes_kernel(DtpSplitLaunch) {
  __shared__ __align__(16) unsigned char smem[kSLSmemBytes];
  const DtpSplitLaunch* L = (const DtpSplitLaunch*)__builtin_amdgcn_kernarg_segment_ptr();
  const int b = blockIdx.x;
  if (b & 7) return;
  const int M = L->members > 0 ? L->members : 1;
  const int idx = b >> 3, s = idx / M, gk = idx - s * M;
  if (s >= L->n) return;
  const int shape = L->shape_id[s];
  const DtpSplitStageArgs a = L->stage[s];
  int id = 0;
#define X(I, H, N, O, F, FI)                                                               \
  if constexpr (N <= MAXNL) {                                                              \
    if (shape == id) split_lanes_body<Stage<I, H, N, O, F>, (bool)FI, !F>(a, smem, M, gk); \
  }                                                                                        \
  ++id;
  DTP_SPLIT_LANES_SHAPES(X)
#undef X
}

}  // namespace dtp

extern "C" {

// the shape list must stay split_train.hip's DTP_SPLIT_SHAPES (shape ids are shared)
int dtp_split_lanes_supported(int in, int h, int nl, int out, int final_act, int first) {
  const int id = dtp_split_shape_id(in, h, nl, out, final_act, first);
  if (id < 0) return 0;
  int k = 0;
#define X(I, H, N, O, F, FI)                                                                         \
  if (k == id) return (in == I && h == H && nl == N && out == O && (bool)final_act == F && (bool)first == (bool)FI); \
  ++k;
  DTP_SPLIT_LANES_SHAPES(X)
#undef X
  return 0;
}

// bytes of a stage's member exchange buffer (grp_core.h: [2 parities][members][slot16])
long long dtp_split_lanes_grp_bytes(int P, int members) {
  const int npt = (P + 255) / 256;
  return 2ll * members * dtp::grp_slot16(P, npt) * 16ll;
}

int dtp_split_lanes_launch(const DtpSplitLaunch* L, void* stream) {
  using dtp::set_err;
  if (!L || L->n < 1 || L->n > DTP_SPLIT_MAX_LOCAL) return set_err(-1, "split lanes: 1..8 stages per GPU");
  const int M = L->members;
  if (M < 1 || M > dtp::kSLMaxM) return set_err(-1, "split lanes: 1..8 members per stage");
  static const int layers_of[] = {
#define X(I, H, N, O, F, FI) N,
      DTP_SPLIT_LANES_SHAPES(X)
#undef X
  };
  static const int in_of[] = {
#define X(I, H, N, O, F, FI) I,
      DTP_SPLIT_LANES_SHAPES(X)
#undef X
  };
  static const int out_of[] = {
#define X(I, H, N, O, F, FI) O,
      DTP_SPLIT_LANES_SHAPES(X)
#undef X
  };
  static const int first_of[] = {
#define X(I, H, N, O, F, FI) FI,
      DTP_SPLIT_LANES_SHAPES(X)
#undef X
  };
  static const int last_of[] = {
#define X(I, H, N, O, F, FI) !F,
      DTP_SPLIT_LANES_SHAPES(X)
#undef X
  };
  constexpr int nshapes = sizeof(layers_of) / sizeof(layers_of[0]);
  int maxnl = 0;
  for (int i = 0; i < L->n; ++i) {
    const DtpSplitStageArgs& a = L->stage[i];
    const int id = L->shape_id[i];
    if (id < 0 || id >= nshapes) return set_err(-2, "split lanes: stage shape not instantiated");
    if (!a.params || !a.opt_m || !a.step || !a.status) return set_err(-1, "split lanes: missing buffers");
    if (a.n_steps <= 0 || a.n_steps != L->stage[0].n_steps) return set_err(-1, "split lanes: n_steps");
    if (a.optim != DTP_MODE_ADAM && a.optim != DTP_MODE_SGD) return set_err(-1, "split lanes: adam or sgd");
    if (a.optim == DTP_MODE_ADAM && !a.opt_v) return set_err(-1, "split lanes: Adam needs opt_v");
    const dtp::SamplerCfg& s = a.smp;
    if (s.batch <= 0 || (s.batch + M - 1) / M > 64) return set_err(-1, "split lanes: batch / members must be <= 64");
    // the link buffers hold batch x 5 granules (dtp_split_link_bytes, width 10): batch x 4
    // lane slices, then the members' hello granules
    if (M > s.batch) return set_err(-1, "split lanes: at most one member per sample");
    const bool first = first_of[id], last = last_of[id];
    if ((first || last) && (s.mode != dtp::SAMPLER_TABLE || !s.perm || s.perm_epochs <= 0 ||
                            (s.perm_epochs & (s.perm_epochs - 1))))
      return set_err(-1, "split lanes: the gathering stages read the device permutation ring (SAMPLER_TABLE)");
    if (s.n * ((first ? in_of[id] : 0) + (last ? out_of[id] : 0)) > dtp::kSLData)
      return set_err(-1, "split lanes: dataset exceeds the LDS cache");
    if (first && !a.X) return set_err(-1, "split lanes: the first stage needs the inputs");
    if (last && !a.Y) return set_err(-1, "split lanes: the last stage needs the targets");
    if (!first && (!a.act_in || !a.grad_out)) return set_err(-1, "split lanes: missing links to the previous stage");
    if (!last && (!a.act_out || !a.grad_in)) return set_err(-1, "split lanes: missing links to the next stage");
    if (a.dp_world > 1) {
      if (!a.dp_peers || a.dp_world * M > dtp::kXgmiMaxWorld || a.dp_rank < 0 || a.dp_rank >= a.dp_world)
        return set_err(-1, "split lanes: the cross-rank exchange serves ranks x members <= 8 with a peer table");
    } else if (M > 1 && !a.grp_buf) {
      return set_err(-1, "split lanes: members > 1 need the member exchange buffer");
    }
    maxnl = layers_of[id] > maxnl ? layers_of[id] : maxnl;
  }
  const dim3 grid(8 * L->n * M);
  if (maxnl <= 3) hipLaunchKernelGGL(dtp::split_lanes_kernel<3>, grid, dim3(256), 0, (hipStream_t)stream, *L);
  else hipLaunchKernelGGL(dtp::split_lanes_kernel<5>, grid, dim3(256), 0, (hipStream_t)stream, *L);
  return dtp::check_launch("split_lanes_kernel");
}

}  // extern "C"
