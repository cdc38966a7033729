// On-chip all-reduce among the GR workgroups that share ONE model's batch inside one
// launch (the split-batch step of mlp_train.hip: a model's per-rank batch spread over GR
// CUs, each running the several-lanes step on batch / GR samples).
//
// Why: the one-lane step at batch 256 keeps one CU per model busy and is latency-bound
// (4.1 us/step); the 4-lanes step does 64 samples in ~2.2 us.  Splitting the batch over
// GR = batch / 64 workgroups and summing their partial weight gradients on chip before
// the (redundant, bitwise identical) optimizer step trades ~half the step's chain for
// one on-chip hand-off.
//
// Protocol: the granule form of xgmi_core.h at device scope (MI355X_MICROARCH.md
// "Workgroup dispatch ... inter-workgroup visibility", recipe R2 of
// cdna_hip_programming.md Guideline 16):
//   * one coarse-grained device buffer, layout [parity 2][model][src workgroup][slot] of
//     16-byte granules {tag = exchange epoch, two fp32 values, check word};
//   * a workgroup stores each of its granules ONCE (every member reads the same slot --
//     no per-peer copies as over xGMI), with ONE 16-byte write-through (sc1) store;
//   * members poll the other GR - 1 slots with sc1 loads (L1 bypassed, so no acquire
//     fence is needed: every load of the handed-off bytes is an sc1 load and every store
//     an sc1 store) until tag and check word match; the own contribution stays in registers;
//   * sums run in workgroup order 0..GR-1 on every member -> bitwise identical gradients,
//     hence bitwise identical optimizer steps and weight replicas in every member;
//   * two parities + a monotonic epoch (device counter, never rewound): a member can run
//     at most one exchange ahead of another, so exchange e+1 never overwrites a slot still
//     being read for exchange e, and a granule from an earlier launch never matches;
//   * spins are bounded; a timeout sets status[0] / status[1] = epoch, the step continues.
// Placement: the members of a model are blocks m, m + 8, m + 16, ... (one XCD under the
// observed round-robin dispatch, so the hand-off stays in that XCD's L2) -- speed only:
// the protocol is correct under any placement (sc1 on both sides).
#pragma once
#include "xgmi_core.h"

namespace dtp {

constexpr int kGrpMax = 8;  // workgroups per model (batch <= 512 at 64 samples each)

#ifndef DTP_GRP_ST_AUX
#define DTP_GRP_ST_AUX 16  // granule stores: sc1 (write-through, device scope)
#endif
#ifndef DTP_GRP_LD_AUX
#define DTP_GRP_LD_AUX 16  // granule polls: sc1 (L2-served, L1 bypassed)
#endif
#ifndef DTP_GRP_SAME_XCD
// 1: after a launch's first exchange (write-through stores) has shown every member of the
// model on ONE XCD, publish with plain stores: the lines stay in that XCD's L2 and the
// members' sc1 polls hit there (a write-through store drops its line from L2, so a poll of
// it reads beyond L2).  Each member sends its XCC id in the loss granule's spare word, so
// every member takes the same decision.  Members on different XCDs keep write-through.
#define DTP_GRP_SAME_XCD 1
#endif
#ifndef DTP_GRP_SENTINEL
// 1: pollers wait on one granule per peer before sweeping: measured slower (4.43 vs 4.05
// us/step, profiles/r5_exchange/)
#define DTP_GRP_SENTINEL 0
#endif
#ifndef DTP_GRP_PUB_FIRST
#define DTP_GRP_PUB_FIRST 1  // pollers start after a barrier behind the publisher's store issue
#endif
#ifndef DTP_GRP_PIPE
#define DTP_GRP_PIPE 1  // split exchange pollers: two polls in flight
#endif
#ifndef DTP_GRP_SLEEP0
#define DTP_GRP_SLEEP0 0  // s_sleep units (64 cycles) before the pollers' first poll (the peers' stores land meanwhile)
#endif

#ifndef DTP_GRP_CHEAP_CHECK
// 1: the split exchange's granules carry a linear check word (3 VALU ops) instead of the
// two-round hash of the xGMI granules (~25 ops, per granule on the publisher AND per poll
// item on every poller, on the exchange's critical path).  On chip a granule is one 16-byte
// store that lands in one XCD's L2 (untorn on gfx950, MI355X_MICROARCH.md "Valid forms", R2);
// the tag is the exchange epoch, and the check word still rejects the tear the round-2 XOR
// form was weak against only up to a rotation (the cross-GPU exchange keeps the hash).
#define DTP_GRP_CHEAP_CHECK 1
#endif

DTP_DEV uint32_t grp_check(uint32_t e, uint32_t a, uint32_t b) {
#if DTP_GRP_CHEAP_CHECK
  return e ^ a ^ ((b << 13) | (b >> 19)) ^ 0x9E3779B9u;
#else
  return xgmi_check(e, a, b);
#endif
}

// granules per (parity, model, member) slot -- the xGMI slot size (xgmi_core.h)
DTP_HD constexpr int grp_slot16(int P, int npt) { return xgmi_slot16(P, npt); }

#ifndef DTP_GRP_G3
// 1: the split exchange packs THREE payload floats per 16-byte granule, {epoch ^ h, v0, v1,
// v2} (the tag word carries the check: a granule passes only as (epoch ^ h) ^ h(v) == epoch,
// so a stale slot of an earlier epoch never passes and a torn one only on a hash collision):
// 125 granules per member instead of 187 (toy shape), a third fewer publish stores, and the
// pollers request exactly their items (2 per lane at 4 members instead of 4)
#define DTP_GRP_G3 1
#endif
#ifndef DTP_GRP_OVERLAP
// 1: the caller's exchange-independent work (next sample gather, index request) runs inside
// the exchange's waits (grp_allreduce_split3's ov).  Measured slower: 3.90-3.92 vs 3.40 us/step
// (profiles/r5_exchange/overlap/) -- the wait counts around the polls lose their slack
#define DTP_GRP_OVERLAP 0
#endif
#ifndef DTP_GRP_ZERO_MISSING
// 1: a timed-out exchange's missing items add +0 (grp_allreduce_split3) instead of what an
// earlier exchange left in their LDS rows.  Off: the code on the pollers' path alone cost
// 3.42 vs 3.36 us/step (profiles/r5_exchange/zero_missing/); a timeout already marks the run
// failed through the status word (check_comm raises), whatever the values
#define DTP_GRP_ZERO_MISSING 0
#endif
#ifndef DTP_GRP_PIPE3
// the 3-float form's pollers: 0 = one poll in flight, 1 = two.  With 2 items per lane one poll
// measured faster (3.40 vs 3.44-3.46 us/step, profiles/r5_exchange/g3/); the 2-float form
// (4 items per lane) gained from two
#define DTP_GRP_PIPE3 0
#endif
// 3-float granules of a member: the P gradients, the loss and the member's XCC id
DTP_HD constexpr int grp_ng3(int P) { return (P + 2 + 2) / 3; }
// LDS floats per member of the 3-float form (pub, then one row per member)
DTP_HD constexpr int grp_ps3(int P) { return (3 * grp_ng3(P) + 3) & ~3; }
DTP_DEV uint32_t grp_hash3(uint32_t a, uint32_t b, uint32_t c) {
  return a ^ ((b << 11) | (b >> 21)) ^ ((c << 22) | (c >> 10)) ^ 0x9E3779B9u;
}

struct GrpCtx {
  void* buf;    // [2][n_models][GR][slot16] granules
  int* status;  // sticky timeout word pair (nullable)
  int GR, k, n_models, timeout_us;
};

// diagnostic (PROF instances only): s_memtime when the publish stores were issued, when the
// first poll was consumed and when the last granule arrived, and the number of polls
struct GrpProf {
  unsigned long long t_pub, t_first, t_end;
  unsigned polls;
  unsigned long long rt_pub = 0, rt_end = 0;  // s_memrealtime (chip-wide 100 MHz): publisher done, last granule
};

DTP_DEV unsigned grp_xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xFu;
}

DTP_DEV unsigned long long grp_clock() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// g (in): this member's partial sums of its NPT owned parameters; out: the sum over the
// GR members.  Returns the summed loss partial.  Called by every thread of the member.
template <int NPT, int NTHREADS>
// dead: the caller's sticky timeout flag (read from the status word once per launch)
DTP_DEV float grp_allreduce(const GrpCtx& c, int model, int P, float (&g)[NPT], float loss, unsigned epoch, int tid,
                            bool& dead, GrpProf* prof = nullptr) {
  constexpr int GPT = xgmi_gpt<NPT>();
  const int slot = grp_slot16(P, NPT);
  const int nthr = xgmi_nthr(P, NPT);
  const int ltid = xgmi_loss_tid<NPT>(P, NTHREADS);
  const size_t base = (size_t)((int)(epoch & 1u) * c.n_models + model) * c.GR;
  const bool has_g = tid < nthr;
  const bool has_l = tid == ltid;
  float v[GPT + 1][2];
#pragma unroll
  for (int k = 0; k < GPT; ++k) {
    v[k][0] = 2 * k < NPT ? g[2 * k] : 0.f;
    v[k][1] = 2 * k + 1 < NPT ? g[2 * k + 1] : 0.f;
  }
  v[GPT][0] = loss;
  v[GPT][1] = 0.f;
  auto gidx = [&](int k) { return k < GPT ? tid * GPT + k : nthr * GPT; };
  auto mine_k = [&](int k) { return k < GPT ? has_g : has_l; };
  const __amdgpu_buffer_rsrc_t rs = xgmi_rsrc(c.buf);
  // publish once: every member reads this slot
#pragma unroll
  for (int k = 0; k <= GPT; ++k) {
    if (!mine_k(k)) continue;
    const uint32_t x0 = __float_as_uint(v[k][0]), x1 = __float_as_uint(v[k][1]);
    const u32x4 q = {epoch, x0, x1, xgmi_check(epoch, x0, x1)};
    __builtin_amdgcn_raw_buffer_store_b128(q, rs, (int)(((base + c.k) * slot + gidx(k)) * 16), 0, DTP_GRP_ST_AUX);
  }
  float val[kGrpMax][GPT + 1][2];
  static_assert(kGrpMax * (GPT + 1) <= 64, "pending mask holds every (member, granule) pair");
  uint64_t pending = 0ull;
#pragma unroll
  for (int r = 0; r < kGrpMax; ++r) {
#pragma unroll
    for (int k = 0; k <= GPT; ++k) {
      val[r][k][0] = (r == c.k) ? v[k][0] : 0.f;
      val[r][k][1] = (r == c.k) ? v[k][1] : 0.f;
      if (r < c.GR && r != c.k && mine_k(k)) pending |= 1ull << (r * (GPT + 1) + k);
    }
  }
  if (prof) prof->t_pub = grp_clock();
  unsigned long long deadline = 0;
  unsigned spins = 0;
  while (pending && !dead) {
    u32x4 x[kGrpMax][GPT + 1];
    asm volatile("" ::: "memory");  // a poll is never merged with, or hoisted above, an earlier one
#pragma unroll
    for (int r = 0; r < kGrpMax; ++r) {
#pragma unroll
      for (int k = 0; k <= GPT; ++k) {
        x[r][k] = u32x4{0u, 0u, 0u, 0u};
        if ((pending >> (r * (GPT + 1) + k)) & 1ull)
          x[r][k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((base + r) * slot + gidx(k)) * 16), 0,
                                                          DTP_GRP_LD_AUX);
      }
    }
#pragma unroll
    for (int r = 0; r < kGrpMax; ++r) {
#pragma unroll
      for (int k = 0; k <= GPT; ++k) {
        const u32x4 q = x[r][k];
        if (((pending >> (r * (GPT + 1) + k)) & 1ull) && q.x == epoch && q.w == xgmi_check(epoch, q.y, q.z)) {
          val[r][k][0] = __uint_as_float(q.y);
          val[r][k][1] = __uint_as_float(q.z);
          pending &= ~(1ull << (r * (GPT + 1) + k));
        }
      }
    }
    if (prof && spins == 0) prof->t_first = grp_clock();
    if (!pending) break;
    // the clock is an SMEM read (it would hold the next LDS wait at lgkmcnt(0)): read it
    // only every 64 polls
    if ((++spins & 63u) == 0u) {
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      if (!deadline) {
        deadline = now + (unsigned long long)(c.timeout_us > 0 ? c.timeout_us : 2000000) * 100ull;
      } else if (now > deadline) {
        if (c.status) {
          atomicExch(&c.status[0], 1);
          atomicExch(&c.status[1], (int)epoch);
        }
        dead = true;
      }
    }
  }
  if (prof) {
    prof->t_end = grp_clock();
    prof->polls = spins + 1;
  }
  // member order 0..GR-1 on every member (absent members add +0)
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < kGrpMax; ++r) acc += val[r][k / 2][k & 1];
    g[k] = acc;
  }
  float lacc = 0.f;
#pragma unroll
  for (int r = 0; r < kGrpMax; ++r) lacc += val[r][GPT][0];
  return lacc;
}

// The same exchange with the roles split over the waves (the default): wave 0 publishes the
// member's granules, waves 1.. poll the peers'.  Why: on gfx9 loads and stores share ONE
// in-order vmcnt, so a wave that polls right after its own publish stores cannot consume its
// first poll before those write-through stores are acknowledged (measured: one poll after
// the publish took ~2.9 k cycles, every peer granule already there).  Pollers that never
// stored see a plain load round trip.  The member's own sums and the peers' values meet in
// LDS (two barriers):
//   pub [slot] float2 -- this member's granule payloads (written by their owner threads)
//   peer[kGrpMax][slot] float2 -- every peer's payloads, in member order
// Every thread then sums its parameters over the members in order 0..GR-1 (its own value
// from registers), exactly as grp_allreduce does: the results are the same bits.
// xcc: this member's XCC id; plain (in/out, per launch, starts false): publish with plain
// stores (DTP_GRP_SAME_XCD)
// pubfn (optional): pubfn(j) returns the payload of granule tid + 64 j of this member for the
// publisher wave, computed straight from the caller's data (the per-wave dW tiles): the
// owners then write nothing to LDS and the publisher starts without a barrier.  Without it
// the owners stage their payloads in pub[] first.
template <int P, int NPT, int NTHREADS, class PubFn = std::nullptr_t>
DTP_DEV float grp_allreduce_split(const GrpCtx& c, int model, float (&g)[NPT], float loss, unsigned epoch, int tid,
                                  bool& dead, float2* __restrict__ pub, float2* __restrict__ peer, unsigned xcc,
                                  bool& plain, GrpProf* prof = nullptr, PubFn pubfn = nullptr) {
  constexpr bool kDirect = !std::is_same_v<PubFn, std::nullptr_t>;
  constexpr int GPT = xgmi_gpt<NPT>();
  constexpr int NPOLL = NTHREADS - kWave;                 // poller lanes (waves 1..)
  constexpr int slot = grp_slot16(P, NPT);
  constexpr int nthr = xgmi_nthr(P, NPT);
  constexpr int ng = nthr * GPT + 1;                      // granules of a member: gradients + the loss
  constexpr int ltid = xgmi_loss_tid<NPT>(P, NTHREADS);
  static_assert(NTHREADS > kWave, "one publisher wave and at least one poller wave");
  const size_t base = (size_t)((int)(epoch & 1u) * c.n_models + model) * c.GR;
  const bool has_g = tid < nthr;
  // 1. the owners' payloads into LDS (unless the publisher computes them itself)
  if constexpr (!kDirect) {
#pragma unroll
    for (int k = 0; k < GPT; ++k)
      if (has_g) pub[tid * GPT + k] = make_float2(2 * k < NPT ? g[2 * k] : 0.f, 2 * k + 1 < NPT ? g[2 * k + 1] : 0.f);
    if (tid == ltid) pub[nthr * GPT] = make_float2(loss, 0.f);
    __syncthreads();
  }
  const __amdgpu_buffer_rsrc_t rs = xgmi_rsrc(c.buf);
  if (tid < kWave) {
    // 2a. wave 0 publishes every granule of this member once (one 16-byte store each:
    // write-through, or plain once every member is known to share this XCD)
    constexpr int MAXJ = (ng + kWave - 1) / kWave;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int q = tid + j * kWave;
      if (q >= ng) break;
      float2 v;
      if constexpr (kDirect) v = pubfn(j);
      else v = pub[q];
      if (q == ng - 1) v.y = __uint_as_float(xcc);  // the loss granule's spare word: the XCC id
      const uint32_t x0 = __float_as_uint(v.x), x1 = __float_as_uint(v.y);
      const u32x4 qq = {epoch, x0, x1, grp_check(epoch, x0, x1)};
      const int off = (int)(((base + c.k) * slot + q) * 16);
      if (DTP_GRP_SAME_XCD && plain) __builtin_amdgcn_raw_buffer_store_b128(qq, rs, off, 0, 0);
      else __builtin_amdgcn_raw_buffer_store_b128(qq, rs, off, 0, DTP_GRP_ST_AUX);
    }
    if (prof) {
      prof->t_pub = grp_clock();
      prof->rt_pub = __builtin_amdgcn_s_memrealtime();
    }
  }
  // the publisher's stores enter the CU's memory pipeline ahead of the pollers' loads (which
  // would otherwise fill it with sweeps of lines that cannot be there yet)
  if (DTP_GRP_PUB_FIRST) __syncthreads();
  if (tid >= kWave) {
    // 2b. waves 1.. poll the peers' granules: item i = (peer index i / ng, granule i % ng),
    // at most MAXI items per lane, all requested at once, only the missing ones re-polled
    constexpr int MAXI = ((kGrpMax - 1) * ng + NPOLL - 1) / NPOLL;
    static_assert(MAXI <= 32, "pending mask");
    const int pl = tid - kWave;
    const int total = (c.GR - 1) * ng;
    int off[MAXI], dst[MAXI];
    uint32_t pending = 0u;
#pragma unroll
    for (int j = 0; j < MAXI; ++j) {
      const int i = pl + j * NPOLL;
      const int ri = i / ng, q = i - ri * ng;
      const int r = ri < c.k ? ri : ri + 1;
      off[j] = (int)(((base + r) * slot + q) * 16);
      dst[j] = r * slot + q;
      if (i < total) pending |= 1u << j;
    }
    unsigned long long deadline = 0;
    unsigned spins = 0;
    if (prof) prof->t_pub = grp_clock();
    if (DTP_GRP_SLEEP0 > 0) __builtin_amdgcn_s_sleep(DTP_GRP_SLEEP0);
    auto expired = [&]() {
      if ((++spins & 63u) != 0u) return false;
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      if (!deadline) {
        deadline = now + (unsigned long long)(c.timeout_us > 0 ? c.timeout_us : 2000000) * 100ull;
      } else if (now > deadline) {
        if (c.status) {
          atomicExch(&c.status[0], 1);
          atomicExch(&c.status[1], (int)epoch);
        }
        return true;
      }
      return false;
    };
#if DTP_GRP_SENTINEL
    // Wait on one granule per peer first -- its loss granule, written by the publisher's LAST
    // store instruction -- with wave-uniform addresses (one request per wave-load), so the
    // poller waves do not flood L2 with sweeps of lines that are not there yet; by the time
    // the sentinels show, most of the payload has landed, and the sweep below collects it
    // (a sentinel orders nothing: the sweep still checks every granule).
    if (pending && !dead) {
      while (true) {
        bool all = true;
        asm volatile("" ::: "memory");
#pragma unroll
        for (int r = 0; r < kGrpMax; ++r) {
          if (r < c.GR && r != c.k) {
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((base + r) * slot + ng - 1) * 16), 0,
                                                                  DTP_GRP_LD_AUX);
            all = all && x.x == epoch;
          }
        }
        if (all) break;
        if (expired()) {
          dead = true;
          break;
        }
      }
    }
#endif
#if DTP_GRP_PIPE
    // Two polls in flight: a granule that lands just after one poll passed is seen by the
    // next one half a round trip later, not a whole one.  Every poll requests all of the
    // lane's items (satisfied ones too): a fixed load count per poll lets the waits stay
    // counted (vmcnt(MAXI)) instead of draining both polls.
    constexpr int PI = MAXI < 4 ? MAXI : 4;  // items a pipelined poll carries (c.GR <= 4: all of them)
    if (MAXI <= 4 || c.GR <= 4) {
      int poff[PI];
#pragma unroll
      for (int j = 0; j < PI; ++j) poff[j] = ((pending >> j) & 1u) ? off[j] : 0;  // absent items: any valid line
      auto issue = [&](u32x4 (&x)[PI]) {
        asm volatile("" ::: "memory");  // a poll is never merged with, or hoisted above, an earlier one
#pragma unroll
        for (int j = 0; j < PI; ++j) x[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, poff[j], 0, DTP_GRP_LD_AUX);
      };
      auto consume = [&](const u32x4 (&x)[PI]) {
#pragma unroll
        for (int j = 0; j < PI; ++j) {
          if (((pending >> j) & 1u) && x[j].x == epoch && x[j].w == grp_check(epoch, x[j].y, x[j].z)) {
            peer[dst[j]] = make_float2(__uint_as_float(x[j].y), __uint_as_float(x[j].z));
            pending &= ~(1u << j);
          }
        }
      };
      u32x4 xa[PI], xb[PI];
      if (pending && !dead) issue(xa);
      while (pending && !dead) {
        issue(xb);
        consume(xa);
        if (prof && spins == 0) prof->t_first = grp_clock();
        if (!pending) break;
        if (expired()) {
          dead = true;
          break;
        }
        issue(xa);
        consume(xb);
        if (!pending) break;
        if (expired()) {
          dead = true;
          break;
        }
      }
      pending = 0u;
    }
#endif
    while (pending && !dead) {
      u32x4 x[MAXI];
      asm volatile("" ::: "memory");  // a poll is never merged with, or hoisted above, an earlier one
#pragma unroll
      for (int j = 0; j < MAXI; ++j) {
        x[j] = u32x4{0u, 0u, 0u, 0u};
        if ((pending >> j) & 1u) x[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off[j], 0, DTP_GRP_LD_AUX);
      }
#pragma unroll
      for (int j = 0; j < MAXI; ++j) {
        if (((pending >> j) & 1u) && x[j].x == epoch && x[j].w == grp_check(epoch, x[j].y, x[j].z)) {
          peer[dst[j]] = make_float2(__uint_as_float(x[j].y), __uint_as_float(x[j].z));
          pending &= ~(1u << j);
        }
      }
      if (prof && spins == 0) prof->t_first = grp_clock();
      if (!pending) break;
      if (expired()) dead = true;
    }
    if (prof) {
      prof->t_end = grp_clock();
      prof->polls = spins + 1;
      prof->rt_end = __builtin_amdgcn_s_memrealtime();
    }
  }
  __syncthreads();
  // a poller that timed out told its workgroup through the status word; every thread of the
  // member takes the flag from there at the next launch (sticky), this step continues
  // 3. member-order sums (absent members and a timed-out peer's missing values add +0)
  float own[GPT + 1][2];
#pragma unroll
  for (int k = 0; k < GPT; ++k) {
    own[k][0] = 2 * k < NPT ? g[2 * k] : 0.f;
    own[k][1] = 2 * k + 1 < NPT ? g[2 * k + 1] : 0.f;
  }
  own[GPT][0] = loss;
  own[GPT][1] = 0.f;
  float acc[GPT + 1][2];
#pragma unroll
  for (int k = 0; k <= GPT; ++k) acc[k][0] = acc[k][1] = 0.f;
  const int gq0 = has_g ? tid * GPT : 0;
  if (DTP_GRP_SAME_XCD && !plain && !dead) {  // every member on this XCD: plain stores from the next exchange on
    bool same = true;
    for (int r = 0; r < c.GR; ++r)
      if (r != c.k) same = same && __float_as_uint(peer[r * slot + nthr * GPT].y) == xcc;
    plain = same;
  }
  for (int r = 0; r < c.GR; ++r) {
#pragma unroll
    for (int k = 0; k <= GPT; ++k) {
      const int q = k < GPT ? gq0 + k : nthr * GPT;
      const float2 pv = r == c.k ? make_float2(own[k][0], own[k][1]) : peer[r * slot + q];
      acc[k][0] += pv.x;
      acc[k][1] += pv.y;
    }
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) g[k] = acc[k / 2][k & 1];
  return acc[GPT][0];
}

// The split exchange with 3-float granules (DTP_GRP_G3, the default).  Same roles and
// barriers as grp_allreduce_split: the owners stage the member's payload in LDS
// (lds[0 .. PS): gradients p = 0..P-1, the loss at P, the XCC id at P + 1), wave 0 publishes
// granule q = floats [3q, 3q + 3) as {epoch ^ h(v), v}, waves 1.. poll the peers' granules
// into lds[PS (1 + r) ..] with PI items per lane (PI = the lane's share at this member count,
// two polls in flight), then every thread sums its parameters over the members in order
// 0..GR-1 (its own value from registers): every member computes the same bits.
// ov(): the caller's work that does not depend on the exchange (the next step's sample
// gather and index request), run exactly once by every thread while its memory requests are
// in flight: the publisher after its stores, a poller between its first poll's issue and
// its consumption.
template <int P, int NPT, int NTHREADS, int NG, class OverlapFn>
DTP_DEV float grp_allreduce_split3_ng(const GrpCtx& c, int model, float (&g)[NPT], float loss, unsigned epoch, int tid,
                                      bool& dead, float* __restrict__ lds, unsigned xcc, bool& plain, GrpProf* prof,
                                      OverlapFn ov) {
  constexpr int NGF = grp_ng3(P), PS = grp_ps3(P);
  constexpr int NPOLL = NTHREADS - kWave;  // poller lanes (waves 1..)
  constexpr int slot = grp_slot16(P, NPT);
  static_assert(NGF <= slot, "a member's 3-float granules fit its slot of the exchange buffer");
  static_assert(NTHREADS > kWave, "one publisher wave and at least one poller wave");
  float* const pub = lds;
  float* const peer = lds + PS;  // peer[r * PS + i]: member r's float i
  const size_t base = (size_t)((int)(epoch & 1u) * c.n_models + model) * c.GR;
  // 1. the payload into LDS
#pragma unroll
  for (int k = 0; k < NPT; ++k)
    if (NPT * tid + k < P) pub[NPT * tid + k] = g[k];
  if (tid == 0) {
    pub[P] = loss;
    pub[P + 1] = __uint_as_float(xcc);
#pragma unroll
    for (int i = P + 2; i < 3 * NGF; ++i) pub[i] = 0.f;
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = xgmi_rsrc(c.buf);
  if (tid < kWave) {
    // 2a. wave 0 publishes every granule of this member (all its LDS reads first, then the
    // stores back to back)
    constexpr int MAXJ = (NG + kWave - 1) / kWave;
    float v[MAXJ][3];
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int q = tid + j * kWave < NG ? tid + j * kWave : NG - 1;
      v[j][0] = pub[3 * q];
      v[j][1] = pub[3 * q + 1];
      v[j][2] = pub[3 * q + 2];
    }
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int q = tid + j * kWave;
      if (q < NG) {
        const uint32_t x0 = __float_as_uint(v[j][0]), x1 = __float_as_uint(v[j][1]), x2 = __float_as_uint(v[j][2]);
        const u32x4 qq = {epoch ^ grp_hash3(x0, x1, x2), x0, x1, x2};
        const int off = (int)(((base + c.k) * slot + q) * 16);
        if (DTP_GRP_SAME_XCD && plain) __builtin_amdgcn_raw_buffer_store_b128(qq, rs, off, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b128(qq, rs, off, 0, DTP_GRP_ST_AUX);
      }
    }
    if (prof) {
      prof->t_pub = grp_clock();
      prof->rt_pub = __builtin_amdgcn_s_memrealtime();
    }
    if (DTP_GRP_OVERLAP) ov();
  }
  if (DTP_GRP_PUB_FIRST) __syncthreads();
  if (tid >= kWave) {
    // 2b. item i = (peer index i / NG, granule i % NG), lane pl holds items pl + j NPOLL
    const int pl = tid - kWave;
    const int total = (c.GR - 1) * NG;
    unsigned long long deadline = 0;
    unsigned spins = 0;
    if (prof) prof->t_pub = grp_clock();
    auto expired = [&]() {
      if ((++spins & 63u) != 0u) return false;
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      if (!deadline) {
        deadline = now + (unsigned long long)(c.timeout_us > 0 ? c.timeout_us : 2000000) * 100ull;
      } else if (now > deadline) {
        if (c.status) {
          atomicExch(&c.status[0], 1);
          atomicExch(&c.status[1], (int)epoch);
        }
        return true;
      }
      return false;
    };
    // PI items per lane (one or two polls in flight, DTP_GRP_PIPE3); every poll requests all PI
    // items (a fixed load count keeps the waits counted), absent items read offset 0
    auto run = [&](auto PIC) {
      constexpr int PI = decltype(PIC)::value;
      int off[PI], dst[PI];
      uint32_t pending = 0u;
#pragma unroll
      for (int j = 0; j < PI; ++j) {
        const int i = pl + j * NPOLL;
        const int ri = i / NG, q = i - ri * NG;
        const int r = ri < c.k ? ri : ri + 1;
        const bool in = i < total;
        off[j] = in ? (int)(((base + r) * slot + q) * 16) : 0;
        dst[j] = r * PS + 3 * q;
        if (in) pending |= 1u << j;
      }
      auto issue = [&](u32x4 (&x)[PI]) {
        asm volatile("" ::: "memory");  // a poll is never merged with, or hoisted above, an earlier one
#pragma unroll
        for (int j = 0; j < PI; ++j) x[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off[j], 0, DTP_GRP_LD_AUX);
      };
      auto consume = [&](const u32x4 (&x)[PI]) {
#pragma unroll
        for (int j = 0; j < PI; ++j) {
          if (((pending >> j) & 1u) && (x[j].x ^ grp_hash3(x[j].y, x[j].z, x[j].w)) == epoch) {
            float* d = peer + dst[j];
            d[0] = __uint_as_float(x[j].y);
            d[1] = __uint_as_float(x[j].z);
            d[2] = __uint_as_float(x[j].w);
            pending &= ~(1u << j);
          }
        }
      };
      // a timed-out (or already dead) exchange: the items still missing add +0, not the
      // values an earlier exchange left in the LDS rows (the status word reports the timeout)
      auto zero_missing = [&]() {
#pragma unroll
        for (int j = 0; j < PI; ++j) {
          if ((pending >> j) & 1u) {
            float* d = peer + dst[j];
            d[0] = d[1] = d[2] = 0.f;
          }
        }
      };
      u32x4 xa[PI], xb[PI];
      bool ovd = !DTP_GRP_OVERLAP;
      if (!DTP_GRP_PIPE3) {  // one poll in flight (the default with 3-float granules)
        while (pending && !dead) {
          issue(xa);
          if (!ovd) {
            ov();
            ovd = true;
          }
          consume(xa);
          if (prof && spins == 0) prof->t_first = grp_clock();
          if (pending && expired()) dead = true;
        }
        if (!ovd) ov();
        if (DTP_GRP_ZERO_MISSING && pending) zero_missing();
        return;
      }
      if (pending && !dead) issue(xa);
      if (!ovd) {
        ov();
        ovd = true;
      }
      while (pending && !dead) {
        issue(xb);
        consume(xa);
        if (prof && spins == 0) prof->t_first = grp_clock();
        if (!pending) break;
        if (expired()) {
          dead = true;
          break;
        }
        issue(xa);
        consume(xb);
        if (!pending) break;
        if (expired()) {
          dead = true;
          break;
        }
      }
      if (DTP_GRP_ZERO_MISSING && pending) zero_missing();
    };
    constexpr int MAXI = ((kGrpMax - 1) * NGF + NPOLL - 1) / NPOLL;
    const int pi = (total + NPOLL - 1) / NPOLL;
    if (pi <= 1) run(std::integral_constant<int, 1>{});
    else if (pi <= 2) run(std::integral_constant<int, 2>{});
    else if (pi <= 3) run(std::integral_constant<int, 3>{});
    else run(std::integral_constant<int, MAXI>{});
    if (prof) {
      prof->t_end = grp_clock();
      prof->polls = spins + 1;
      prof->rt_end = __builtin_amdgcn_s_memrealtime();
    }
  }
  __syncthreads();
  // 3. member-order sums
  if (DTP_GRP_SAME_XCD && !plain && !dead) {  // every member on this XCD: plain stores from the next exchange on
    bool same = true;
    for (int r = 0; r < c.GR; ++r)
      if (r != c.k) same = same && __float_as_uint(peer[r * PS + P + 1]) == xcc;
    plain = same;
  }
  float acc[NPT], lacc = 0.f;
#pragma unroll
  for (int k = 0; k < NPT; ++k) acc[k] = 0.f;
  const int p0 = NPT * tid < P ? NPT * tid : 0;
  for (int r = 0; r < c.GR; ++r) {
    const float* row = peer + r * PS;
    const bool me = r == c.k;
#pragma unroll
    for (int k = 0; k < NPT; ++k) acc[k] += me ? g[k] : row[p0 + k];
    lacc += me ? loss : row[P];
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) g[k] = acc[k];
  return lacc;
}

#ifndef DTP_GRP_SHORT
// 1: drop the XCC id from the payload once plain (grp_allreduce_split3).  Measured slower
// (toy 3.43 vs 3.35, CE head 3.96 vs 3.93 us/step, profiles/r5_exchange/short/): a second
// instance of the exchange costs more than the granule it saves
#define DTP_GRP_SHORT 0
#endif

// NG granules per member: the full payload (gradients, loss, XCC id) until every member is
// known to share this XCD (plain), then without the XCC id, which has done its job: (P + 1)
// floats (the CE head's 383 gradients + loss: 128 granules, 2 poll items per lane instead of 3)
template <int P, int NPT, int NTHREADS, class OverlapFn>
DTP_DEV float grp_allreduce_split3(const GrpCtx& c, int model, float (&g)[NPT], float loss, unsigned epoch, int tid,
                                   bool& dead, float* __restrict__ lds, unsigned xcc, bool& plain, GrpProf* prof,
                                   OverlapFn ov) {
  constexpr int NGF = grp_ng3(P), NGS = (P + 1 + 2) / 3;
  if (DTP_GRP_SAME_XCD && DTP_GRP_SHORT && NGS < NGF && plain)
    return grp_allreduce_split3_ng<P, NPT, NTHREADS, NGS>(c, model, g, loss, epoch, tid, dead, lds, xcc, plain, prof, ov);
  return grp_allreduce_split3_ng<P, NPT, NTHREADS, NGF>(c, model, g, loss, epoch, tid, dead, lds, xcc, plain, prof, ov);
}

#ifndef DTP_GRP_DIRECT3
// 1: the 3-float exchange publishes straight from the per-wave dW tiles (grp_allreduce_split3d):
// no staging pass, no staging barrier.  Measured slower: 3.50 vs 3.35-3.36 us/step
// (profiles/r5_exchange/direct3/): the publish leaves ~300 cycles earlier, but two poller
// waves with 3 items per lane end later than three with 2
#define DTP_GRP_DIRECT3 0
#endif

// The 3-float exchange without the staging pass.  Right after the tile-park barrier, lane q
// of the first ceil(NG / 64) waves forms granule q itself (pub3(q): the wave-order sums of
// its three payload floats, straight from the parked tiles) and stores it; the other waves
// form their own parameters' sums meanwhile (own()), then poll after the publisher-first
// barrier while the publishers form theirs.  Same member-order sums as grp_allreduce_split3,
// so the same bits on every member -- as long as pub3 and own sum the waves in the same order.
template <int P, int NPT, int NTHREADS, class Pub3Fn, class OwnFn>
DTP_DEV float grp_allreduce_split3d(const GrpCtx& c, int model, float (&g)[NPT], const float& loss, unsigned epoch,
                                    int tid, bool& dead, float* __restrict__ lds, unsigned xcc, bool& plain,
                                    GrpProf* prof, Pub3Fn pub3, OwnFn own) {
  constexpr int NG = grp_ng3(P), PS = grp_ps3(P);
  constexpr int NPUB = ((NG + kWave - 1) / kWave) * kWave;  // publisher lanes (whole waves)
  constexpr int NPOLL = NTHREADS - NPUB;                    // poller lanes
  constexpr int slot = grp_slot16(P, NPT);
  static_assert(NG <= slot, "a member's 3-float granules fit its slot of the exchange buffer");
  static_assert(NPOLL >= kWave, "at least one poller wave");
  float* const peer = lds;  // peer[r * PS + i]: member r's float i (this member's row unused)
  const size_t base = (size_t)((int)(epoch & 1u) * c.n_models + model) * c.GR;
  const __amdgpu_buffer_rsrc_t rs = xgmi_rsrc(c.buf);
  if (tid < NPUB) {
    if (tid < NG) {
      float v[3];
      pub3(tid, v);
      const uint32_t x0 = __float_as_uint(v[0]), x1 = __float_as_uint(v[1]), x2 = __float_as_uint(v[2]);
      const u32x4 qq = {epoch ^ grp_hash3(x0, x1, x2), x0, x1, x2};
      const int off = (int)(((base + c.k) * slot + tid) * 16);
      if (DTP_GRP_SAME_XCD && plain) __builtin_amdgcn_raw_buffer_store_b128(qq, rs, off, 0, 0);
      else __builtin_amdgcn_raw_buffer_store_b128(qq, rs, off, 0, DTP_GRP_ST_AUX);
    }
    if (prof) {
      prof->t_pub = grp_clock();
      prof->rt_pub = __builtin_amdgcn_s_memrealtime();
    }
  } else {
    own();
  }
  if (DTP_GRP_PUB_FIRST) __syncthreads();
  if (tid >= NPUB) {
    const int pl = tid - NPUB;
    const int total = (c.GR - 1) * NG;
    unsigned long long deadline = 0;
    unsigned spins = 0;
    if (prof) prof->t_pub = grp_clock();
    auto expired = [&]() {
      if ((++spins & 63u) != 0u) return false;
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      if (!deadline) {
        deadline = now + (unsigned long long)(c.timeout_us > 0 ? c.timeout_us : 2000000) * 100ull;
      } else if (now > deadline) {
        if (c.status) {
          atomicExch(&c.status[0], 1);
          atomicExch(&c.status[1], (int)epoch);
        }
        return true;
      }
      return false;
    };
    auto run = [&](auto PIC) {
      constexpr int PI = decltype(PIC)::value;
      int off[PI], dst[PI];
      uint32_t pending = 0u;
#pragma unroll
      for (int j = 0; j < PI; ++j) {
        const int i = pl + j * NPOLL;
        const int ri = i / NG, q = i - ri * NG;
        const int r = ri < c.k ? ri : ri + 1;
        const bool in = i < total;
        off[j] = in ? (int)(((base + r) * slot + q) * 16) : 0;
        dst[j] = r * PS + 3 * q;
        if (in) pending |= 1u << j;
      }
      while (pending && !dead) {
        u32x4 x[PI];
        asm volatile("" ::: "memory");  // a poll is never merged with, or hoisted above, an earlier one
#pragma unroll
        for (int j = 0; j < PI; ++j) x[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off[j], 0, DTP_GRP_LD_AUX);
#pragma unroll
        for (int j = 0; j < PI; ++j) {
          if (((pending >> j) & 1u) && (x[j].x ^ grp_hash3(x[j].y, x[j].z, x[j].w)) == epoch) {
            float* d = peer + dst[j];
            d[0] = __uint_as_float(x[j].y);
            d[1] = __uint_as_float(x[j].z);
            d[2] = __uint_as_float(x[j].w);
            pending &= ~(1u << j);
          }
        }
        if (prof && spins == 0) prof->t_first = grp_clock();
        if (pending && expired()) dead = true;
      }
    };
    constexpr int MAXI = ((kGrpMax - 1) * NG + NPOLL - 1) / NPOLL;
    const int pi = (total + NPOLL - 1) / NPOLL;
    if (pi <= 1) run(std::integral_constant<int, 1>{});
    else if (pi <= 2) run(std::integral_constant<int, 2>{});
    else if (pi <= 3) run(std::integral_constant<int, 3>{});
    else if (pi <= 4) run(std::integral_constant<int, 4>{});
    else run(std::integral_constant<int, MAXI>{});
    if (prof) {
      prof->t_end = grp_clock();
      prof->polls = spins + 1;
      prof->rt_end = __builtin_amdgcn_s_memrealtime();
    }
  } else {
    own();
  }
  __syncthreads();
  if (DTP_GRP_SAME_XCD && !plain && !dead) {  // every member on this XCD: plain stores from the next exchange on
    bool same = true;
    for (int r = 0; r < c.GR; ++r)
      if (r != c.k) same = same && __float_as_uint(peer[r * PS + P + 1]) == xcc;
    plain = same;
  }
  float acc[NPT], lacc = 0.f;
#pragma unroll
  for (int k = 0; k < NPT; ++k) acc[k] = 0.f;
  const int p0 = NPT * tid < P ? NPT * tid : 0;
  for (int r = 0; r < c.GR; ++r) {
    const float* row = peer + r * PS;
    const bool me = r == c.k;
#pragma unroll
    for (int k = 0; k < NPT; ++k) acc[k] += me ? g[k] : row[p0 + k];
    lacc += me ? loss : row[P];
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) g[k] = acc[k];
  return lacc;
}

}  // namespace dtp
