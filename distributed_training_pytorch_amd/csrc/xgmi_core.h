// In-kernel one-shot all-reduce over xGMI (MI355X: 8 GPUs, fully connected,
// 7 point-to-point links per GPU).
//
// Protocol (the "data is the flag" granule form; cdna_hip_programming.md §6
// Guideline 16 recipe R2, extended to the system scope):
//   * every rank owns a receive buffer in fine-grained, uncached device memory
//     (hipExtMallocWithFlags(hipDeviceMallocUncached)), IPC-mapped into every
//     other rank;  layout [parity 2][model][src rank][slot] of 16-byte granules;
//   * a granule is {tag = exchange epoch, two fp32 values, check word}, written
//     by ONE 16-byte system-scope store; it needs no separate flag or fence: the
//     consumer polls each granule until its tag equals the epoch it expects and
//     its check word matches (a torn granule fails the check and is re-polled,
//     up to a 2^-32 collision of the hashed check word);
//   * PUSH: each rank stores its slot into every peer's buffer (posted xGMI
//     writes over all 7 links in parallel), then reads only its LOCAL buffer
//     (its own contribution stays in registers);
//   * two parities: a fast rank can be at most one exchange ahead of a slow one
//     (it cannot finish exchange e+1 before the slow rank published e+1), so
//     exchange e+1 never overwrites slots still being read for exchange e;
//   * every rank sums the W slots in rank order 0..W-1 -> bitwise identical
//     results on all ranks (DDP replica consistency by construction);
//   * spins are bounded (s_memrealtime, 100 MHz); a timeout sets status[0] and
//     status[1] = epoch and the step continues, so a wedged peer can never hang
//     the GPU; the host checks the status word and raises.
#pragma once
#include "dtp_api.h"
#include "dtp_common.h"

namespace dtp {

DTP_DEV unsigned long long pack_granule(unsigned epoch, float v) {
  return ((unsigned long long)epoch << 32) | (unsigned long long)__float_as_uint(v);
}

DTP_DEV void store_granule_sys(unsigned long long* p, unsigned long long g) {
  __hip_atomic_store(p, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

DTP_DEV unsigned long long load_granule_sys(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// largest world the in-kernel exchange serves (one node: 8 GPUs, 7 xGMI links each)
constexpr int kXgmiMaxWorld = 8;

#ifndef DTP_XGMI_PIPE_POLL
// 1: software-pipelined polls (next poll in flight while the previous one is checked).
// Measured slower in the one-GPU rehearsal (2 ranks 7.6 vs 6.6 us/step, 8 ranks 12.4 vs
// 10.0; profiles/r2_s3/ab_poll.txt), so the default is the plain poll-wait-check-sleep loop.
#define DTP_XGMI_PIPE_POLL 0
#endif

// ---- fused-step exchange: 16-byte granules -----------------------------------
// The fused train step owns its parameters in blocks: thread t holds parameters
// NPT*t .. NPT*t + NPT-1 (P = total).  Each thread publishes its NPT gradient values
// as ceil(NPT/2) granules of 16 bytes {epoch, v0, v1, check}; the global mean loss
// rides in one more granule (thread xgmi_loss_tid).  A granule is written by ONE
// 16-byte system-scope store and accepted only when its tag equals the expected
// epoch AND its hashed check word matches the payload, so a torn granule (a 16-byte
// store landing as two halves) fails the check and is re-polled (2^-32 collisions aside).
// Half the transactions of one 8-byte {epoch, value} granule per value, and a rank's
// own contribution never leaves its registers.  (Splitting the workgroup into
// sender and receiver waves, so no poll waits behind the wave's own remote stores,
// measured slower: two more barriers; branch exp/xgmi-split.)
template <int NPT>
DTP_HD constexpr int xgmi_gpt() { return (NPT + 1) / 2; }  // granules per thread
DTP_HD constexpr int xgmi_nthr(int P, int npt) { return (P + npt - 1) / npt; }
template <int NPT>
DTP_HD constexpr int xgmi_loss_tid(int P, int nthreads) {
  return xgmi_nthr(P, NPT) < nthreads ? xgmi_nthr(P, NPT) : 0;
}
// granules per (parity, model, source rank) slot, rounded to 64 bytes
DTP_HD constexpr int xgmi_slot16(int P, int npt) { return (xgmi_nthr(P, npt) * ((npt + 1) / 2) + 1 + 3) & ~3; }

// Check word of a granule: a NONLINEAR mix of tag and payload.  A linear (XOR) check
// accepts a tear {epoch e, v0 new | v1, check from exchange e-2} whenever
// v0_new ^ v0_old == e ^ (e-2), a small low-mantissa pattern; through two hash32
// rounds a tear passes only by a 2^-32 collision.  (A few VALU ops per granule.)
DTP_DEV uint32_t xgmi_check(uint32_t e, uint32_t a, uint32_t b) {
  return hash32(e ^ hash32(a ^ ((b << 13) | (b >> 19)) ^ 0x9E3779B9u));
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSysCoherent = 17;  // buffer cache policy sc0 | sc1: system scope, no cache allocation

DTP_DEV __amdgpu_buffer_rsrc_t xgmi_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// Who takes part in one exchange: every rank's receive buffer (peer-mapped), this
// rank's place, the sticky status word and the spin bound.  The fused train step
// builds it from its DtpTrainArgs; the layer-split stage kernels (split_train.hip)
// use one per pipeline stage (the stage's gradient reduced over the ranks).
struct XgmiCtx {
  float* const* peers;
  int* status;
  int world, rank, n_models, timeout_us;
};

// waited (nullable, 2 words): [0] += s_memrealtime ticks (100 MHz) from this thread's last
// publish store issued to its last granule accepted, [1] += ticks from its first to its last
// publish store issued -- the exchange-wait and publish diagnostics of the bench (status
// words [4..14), written back once per launch by the caller)
// GR > 1 (the split-batch step, grp_core.h): every rank runs the step on GR workgroups per
// model, and the exchange is ONE flat all-reduce over V = W GR virtual members -- member k
// of rank R is slot R GR + k of every receive buffer, stored once into each rank's buffer
// (its own rank's too: the other local members read it there), so the on-chip partial sums
// and the cross-GPU sum cost one hop, not two.  Sums run in slot order (rank-major).
template <int NPT, int NTHREADS = kBlock>
// dead_io (nullable): the caller's sticky "an exchange timed out" flag, read from the status
// word ONCE per launch (a status load here would be a vector load behind the publish
// stores: its vmcnt wait would hold the first poll until every store was acknowledged)
DTP_DEV float xgmi_allreduce_slots(const XgmiCtx& a, int model, int P, float (&g)[NPT], float loss, unsigned epoch,
                                   int tid, unsigned long long* waited = nullptr, int GR = 1, int gk = 0,
                                   bool* dead_io = nullptr) {
  constexpr int GPT = xgmi_gpt<NPT>();
  const int W = a.world * GR, R = a.rank * GR + gk;  // virtual members (slots) and this member's slot
  const int slot = xgmi_slot16(P, NPT);
  const int nthr = xgmi_nthr(P, NPT);
  const int ltid = xgmi_loss_tid<NPT>(P, NTHREADS);
  const size_t base = (size_t)((int)(epoch & 1u) * a.n_models + model) * W;
  // this thread's granules: its gradient blocks (threads < nthr) and the loss (ltid)
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
  auto gidx = [&](int k) { return k < GPT ? tid * GPT + k : nthr * GPT; };  // granule index in a slot
  auto mine_k = [&](int k) { return k < GPT ? has_g : has_l; };
  const unsigned long long t_pub0 = waited ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // publish to every rank that has a reader of this slot (posted xGMI writes; our own
  // contribution stays in registers)
  for (int r = 0; r < a.world; ++r) {
    if (r == a.rank && GR == 1) continue;
    const __amdgpu_buffer_rsrc_t rs = xgmi_rsrc(a.peers[r]);
#pragma unroll
    for (int k = 0; k <= GPT; ++k) {
      if (!mine_k(k)) continue;
      const uint32_t x0 = __float_as_uint(v[k][0]), x1 = __float_as_uint(v[k][1]);
      const u32x4 q = {epoch, x0, x1, xgmi_check(epoch, x0, x1)};
      __builtin_amdgcn_raw_buffer_store_b128(q, rs, (int)(((base + R) * slot + gidx(k)) * 16), 0, kSysCoherent);
    }
  }
  // consume every peer's granules from our local buffer: all pending ones requested
  // at once, only the missing ones re-polled; bounded by the deadline
  const __amdgpu_buffer_rsrc_t ms = xgmi_rsrc(a.peers[a.rank]);
  const unsigned long long t_pub = __builtin_amdgcn_s_memrealtime();
  const unsigned long long deadline = t_pub + (unsigned long long)(a.timeout_us > 0 ? a.timeout_us : 2000000) * 100ull;
  bool dead = dead_io ? *dead_io
                      : (a.status ? (__hip_atomic_load(&a.status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
                                  : false);
  float val[kXgmiMaxWorld][GPT + 1][2];
  static_assert(kXgmiMaxWorld * (GPT + 1) <= 64, "pending mask holds every (rank, granule) pair");
  uint64_t pending = 0ull;
#pragma unroll
  for (int r = 0; r < kXgmiMaxWorld; ++r) {
#pragma unroll
    for (int k = 0; k <= GPT; ++k) {
      val[r][k][0] = (r == R) ? v[k][0] : 0.f;
      val[r][k][1] = (r == R) ? v[k][1] : 0.f;
      if (r < W && r != R && mine_k(k)) pending |= 1ull << (r * (GPT + 1) + k);
    }
  }
  // one poll: the pending granules requested at once (absent ones read as zero)
  auto issue = [&](u32x4 (&x)[kXgmiMaxWorld][GPT + 1], uint64_t pend) {
    // compiler-only memory clobber (no instruction, no wait): a poll is never merged
    // with, or hoisted above, an earlier poll of the same granules
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = 0; r < kXgmiMaxWorld; ++r) {
#pragma unroll
      for (int k = 0; k <= GPT; ++k) {
        x[r][k] = u32x4{0u, 0u, 0u, 0u};
        if ((pend >> (r * (GPT + 1) + k)) & 1ull)
          x[r][k] = __builtin_amdgcn_raw_buffer_load_b128(ms, (int)(((base + r) * slot + gidx(k)) * 16), 0,
                                                          kSysCoherent);
      }
    }
  };
  // accept every still-pending granule of a poll whose tag and check word match
  auto consume = [&](const u32x4 (&x)[kXgmiMaxWorld][GPT + 1]) {
#pragma unroll
    for (int r = 0; r < kXgmiMaxWorld; ++r) {
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
  };
  auto expired = [&]() {
    if (__builtin_amdgcn_s_memrealtime() <= deadline) return false;
    if (a.status) {
      atomicExch(&a.status[0], 1);
      atomicExch(&a.status[1], (int)epoch);
    }
    return true;
  };
#if DTP_XGMI_PIPE_POLL
  // Software-pipelined polling: the next poll is in flight while the previous one is
  // checked (the compiler's vmcnt waits only for the older loads), so a granule is
  // seen about one memory round trip after it lands instead of up to two.  A poll
  // issued for a granule that an older poll already accepted is simply ignored.
  if (pending && !dead) {
    u32x4 xa[kXgmiMaxWorld][GPT + 1], xb[kXgmiMaxWorld][GPT + 1];
    issue(xa, pending);
    while (true) {
      issue(xb, pending);
      consume(xa);
      if (!pending) break;
      if (expired()) {
        dead = true;
        break;
      }
      issue(xa, pending);
      consume(xb);
      if (!pending) break;
      if (expired()) {
        dead = true;
        break;
      }
    }
  }
#else
  while (pending && !dead) {
    u32x4 x[kXgmiMaxWorld][GPT + 1];
    issue(x, pending);
    consume(x);
    if (!pending) break;
    if (expired()) {
      dead = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#endif
  if (waited) {
    waited[0] += __builtin_amdgcn_s_memrealtime() - t_pub;
    waited[1] += t_pub - t_pub0;
  }
  if (dead_io) *dead_io = dead;
  // sum in rank order 0..W-1 (bitwise identical on every rank; absent ranks add +0)
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < kXgmiMaxWorld; ++r) acc += val[r][k / 2][k & 1];
    g[k] = acc;
  }
  float lacc = 0.f;
#pragma unroll
  for (int r = 0; r < kXgmiMaxWorld; ++r) lacc += val[r][GPT][0];
  return lacc;
}

#ifndef DTP_XGMI_SPLIT
// 1: the fused steps' xGMI exchange with publisher / poller waves (xgmi_allreduce_split).
// Off: in the one-GPU multi-rank rehearsal it measured slower (W = 2 / 4 / 8: 5.65 / 6.58 /
// 9.00 vs 5.60 / 6.40 / 8.04 us/step, profiles/r5_exchange/), the single publisher wave
// issuing (W - 1) x 187 stores at W = 8.  The on-chip split-batch exchange keeps its split
// (grp_core.h), where it measured faster.
#define DTP_XGMI_SPLIT 0
#endif
#ifndef DTP_XGMI_PUB_WAVES
#define DTP_XGMI_PUB_WAVES 1  // waves that publish (the rest poll)
#endif

// LDS of the split exchange: this member's payloads [slot], then every virtual member's [8][slot]
template <int P, int NPT>
DTP_HD constexpr int xgmi_split_lds_f2() {
  return (1 + kXgmiMaxWorld) * xgmi_slot16(P, NPT);
}

// The same all-reduce with the roles split over the waves, as grp_allreduce_split
// (grp_core.h): gfx9 counts loads and stores in ONE in-order vmcnt, so a thread that polls
// right after its own publish stores cannot consume its first poll before those stores --
// posted xGMI writes to every peer -- are acknowledged.  Here the first DTP_XGMI_PUB_WAVES
// waves publish every granule of this (virtual) member to every rank that reads it, the
// other waves poll, and the payloads meet in LDS (two barriers).  Sums run in slot order, so
// the result is bitwise that of xgmi_allreduce_slots.  waited: the polling thread's wait
// (publish -> last granule accepted, s_memrealtime ticks), for the bench diagnostic.
template <int P, int NPT, int NTHREADS>
DTP_DEV float xgmi_allreduce_split(const XgmiCtx& a, int model, float (&g)[NPT], float loss, unsigned epoch, int tid,
                                   float2* __restrict__ pub, float2* __restrict__ peer, bool& dead,
                                   unsigned long long* waited = nullptr, int GR = 1, int gk = 0) {
  constexpr int GPT = xgmi_gpt<NPT>();
  constexpr int NPUB = kWave * DTP_XGMI_PUB_WAVES;          // publisher lanes
  constexpr int NPOLL = NTHREADS - NPUB;                     // poller lanes
  static_assert(NPOLL >= kWave, "at least one poller wave");
  constexpr int slot = xgmi_slot16(P, NPT);
  constexpr int nthr = xgmi_nthr(P, NPT);
  constexpr int ng = nthr * GPT + 1;                         // granules of a member: gradients + the loss
  constexpr int ltid = xgmi_loss_tid<NPT>(P, NTHREADS);
  const int V = a.world * GR, R = a.rank * GR + gk;          // virtual members (slots), this member's slot
  const size_t base = (size_t)((int)(epoch & 1u) * a.n_models + model) * V;
  const bool has_g = tid < nthr;
#pragma unroll
  for (int k = 0; k < GPT; ++k)
    if (has_g) pub[tid * GPT + k] = make_float2(2 * k < NPT ? g[2 * k] : 0.f, 2 * k + 1 < NPT ? g[2 * k + 1] : 0.f);
  if (tid == ltid) pub[nthr * GPT] = make_float2(loss, 0.f);
  __syncthreads();
  if (tid < NPUB) {
    // publish: every granule once into every rank's buffer that has a reader of this slot
    // (this rank's own buffer too when other members of the rank read it)
    for (int r = 0; r < a.world; ++r) {
      if (r == a.rank && GR == 1) continue;
      const __amdgpu_buffer_rsrc_t rs = xgmi_rsrc(a.peers[r]);
      for (int q = tid; q < ng; q += NPUB) {
        const float2 v = pub[q];
        const uint32_t x0 = __float_as_uint(v.x), x1 = __float_as_uint(v.y);
        const u32x4 qq = {epoch, x0, x1, xgmi_check(epoch, x0, x1)};
        __builtin_amdgcn_raw_buffer_store_b128(qq, rs, (int)(((base + R) * slot + q) * 16), 0, kSysCoherent);
      }
    }
  } else {
    // poll the other V - 1 slots of the local buffer: item i = (slot index i / ng, granule
    // i % ng), at most MAXI per lane, all requested at once, only the missing ones re-polled
    constexpr int MAXI = ((kXgmiMaxWorld - 1) * ng + NPOLL - 1) / NPOLL;
    static_assert(MAXI <= 32, "pending mask");
    const __amdgpu_buffer_rsrc_t ms = xgmi_rsrc(a.peers[a.rank]);
    const int pl = tid - NPUB;
    const int total = (V - 1) * ng;
    int off[MAXI], dst[MAXI];
    uint32_t pending = 0u;
#pragma unroll
    for (int j = 0; j < MAXI; ++j) {
      const int i = pl + j * NPOLL;
      const int vi = i / ng, q = i - vi * ng;
      const int v = vi < R ? vi : vi + 1;
      off[j] = (int)(((base + v) * slot + q) * 16);
      dst[j] = v * slot + q;
      if (i < total) pending |= 1u << j;
    }
    const unsigned long long t_pub = __builtin_amdgcn_s_memrealtime();
    const unsigned long long deadline = t_pub + (unsigned long long)(a.timeout_us > 0 ? a.timeout_us : 2000000) * 100ull;
    unsigned spins = 0;
    while (pending && !dead) {
      u32x4 x[MAXI];
      asm volatile("" ::: "memory");  // a poll is never merged with, or hoisted above, an earlier one
#pragma unroll
      for (int j = 0; j < MAXI; ++j) {
        x[j] = u32x4{0u, 0u, 0u, 0u};
        if ((pending >> j) & 1u) x[j] = __builtin_amdgcn_raw_buffer_load_b128(ms, off[j], 0, kSysCoherent);
      }
#pragma unroll
      for (int j = 0; j < MAXI; ++j) {
        if (((pending >> j) & 1u) && x[j].x == epoch && x[j].w == xgmi_check(epoch, x[j].y, x[j].z)) {
          peer[dst[j]] = make_float2(__uint_as_float(x[j].y), __uint_as_float(x[j].z));
          pending &= ~(1u << j);
        }
      }
      if (!pending) break;
      if ((++spins & 15u) == 0u && __builtin_amdgcn_s_memrealtime() > deadline) {
        if (a.status) {
          atomicExch(&a.status[0], 1);
          atomicExch(&a.status[1], (int)epoch);
        }
        dead = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (waited) waited[0] += __builtin_amdgcn_s_memrealtime() - t_pub;
  }
  __syncthreads();
  // slot-order sums (absent slots add nothing; a timed-out peer's stale values are flagged)
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
  for (int v = 0; v < V; ++v) {
#pragma unroll
    for (int k = 0; k <= GPT; ++k) {
      const int q = k < GPT ? gq0 + k : nthr * GPT;
      const float2 pv = v == R ? make_float2(own[k][0], own[k][1]) : peer[v * slot + q];
      acc[k][0] += pv.x;
      acc[k][1] += pv.y;
    }
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) g[k] = acc[k / 2][k & 1];
  return acc[GPT][0];
}

#ifndef DTP_XGMI_G3
// 1: the several-lanes steps (4 waves) run the cross-GPU exchange on 3-float granules with a
// destination-dealt publish (xgmi_allreduce_g3); 0: the 2-float owner-thread form above
#define DTP_XGMI_G3 1
#endif
#ifndef DTP_XGMI_G3_PUBW
// xgmi_allreduce_g3 roles: 0 = every wave publishes its dealt destinations, then polls;
// n > 0 = waves 0..n-1 publish every destination, the other waves poll
#define DTP_XGMI_G3_PUBW 0
#endif
#ifndef DTP_XGMI_G3_SLEEP
#define DTP_XGMI_G3_SLEEP 0  // s_sleep units between two polls of xgmi_allreduce_g3 (0: none)
#endif

// 3-float granules of a member's cross-GPU payload: the P gradients and the loss
DTP_HD constexpr int xgmi_ng3(int P) { return (P + 1 + 2) / 3; }
// LDS floats per member row of xgmi_allreduce_g3 (a float4 multiple)
DTP_HD constexpr int xgmi_ps3(int P) { return (3 * xgmi_ng3(P) + 3) & ~3; }
// LDS floats of xgmi_allreduce_g3: this member's row, then one row per virtual member
DTP_HD constexpr int xgmi_g3_lds_floats(int P) { return (1 + kXgmiMaxWorld) * xgmi_ps3(P); }

// Tag of a 3-float cross-GPU granule {epoch ^ h(v0, v1, v2), v0, v1, v2}: nonlinear in the
// payload (two hash32 rounds), so a granule torn across an xGMI link -- new and old halves
// of a slot two exchanges apart -- passes only on a 2^-32 collision.
DTP_DEV uint32_t xgmi_hash3(uint32_t a, uint32_t b, uint32_t c) {
  return hash32(a ^ hash32(b ^ ((c << 13) | (c >> 19)) ^ 0x9E3779B9u));
}

// The cross-GPU all-reduce on 3-float granules (round 6; the on-chip split exchange's form,
// grp_core.h:grp_allreduce_split3, carried to the system scope):
//   * the owners stage the member's payload in LDS as one flat row (gradients 0..P-1, the
//     loss at P); granule q = floats [3q, 3q + 3) as {epoch ^ xgmi_hash3(v), v}: 124 granules
//     for the toy model instead of 187 two-float ones;
//   * publish: the destination ranks (every rank with a reader of this slot -- the own
//     rank too when other local members read it, GR > 1) are dealt to the waves, d-th
//     destination to wave d % NPW; a wave stores all NG granules of its destination
//     (2 coalesced 16-byte stores per lane, a wave-uniform buffer resource), so no lane
//     issues more than 2 ceil(D / NPW) stores (W = 8: 4, was 7 per owner thread);
//   * poll: items (virtual member v != R, granule q) spread over the poller lanes (W = 8:
//     <= 4 per lane), every still-missing item re-requested each round, accepted granules
//     parked in LDS;
//   * one barrier, then every thread sums its parameters over the slots in order 0..V-1
//     (its own value from registers): the same bits on every rank, and the same bits as
//     xgmi_allreduce_slots (identical add order).
// lds: xgmi_g3_lds_floats(P) floats.  Spins bounded (status word, dead flag), as above.
template <int P, int NPT, int NTHREADS>
DTP_DEV float xgmi_allreduce_g3(const XgmiCtx& a, int model, float (&g)[NPT], float loss, unsigned epoch, int tid,
                                float* __restrict__ lds, bool& dead, unsigned long long* waited = nullptr, int GR = 1,
                                int gk = 0) {
  constexpr int NG = xgmi_ng3(P), PS = xgmi_ps3(P);
  constexpr int NW = NTHREADS / kWave;
  constexpr int NPW = DTP_XGMI_G3_PUBW > 0 ? DTP_XGMI_G3_PUBW : NW;  // publisher waves
  constexpr int NPOLL = DTP_XGMI_G3_PUBW > 0 ? NTHREADS - kWave * DTP_XGMI_G3_PUBW : NTHREADS;
  constexpr int P0 = DTP_XGMI_G3_PUBW > 0 ? kWave * DTP_XGMI_G3_PUBW : 0;  // first poller lane
  constexpr int slot = xgmi_slot16(P, NPT);
  constexpr int MAXJ = (NG + kWave - 1) / kWave;  // granules per publisher lane and destination
  static_assert(NG <= slot, "a member's 3-float granules fit its slot of the receive buffer");
  static_assert(NPW <= NW && NPOLL >= kWave, "publisher and poller waves");
  float* const pub = lds;
  float* const peer = lds + PS;  // peer[v * PS + i]: virtual member v's float i
  const int V = a.world * GR, R = a.rank * GR + gk;
  const size_t base = (size_t)((int)(epoch & 1u) * a.n_models + model) * V;
  const int wave = tid / kWave, lane = tid - (tid / kWave) * kWave;
  // 1. the payload into LDS
#pragma unroll
  for (int k = 0; k < NPT; ++k)
    if (NPT * tid + k < P) pub[NPT * tid + k] = g[k];
  if (tid == 0) {
    pub[P] = loss;
#pragma unroll
    for (int i = P + 1; i < 3 * NG; ++i) pub[i] = 0.f;
  }
  __syncthreads();
  const unsigned long long t_pub0 = waited ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // 2. publish: this wave's dealt destinations (the ranks other than this one first, in
  // ring order from rank + 1, then this rank's own buffer when GR > 1)
  if (wave < NPW) {
    u32x4 gq[MAXJ];
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int q = lane + j * kWave < NG ? lane + j * kWave : NG - 1;
      const uint32_t x0 = __float_as_uint(pub[3 * q]), x1 = __float_as_uint(pub[3 * q + 1]),
                     x2 = __float_as_uint(pub[3 * q + 2]);
      gq[j] = u32x4{epoch ^ xgmi_hash3(x0, x1, x2), x0, x1, x2};
    }
    const int D = GR > 1 ? a.world : a.world - 1;
    for (int di = wave; di < D; di += NPW) {
      int d = a.rank + 1 + di;
      d = d >= a.world ? d - a.world : d;  // di = world - 1 (GR > 1 only): this rank
      const __amdgpu_buffer_rsrc_t rs = xgmi_rsrc(a.peers[d]);
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) {
        const int q = lane + j * kWave;
        if (q < NG)
          __builtin_amdgcn_raw_buffer_store_b128(gq[j], rs, (int)(((base + R) * slot + q) * 16), 0, kSysCoherent);
      }
    }
  }
  const unsigned long long t_pub = waited ? __builtin_amdgcn_s_memrealtime() : 0ull;
  if (waited && wave < NPW) waited[1] += t_pub - t_pub0;
  // 3. poll the other V - 1 slots of the local buffer
  if (tid >= P0) {
    const __amdgpu_buffer_rsrc_t ms = xgmi_rsrc(a.peers[a.rank]);
    const int pl = tid - P0;
    const int total = (V - 1) * NG;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long deadline = t0 + (unsigned long long)(a.timeout_us > 0 ? a.timeout_us : 2000000) * 100ull;
    unsigned spins = 0;
    auto run = [&](auto PIC) {
      constexpr int PI = decltype(PIC)::value;
      int off[PI], dst[PI];
      uint32_t pending = 0u;
#pragma unroll
      for (int j = 0; j < PI; ++j) {
        const int i = pl + j * NPOLL;
        const int vi = i / NG, q = i - vi * NG;
        const int v = vi < R ? vi : vi + 1;
        const bool in = i < total;
        off[j] = in ? (int)(((base + v) * slot + q) * 16) : 0;
        dst[j] = v * PS + 3 * q;
        if (in) pending |= 1u << j;
      }
      while (pending && !dead) {
        u32x4 x[PI];
        asm volatile("" ::: "memory");  // a poll is never merged with, or hoisted above, an earlier one
#pragma unroll
        for (int j = 0; j < PI; ++j) x[j] = __builtin_amdgcn_raw_buffer_load_b128(ms, off[j], 0, kSysCoherent);
#pragma unroll
        for (int j = 0; j < PI; ++j) {
          if (((pending >> j) & 1u) && (x[j].x ^ xgmi_hash3(x[j].y, x[j].z, x[j].w)) == epoch) {
            float* d = peer + dst[j];
            d[0] = __uint_as_float(x[j].y);
            d[1] = __uint_as_float(x[j].z);
            d[2] = __uint_as_float(x[j].w);
            pending &= ~(1u << j);
          }
        }
        if (!pending) break;
        if ((++spins & 15u) == 0u && __builtin_amdgcn_s_memrealtime() > deadline) {
          if (a.status) {
            atomicExch(&a.status[0], 1);
            atomicExch(&a.status[1], (int)epoch);
          }
          dead = true;
        }
        if (DTP_XGMI_G3_SLEEP > 0) __builtin_amdgcn_s_sleep(DTP_XGMI_G3_SLEEP);
      }
      // a timed-out exchange adds +0 for what never arrived (not an earlier exchange's rows)
      if (pending) {
#pragma unroll
        for (int j = 0; j < PI; ++j)
          if ((pending >> j) & 1u) peer[dst[j]] = peer[dst[j] + 1] = peer[dst[j] + 2] = 0.f;
      }
    };
    constexpr int MAXI = ((kXgmiMaxWorld - 1) * NG + NPOLL - 1) / NPOLL;
    static_assert(MAXI <= 32, "pending mask");
    const int pi = (total + NPOLL - 1) / NPOLL;
    if (pi <= 1) run(std::integral_constant<int, 1>{});
    else if (pi <= 2) run(std::integral_constant<int, 2>{});
    else if (pi <= 4) run(std::integral_constant<int, 4 < MAXI ? 4 : MAXI>{});
    else run(std::integral_constant<int, MAXI>{});
    if (waited) waited[0] += __builtin_amdgcn_s_memrealtime() - t0;
  }
  __syncthreads();
  // 4. slot-order sums (a dead exchange's rows hold +0 where nothing arrived)
  float acc[NPT], lacc = 0.f;
#pragma unroll
  for (int k = 0; k < NPT; ++k) acc[k] = 0.f;
  const int p0 = NPT * tid < P ? NPT * tid : 0;
  for (int v = 0; v < V; ++v) {
    const float* row = peer + v * PS;
    const bool me = v == R;
#pragma unroll
    for (int k = 0; k < NPT; ++k) acc[k] += me ? g[k] : row[p0 + k];
    lacc += me ? loss : row[P];
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) g[k] = acc[k];
  return lacc;
}

template <int NPT, int NTHREADS = kBlock>
DTP_DEV float xgmi_allreduce_model(const DtpTrainArgs& a, int model, int P, float (&g)[NPT], float loss,
                                   unsigned epoch, int tid, unsigned long long* waited = nullptr, int GR = 1,
                                   int gk = 0, bool* dead_io = nullptr) {
  const XgmiCtx c{a.peers, a.status, a.smp.world, a.smp.rank, a.n_models, a.timeout_us};
  return xgmi_allreduce_slots<NPT, NTHREADS>(c, model, P, g, loss, epoch, tid, waited, GR, gk, dead_io);
}

// the fused step's exchange diagnostics in the status block, for model 0's workgroup:
// [4..6) u64 += the launch's exchange-wait ticks of its SLOWEST thread (the step cannot
// pass its closing barrier before that thread has every peer granule), [6..8) u64 +=
// the launch's exchanges; [8..10) is the per-launch max scratch; [10..12) u64 += the
// launch's publish ticks of its slowest publisher, [12..14) its max scratch.  Accumulated
// over launches; the host zeroes them around a timed region.  Called by EVERY thread of
// the workgroup at the end of the launch (contains a barrier).
DTP_DEV void xgmi_record_wait(int* status, const unsigned long long (&ticks)[2], unsigned long long n, int tid) {
  unsigned long long* w = reinterpret_cast<unsigned long long*>(status + 4);
  atomicMax(w + 2, ticks[0]);
  atomicMax(w + 4, ticks[1]);
  __syncthreads();  // every thread's max has landed (device-coherent atomics, then the barrier)
  if (tid == 0) {
    const unsigned long long m = atomicExch(w + 2, 0ull);
    const unsigned long long mp = atomicExch(w + 4, 0ull);
    atomicAdd(w, m);
    atomicAdd(w + 1, n);
    atomicAdd(w + 3, mp);
  }
}

}  // namespace dtp
