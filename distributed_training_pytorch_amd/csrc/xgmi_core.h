// In-kernel one-shot all-reduce over xGMI (MI355X: 8 GPUs, fully connected,
// 7 point-to-point links per GPU).
//
// Protocol (the "data is the flag" granule form; cdna_hip_programming.md §6
// Guideline 16 recipe R2, extended to the system scope):
//   * every rank owns a receive buffer in fine-grained, uncached device memory
//     (hipExtMallocWithFlags(hipDeviceMallocUncached)), IPC-mapped into every
//     other rank;  layout [parity 2][model][src rank][slot] of 8-byte granules;
//   * a granule is {tag = exchange epoch (32 bit), value = fp32 bits}, written by
//     ONE 8-byte system-scope store, so it can never be observed torn and needs
//     no separate flag or fence: the consumer polls each granule until its tag
//     equals the epoch it expects;
//   * PUSH: each rank stores its slot into every peer's buffer (posted xGMI
//     writes over all 7 links in parallel), then reads only its LOCAL buffer;
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

// granules per (model, src rank) slot: P gradient values + 1 loss, 64-byte rounded
DTP_HD int xgmi_slot_granules(int P) { return (P + 1 + 7) & ~7; }

template <int NPT, int NTHREADS = kBlock>
DTP_DEV float xgmi_allreduce_model(const DtpTrainArgs& a, int model, int P, float (&g)[NPT], float loss,
                                   unsigned epoch, int tid) {
  const int W = a.smp.world, R = a.smp.rank;
  const int slot = xgmi_slot_granules(P);
  const int par = (int)(epoch & 1u);
  const size_t base = (size_t)(par * a.n_models + model) * W;
  // publish our slot into every rank's buffer (our own included)
  for (int r = 0; r < W; ++r) {
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(a.peers[r]) + (base + R) * slot;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int p = tid + k * NTHREADS;
      if (p < P) store_granule_sys(dst + p, pack_granule(epoch, g[k]));
    }
    if (tid == 0) store_granule_sys(dst + P, pack_granule(epoch, loss));
  }
  // consume every rank's slot from our local buffer: every granule this thread
  // needs (W x (NPT + loss)) is requested at once and only the missing ones are
  // re-polled, so an exchange costs ONE uncached round trip once the data is
  // there, not W sequential ones; then sum in rank order 0..W-1 (bitwise
  // identical on every rank)
  const unsigned long long* mine = reinterpret_cast<const unsigned long long*>(a.peers[R]);
  const unsigned long long deadline =
      __builtin_amdgcn_s_memrealtime() + (unsigned long long)(a.timeout_us > 0 ? a.timeout_us : 2000000) * 100ull;
  // sticky failure: once any exchange of this rank timed out, later ones do not
  // wait again (a persistent launch must not multiply the timeout by its steps)
  bool dead = a.status ? (__hip_atomic_load(&a.status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) : false;
  constexpr int NG = NPT + 1;  // + the loss granule (thread 0)
  float val[kXgmiMaxWorld][NG];
  static_assert(kXgmiMaxWorld * NG <= 64, "pending mask holds every (rank, granule) pair");
  uint64_t pending = 0ull;  // bit r*NG + k: granule (r, k) still missing
#pragma unroll
  for (int r = 0; r < kXgmiMaxWorld; ++r) {
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      val[r][k] = 0.f;
      const int p = k < NPT ? tid + k * NTHREADS : P;
      const bool mine_to_read = r < W && (k < NPT ? p < P : tid == 0);
      if (mine_to_read) pending |= 1ull << (r * NG + k);
    }
  }
  while (pending && !dead) {
    unsigned long long x[kXgmiMaxWorld][NG];
#pragma unroll
    for (int r = 0; r < kXgmiMaxWorld; ++r) {
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        const int p = k < NPT ? tid + k * NTHREADS : P;
        x[r][k] = (pending >> (r * NG + k)) & 1ull ? load_granule_sys(mine + (base + r) * slot + p) : 0ull;
      }
    }
#pragma unroll
    for (int r = 0; r < kXgmiMaxWorld; ++r) {
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        if (((pending >> (r * NG + k)) & 1ull) && (unsigned)(x[r][k] >> 32) == epoch) {
          val[r][k] = __uint_as_float((unsigned)x[r][k]);
          pending &= ~(1ull << (r * NG + k));
        }
      }
    }
    if (!pending) break;
    if (__builtin_amdgcn_s_memrealtime() > deadline) {
      dead = true;
      if (a.status) {
        atomicExch(&a.status[0], 1);
        atomicExch(&a.status[1], (int)epoch);
      }
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  float lacc = 0.f;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < kXgmiMaxWorld; ++r) acc += val[r][k];  // absent ranks contribute +0.0f
    g[k] = acc;
  }
#pragma unroll
  for (int r = 0; r < kXgmiMaxWorld; ++r) lacc += val[r][NPT];
  return lacc;
}

}  // namespace dtp
