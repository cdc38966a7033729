// Stand-alone one-shot all-reduce over xGMI peer memory for small buffers
// (the FlatDDP gradient buckets of the module / Trainer engines; the fused
// train kernel has the same exchange built in, xgmi_core.h).
//
// Why not RCCL for these: a DDP bucket of the toy workloads is a few KB, where
// a ring all-reduce is pure latency (2(W-1) dependent hops + kernel launch per
// call).  Here every rank pushes its values into every peer's receive buffer in
// one wave of posted xGMI writes (all 7 links at once) and reads its LOCAL
// buffer only: one hop of latency, independent of W.
//
// Protocol = xgmi_core.h (granule {epoch tag, fp32 bits} written by one 8-byte
// system-scope store; two parities; rank-order sum; bounded spin that flags
// status[0] instead of hanging).  Layout of a rank's receive buffer:
// [parity 2][src rank W][cap] granules.  The epoch increases by one per call on
// every rank (calls are stream-ordered), so a fast rank is at most one call
// ahead of a slow one and never overwrites a parity still being read.
//
// The epoch lives in DEVICE memory, one counter per workgroup (a workgroup always
// owns the same granule range, so its counter counts exactly the calls that used
// those granules, identically on every rank): the kernel reads and advances it
// itself, so a hipGraph replay of a captured call is a new exchange -- no host
// state changes per call, and the module engine / Trainer capture their whole
// step, xGMI buckets included.
#include "dtp_api.h"
#include "dtp_common.h"

namespace dtp {

constexpr int kArThreads = 256;
constexpr int kArPerThread = 4;
constexpr int kArMaxWorld = 8;

__global__ __launch_bounds__(kArThreads) void xgmi_allreduce_kernel(float* __restrict__ data, int n, int cap,
                                                                      unsigned long long* const* __restrict__ peers,
                                                                      int world, int rank, unsigned* epochs,
                                                                      float scale, int* status, int timeout_us) {
  __shared__ unsigned s_epoch;
  if (threadIdx.x == 0) s_epoch = epochs[blockIdx.x] + 1u;
  __syncthreads();
  const unsigned epoch = s_epoch;
  const int base = (blockIdx.x * kArThreads + threadIdx.x) * kArPerThread;
  const size_t par = epoch & 1u;
  float v[kArPerThread];
#pragma unroll
  for (int k = 0; k < kArPerThread; ++k) v[k] = (base + k < n) ? data[base + k] : 0.f;
  // push: our values into slot [par][rank] of every rank's buffer (ours included)
  for (int r = 0; r < world; ++r) {
    unsigned long long* dst = peers[r] + (par * world + rank) * (size_t)cap;
#pragma unroll
    for (int k = 0; k < kArPerThread; ++k)
      if (base + k < n)
        __hip_atomic_store(dst + base + k, ((unsigned long long)epoch << 32) | __float_as_uint(v[k]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // pull: every granule this thread needs from the local buffer, all in flight
  const unsigned long long* mine = peers[rank] + par * world * (size_t)cap;
  const unsigned long long deadline =
      __builtin_amdgcn_s_memrealtime() + (unsigned long long)(timeout_us > 0 ? timeout_us : 2000000) * 100ull;
  bool dead = status ? __hip_atomic_load(&status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 : false;
  float got[kArMaxWorld][kArPerThread];
  uint32_t pending = 0u;
#pragma unroll
  for (int r = 0; r < kArMaxWorld; ++r)
#pragma unroll
    for (int k = 0; k < kArPerThread; ++k) {
      got[r][k] = 0.f;
      if (r < world && base + k < n) pending |= 1u << (r * kArPerThread + k);
    }
  while (pending && !dead) {
    unsigned long long x[kArMaxWorld][kArPerThread];
#pragma unroll
    for (int r = 0; r < kArMaxWorld; ++r)
#pragma unroll
      for (int k = 0; k < kArPerThread; ++k)
        x[r][k] = ((pending >> (r * kArPerThread + k)) & 1u)
                      ? __hip_atomic_load(const_cast<unsigned long long*>(mine + r * (size_t)cap + base + k),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                      : 0ull;
#pragma unroll
    for (int r = 0; r < kArMaxWorld; ++r)
#pragma unroll
      for (int k = 0; k < kArPerThread; ++k)
        if (((pending >> (r * kArPerThread + k)) & 1u) && (unsigned)(x[r][k] >> 32) == epoch) {
          got[r][k] = __uint_as_float((unsigned)x[r][k]);
          pending &= ~(1u << (r * kArPerThread + k));
        }
    if (!pending) break;
    if (__builtin_amdgcn_s_memrealtime() > deadline) {
      dead = true;
      if (status) {
        atomicExch(&status[0], 1);
        atomicExch(&status[1], (int)epoch);
      }
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int k = 0; k < kArPerThread; ++k) {
    if (base + k >= n) continue;
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < kArMaxWorld; ++r) s += got[r][k];  // rank order; absent ranks add +0
    data[base + k] = s * scale;
  }
  // the next call of this workgroup (a later kernel on the stream) sees the new epoch
  if (threadIdx.x == 0) epochs[blockIdx.x] = epoch;
}

}  // namespace dtp

// epochs: device counters, one per workgroup of a capacity-sized call
// (dtp_xgmi_allreduce_epoch_slots(cap)), zeroed before the first call on every rank
extern "C" int dtp_xgmi_allreduce_epoch_slots(int cap) {
  const int per_block = dtp::kArThreads * dtp::kArPerThread;
  return (cap + per_block - 1) / per_block;
}

extern "C" int dtp_xgmi_allreduce(float* data, int n, int cap, void* const* peers, int world, int rank,
                                  unsigned* epochs, float scale, int* status, int timeout_us, void* stream) {
  if (!data || !peers || !epochs || n < 0 || n > cap)
    return dtp::set_err(-1, "dtp_xgmi_allreduce: bad buffer, no epoch counters, or size > capacity");
  if (world < 1 || world > dtp::kArMaxWorld || rank < 0 || rank >= world)
    return dtp::set_err(-1, "dtp_xgmi_allreduce: world must be 1..8");
  if (n == 0) return 0;
  const int per_block = dtp::kArThreads * dtp::kArPerThread;
  hipLaunchKernelGGL(dtp::xgmi_allreduce_kernel, dim3((n + per_block - 1) / per_block), dim3(dtp::kArThreads), 0,
                     (hipStream_t)stream, data, n, cap, (unsigned long long* const*)peers, world, rank, epochs, scale,
                     status, timeout_us);
  return dtp::check_launch("xgmi_allreduce_kernel");
}
