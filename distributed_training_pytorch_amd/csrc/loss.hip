// Module-path helpers: a fused MSE loss and the Trainer's two-tensor batch gather.
//
// Fused MSE loss for the module (autograd) path: what nn.MSELoss(reduction="mean") does
// in the reference's training step (demo.py:103-104, demo_pytorch_lightning.py:27-33) as
// ONE launch forward and ONE backward, instead of torch's elementwise square + mean
// reduction forward (2 launches) and its backward.  The Trainer replays a batch's
// optimizer steps as a hipGraph, where every launch costs ~4 us whatever it does
// (profiles/r4_lightning_module/), so the launch count is the cost.
//
// forward: one workgroup of 256 threads (the toy batches are <= a few thousand
// elements); each lane sums (a - b)^2 over a grid stride, then a wave butterfly (DPP row
// and swizzle-free shuffles) and the 4 wave partials in LDS; out = sum / n.
// backward: ga = g * 2 (a - b) / n (and gb = -ga when the target needs a gradient); g is
// read on the device (no host sync in a captured graph).
#include "dtp_api.h"
#include "dtp_common.h"

namespace dtp {

__global__ __launch_bounds__(kBlock) void mse_fwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         long long n, float inv_n, float* __restrict__ out) {
  __shared__ float part[kBlock / kWave];
  const int tid = threadIdx.x;
  float s = 0.f;
  for (long long i = tid; i < n; i += kBlock) {
    const float d = a[i] - b[i];
    s = fmaf(d, d, s);
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
  if ((tid & (kWave - 1)) == 0) part[tid / kWave] = s;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kBlock / kWave; ++w) t += part[w];
    out[0] = t * inv_n;
  }
}

__global__ __launch_bounds__(kBlock) void mse_bwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         const float* __restrict__ g, long long n, float scale,
                                                         float* __restrict__ ga, float* __restrict__ gb) {
  const float gs = g[0] * scale;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long long)gridDim.x * kBlock) {
    const float d = gs * (a[i] - b[i]);
    if (ga) ga[i] = d;
    if (gb) gb[i] = -d;
  }
}

// Two predictions against ONE target (the reference's two models on the same batch,
// demo_pytorch_lightning.py:27-33: loss_X + loss_Y) in one launch: out = {mse(a1, b),
// mse(a2, b), their sum} -- the sum in the same fp32 order as torch's `loss_x + loss_y`.
__global__ __launch_bounds__(kBlock) void mse_pair_fwd_kernel(const float* __restrict__ a1, const float* __restrict__ a2,
                                                              const float* __restrict__ b, long long n, float inv_n,
                                                              float* __restrict__ o1, float* __restrict__ o2,
                                                              float* __restrict__ osum, float* __restrict__ ring,
                                                              long long* __restrict__ slot, int width) {
  __shared__ float part[2][kBlock / kWave];
  const int tid = threadIdx.x;
  float s1 = 0.f, s2 = 0.f;
  for (long long i = tid; i < n; i += kBlock) {
    const float bi = b[i];
    const float d1 = a1[i] - bi, d2 = a2[i] - bi;
    s1 = fmaf(d1, d1, s1);
    s2 = fmaf(d2, d2, s2);
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off, kWave);
    s2 += __shfl_xor(s2, off, kWave);
  }
  if ((tid & (kWave - 1)) == 0) {
    part[0][tid / kWave] = s1;
    part[1][tid / kWave] = s2;
  }
  __syncthreads();
  if (tid == 0) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int w = 0; w < kBlock / kWave; ++w) {
      t1 += part[0][w];
      t2 += part[1][w];
    }
    const float l1 = t1 * inv_n, l2 = t2 * inv_n;
    o1[0] = l1;
    o2[0] = l2;
    osum[0] = l1 + l2;
    if (ring) {  // the engine's device loss log (utils/logging.py LossRing): row[slot] = (l1, l2); slot += 1
      const long long sl = slot[0];
      ring[sl * width] = l1;
      ring[sl * width + 1] = l2;
      slot[0] = sl + 1;
    }
  }
}

// its backward: ga_k = (g_k + g_sum) 2 (a_k - b) / n for the predictions that need a
// gradient (g_k / g_sum read on the device; null = 0), gb = -(ga_1 + ga_2) when the target does
__global__ __launch_bounds__(kBlock) void mse_pair_bwd_kernel(const float* __restrict__ a1, const float* __restrict__ a2,
                                                              const float* __restrict__ b, const float* __restrict__ g1,
                                                              const float* __restrict__ g2, const float* __restrict__ gsum,
                                                              long long n, float scale, float* __restrict__ ga1,
                                                              float* __restrict__ ga2, float* __restrict__ gb) {
  const float gt = gsum ? gsum[0] : 0.f;
  const float gs1 = ((g1 ? g1[0] : 0.f) + gt) * scale;
  const float gs2 = ((g2 ? g2[0] : 0.f) + gt) * scale;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long long)gridDim.x * kBlock) {
    const float bi = b[i];
    const float d1 = gs1 * (a1[i] - bi), d2 = gs2 * (a2[i] - bi);
    if (ga1) ga1[i] = d1;
    if (ga2) ga2[i] = d2;
    if (gb) gb[i] = -(d1 + d2);
  }
}

// the Trainer's replayed batch gather: rows idx of X [nrows, dx] and Y [nrows, dy] into
// the static batch buffers in ONE launch (torch: one index_select per tensor); indices are
// clamped into range (an index past the dataset never reads out of bounds)
__global__ __launch_bounds__(kBlock) void gather_rows2_kernel(const float* __restrict__ X, int dx,
                                                              const float* __restrict__ Y, int dy,
                                                              const long long* __restrict__ idx, int n,
                                                              long long nrows, float* __restrict__ ox,
                                                              float* __restrict__ oy) {
  const int w = dx + dy;
  for (long long t = (long long)blockIdx.x * kBlock + threadIdx.x; t < (long long)n * w;
       t += (long long)gridDim.x * kBlock) {
    const int r = (int)(t / w), c = (int)(t - (long long)r * w);
    long long s = idx[r];
    s = s < 0 ? 0 : (s >= nrows ? nrows - 1 : s);
    if (c < dx) ox[(long long)r * dx + c] = X[s * dx + c];
    else oy[(long long)r * dy + (c - dx)] = Y[s * dy + (c - dx)];
  }
}

// the same gather with the batch's indices read from a device-resident epoch ring
// {cursor, indices of the whole epoch}: batch b = cursor mod steps starts at index
// b * batch, and the kernel advances the cursor itself.  A replayed step then reads a new
// batch every replay with nothing refreshed by the host (the per-batch index copy -- a
// ~3 us blit plus a gap in the replayed stream -- is gone).  ONE workgroup, so every
// thread's read of the cursor precedes the single write (the barrier orders them).
__global__ __launch_bounds__(kBlock) void gather_rows2_ring_kernel(const float* __restrict__ X, int dx,
                                                                   const float* __restrict__ Y, int dy,
                                                                   long long* __restrict__ ring, int batch, int steps,
                                                                   int n, long long nrows, float* __restrict__ ox,
                                                                   float* __restrict__ oy) {
  const long long cur = ring[0];
  const long long* __restrict__ idx = ring + 1 + (cur % steps) * (long long)batch;
  const int w = dx + dy;
  for (int t = threadIdx.x; t < n * w; t += kBlock) {
    const int r = t / w, c = t - r * w;
    long long s = idx[r];
    s = s < 0 ? 0 : (s >= nrows ? nrows - 1 : s);
    if (c < dx) ox[(long long)r * dx + c] = X[s * dx + c];
    else oy[(long long)r * dy + (c - dx)] = Y[s * dy + (c - dx)];
  }
  __syncthreads();
  if (threadIdx.x == 0) ring[0] = cur + 1;
}

// the same gather with the indices computed on the device by the engine's sampler
// (sampler.h: batch_pos + sample_index -- DistributedSampler order from the device
// permutation ring (SAMPLER_TABLE), the keyed shuffle, or the unshuffled orders) for step
// cursor[0], which the kernel advances: a replayed step draws its batch with no index
// buffer refreshed by the host at all, not even per epoch.  ONE workgroup.
__global__ __launch_bounds__(kBlock) void gather_rows2_sampler_kernel(const float* __restrict__ X, int dx,
                                                                      const float* __restrict__ Y, int dy,
                                                                      SamplerCfg smp, long long* __restrict__ cursor,
                                                                      int n, long long nrows, float* __restrict__ ox,
                                                                      float* __restrict__ oy) {
  __shared__ int sidx[kBlock * 4];
  const long long t = cursor[0];
  const BatchPos bp = batch_pos(smp, t);
  uint32_t keys[4] = {0u, 0u, 0u, 0u};
  if (smp.mode == SAMPLER_DIST_SHUFFLE) epoch_keys(smp, bp.epoch, keys);
  const int m = n < bp.size ? n : bp.size;
  for (int r = threadIdx.x; r < m; r += kBlock) {
    int s = sample_index(smp, bp, keys, r);
    s = s < 0 ? 0 : (s >= nrows ? (int)(nrows - 1) : s);
    sidx[r] = s;
  }
  __syncthreads();
  const int w = dx + dy;
  for (int i = threadIdx.x; i < m * w; i += kBlock) {
    const int r = i / w, c = i - r * w;
    const long long s = sidx[r];
    if (c < dx) ox[(long long)r * dx + c] = X[s * dx + c];
    else oy[(long long)r * dy + (c - dx)] = Y[s * dy + (c - dx)];
  }
  if (threadIdx.x == 0) cursor[0] = t + 1;  // every thread read the cursor before the barrier
}

}  // namespace dtp

extern "C" {

long long dtp_gather_ring_max_elems();

int dtp_gather_rows2_sampler(const float* X, int dx, const float* Y, int dy, const dtp::SamplerCfg* smp,
                             long long* cursor, int n, long long nrows, float* ox, float* oy, void* stream) {
  if (!X || !Y || !smp || !cursor || !ox || !oy || n <= 0 || n > 4 * dtp::kBlock || dx <= 0 || dy <= 0 ||
      nrows <= 0 || smp->batch <= 0 || smp->steps_per_epoch <= 0 || smp->n != nrows ||
      (long long)n * (dx + dy) > dtp_gather_ring_max_elems() ||
      (smp->mode == dtp::SAMPLER_TABLE && (!smp->perm || smp->perm_epochs <= 0)))
    return dtp::set_err(-1, "gather_rows2_sampler: bad arguments");
  hipLaunchKernelGGL(dtp::gather_rows2_sampler_kernel, dim3(1), dim3(dtp::kBlock), 0, (hipStream_t)stream, X, dx, Y,
                     dy, *smp, cursor, n, nrows, ox, oy);
  return dtp::check_launch("gather_rows2_sampler_kernel");
}

// one workgroup streams at most this many gathered elements per launch (the toy batches
// are a few hundred); larger batches take the host-refreshed index path
long long dtp_gather_ring_max_elems() { return 1ll << 16; }

int dtp_gather_rows2_ring(const float* X, int dx, const float* Y, int dy, long long* ring, int batch, int steps,
                          int n, long long nrows, float* ox, float* oy, void* stream) {
  if (!X || !Y || !ring || !ox || !oy || n <= 0 || n > batch || steps <= 0 || dx <= 0 || dy <= 0 || nrows <= 0 ||
      (long long)n * (dx + dy) > dtp_gather_ring_max_elems())
    return dtp::set_err(-1, "gather_rows2_ring: bad arguments");
  hipLaunchKernelGGL(dtp::gather_rows2_ring_kernel, dim3(1), dim3(dtp::kBlock), 0, (hipStream_t)stream, X, dx, Y, dy,
                     ring, batch, steps, n, nrows, ox, oy);
  return dtp::check_launch("gather_rows2_ring_kernel");
}

int dtp_gather_rows2(const float* X, int dx, const float* Y, int dy, const long long* idx, int n, long long nrows,
                     float* ox, float* oy, void* stream) {
  if (!X || !Y || !idx || !ox || !oy || n <= 0 || dx <= 0 || dy <= 0 || nrows <= 0)
    return dtp::set_err(-1, "gather_rows2: bad arguments");
  const long long total = (long long)n * (dx + dy);
  const long long blocks = (total + dtp::kBlock - 1) / dtp::kBlock;
  const int grid = (int)(blocks < 1024 ? blocks : 1024);
  hipLaunchKernelGGL(dtp::gather_rows2_kernel, dim3(grid), dim3(dtp::kBlock), 0, (hipStream_t)stream, X, dx, Y, dy,
                     idx, n, nrows, ox, oy);
  return dtp::check_launch("gather_rows2_kernel");
}

// the single-workgroup forward serves up to kMseMax elements (beyond: the caller's torch path)
// (64 Ki: one CU streams 512 KiB in a few us; beyond that torch's multi-block reduction is faster)
long long dtp_mse_max_elems() { return 1ll << 16; }

int dtp_mse_fwd(const float* a, const float* b, long long n, float* out, void* stream) {
  if (!a || !b || !out || n <= 0 || n > dtp_mse_max_elems()) return dtp::set_err(-1, "mse_fwd: 1..2^16 elements");
  hipLaunchKernelGGL(dtp::mse_fwd_kernel, dim3(1), dim3(dtp::kBlock), 0, (hipStream_t)stream, a, b, n,
                     1.f / (float)n, out);
  return dtp::check_launch("mse_fwd_kernel");
}

int dtp_mse_bwd(const float* a, const float* b, const float* g, long long n, float* ga, float* gb, void* stream) {
  if (!a || !b || !g || n <= 0 || (!ga && !gb)) return dtp::set_err(-1, "mse_bwd: bad arguments");
  const long long blocks = (n + dtp::kBlock - 1) / dtp::kBlock;
  const int grid = (int)(blocks < 1024 ? blocks : 1024);
  hipLaunchKernelGGL(dtp::mse_bwd_kernel, dim3(grid), dim3(dtp::kBlock), 0, (hipStream_t)stream, a, b, g, n,
                     2.f / (float)n, ga, gb);
  return dtp::check_launch("mse_bwd_kernel");
}

// ring / slot (nullable): also append (loss1, loss2) to a device loss log of `width` >= 2
// floats per row at row slot[0], and advance slot[0] (the caller sizes the log)
int dtp_mse_pair_fwd(const float* a1, const float* a2, const float* b, long long n, float* o1, float* o2,
                     float* osum, float* ring, long long* slot, int width, void* stream) {
  if (!a1 || !a2 || !b || !o1 || !o2 || !osum || n <= 0 || n > dtp_mse_max_elems())
    return dtp::set_err(-1, "mse_pair_fwd: 1..2^16 elements");
  if (ring && (!slot || width < 2)) return dtp::set_err(-1, "mse_pair_fwd: a loss log needs a slot and width >= 2");
  hipLaunchKernelGGL(dtp::mse_pair_fwd_kernel, dim3(1), dim3(dtp::kBlock), 0, (hipStream_t)stream, a1, a2, b, n,
                     1.f / (float)n, o1, o2, osum, ring, slot, width);
  return dtp::check_launch("mse_pair_fwd_kernel");
}

int dtp_mse_pair_bwd(const float* a1, const float* a2, const float* b, const float* g1, const float* g2,
                     const float* gsum, long long n, float* ga1, float* ga2, float* gb, void* stream) {
  if (!a1 || !a2 || !b || n <= 0 || (!ga1 && !ga2 && !gb)) return dtp::set_err(-1, "mse_pair_bwd: bad arguments");
  const long long blocks = (n + dtp::kBlock - 1) / dtp::kBlock;
  const int grid = (int)(blocks < 1024 ? blocks : 1024);
  hipLaunchKernelGGL(dtp::mse_pair_bwd_kernel, dim3(grid), dim3(dtp::kBlock), 0, (hipStream_t)stream, a1, a2, b, g1,
                     g2, gsum, n, 2.f / (float)n, ga1, ga2, gb);
  return dtp::check_launch("mse_pair_bwd_kernel");
}

}  // extern "C"
