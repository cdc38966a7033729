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
#include "optim_core.h"
#include "xgmi_core.h"

namespace dtp {

constexpr int kDataCache = 4096;  // floats of dataset that may be staged in LDS

template <class S>
struct TrainSmem {
  float w[S::pad4(S::LP)];
  float stage[4][2048];  // per wave: 64 dz rows + 64 h rows; reused for the dW tile reduction
  float data[kDataCache];
  float lred[4];
};

template <class S, int MODE>
__global__ __launch_bounds__(kBlock) void mlp_train_kernel(DtpTrainArgs a) {
  static_assert(4 * S::NL * 256 <= 4 * 2048, "reduction tiles must fit in the staging area");
  __shared__ __align__(16) TrainSmem<S> sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int model = blockIdx.x;
  constexpr int P = S::P;
  constexpr bool kUpdate = MODE != DTP_MODE_GRAD;
  constexpr bool kAdam = MODE == DTP_MODE_ADAM || MODE == DTP_MODE_XGMI_ADAM;
  constexpr bool kXgmi = MODE == DTP_MODE_XGMI_ADAM || MODE == DTP_MODE_XGMI_SGD;
  const bool ce = a.loss == DTP_LOSS_CE;
  const int ydim = ce ? 1 : S::OUT;

  float* __restrict__ gp = a.params + (size_t)model * P;
  for (int p = tid; p < P; p += kBlock) sm.w[lds_pos<S>(p)] = gp[p];

  const int rowf = S::IN + ydim;
  const bool cached = a.cache_data && a.smp.n * rowf <= kDataCache;
  if (cached) {
    for (int e = tid; e < a.smp.n * S::IN; e += kBlock) sm.data[e] = a.X[e];
    for (int e = tid; e < a.smp.n * ydim; e += kBlock) sm.data[a.smp.n * S::IN + e] = a.Y[e];
  }
  const float* __restrict__ Xs = cached ? sm.data : a.X;
  const float* __restrict__ Ys = cached ? sm.data + a.smp.n * S::IN : a.Y;

  // this thread owns parameters tid, tid+256, ... in the optimizer phase
  int lp[S::NPT], tp[S::NPT];
  float mr[S::NPT], vr[S::NPT];
#pragma unroll
  for (int k = 0; k < S::NPT; ++k) {
    const int p = tid + k * kBlock;
    lp[k] = lds_pos<S>(p < P ? p : 0);
    tp[k] = tile_pos<S>(p < P ? p : 0);
    mr[k] = 0.f;
    vr[k] = 0.f;
    if (kUpdate && p < P) {
      mr[k] = a.opt_m[(size_t)model * P + p];
      if (kAdam) vr[k] = a.opt_v[(size_t)model * P + p];
    }
  }
  const long long t0 = a.step[model];
  unsigned xepoch = kXgmi ? a.epoch[model] : 0u;
  __syncthreads();

  for (int it = 0; it < a.n_steps; ++it) {
    const long long t = t0 + it;
    int bsz;
    BatchPos bp{};
    uint32_t keys[4] = {0u, 0u, 0u, 0u};
    const bool explicit_idx = a.smp.mode == SAMPLER_EXPLICIT;
    if (explicit_idx) {
      bsz = a.smp.batch;
    } else {
      bp = batch_pos(a.smp, t);
      epoch_keys(a.smp, bp.epoch, keys);
      bsz = bp.size;
    }
    const float inv = ce ? 1.f / (float)bsz : 1.f / (float)(bsz * S::OUT);

    f32x4 acc[S::NL];
#pragma unroll
    for (int l = 0; l < S::NL; ++l) acc[l] = f32x4{0.f, 0.f, 0.f, 0.f};
    float lsum = 0.f;

    for (int c0 = 0; c0 < bsz; c0 += kBlock) {
      const int k = c0 + tid;
      const bool valid = k < bsz;
      int di = 0;
      if (valid) di = explicit_idx ? a.idx[(size_t)it * a.smp.batch + k] : sample_index(a.smp, bp, keys, k);
      float h[S::NL + 1][16];
      static_for<0, S::IN>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        h[0][i] = valid ? Xs[(size_t)di * S::IN + i] : 0.f;
      });
      mlp_forward<S>(sm.w, h, a.hp.slope);
      float dz[16];
      if (!ce) {
        static_for<0, S::OUT>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          const float d = h[S::NL][j] - (valid ? Ys[(size_t)di * S::OUT + j] : 0.f);
          lsum += valid ? d * d : 0.f;
          dz[j] = valid ? 2.f * d * inv : 0.f;
        });
      } else {
        const int cls = valid ? (int)Ys[di] : 0;
        float mx = h[S::NL][0];
        static_for<1, S::OUT>([&](auto JC) { mx = fmaxf(mx, h[S::NL][decltype(JC)::value]); });
        float se = 0.f, zc = 0.f;
        static_for<0, S::OUT>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          dz[j] = __expf(h[S::NL][j] - mx);
          se += dz[j];
          zc = (j == cls) ? h[S::NL][j] : zc;
        });
        const float lse = mx + __logf(se);
        lsum += valid ? lse - zc : 0.f;
        const float rs = 1.f / se;
        static_for<0, S::OUT>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          dz[j] = valid ? (dz[j] * rs - (j == cls ? 1.f : 0.f)) * inv : 0.f;
        });
      }
      float dx[16];
      mlp_backward<S, false>(sm.w, h, dz, &sm.stage[wave][0], acc, a.hp.slope, lane, dx);
    }

    lsum = wave_sum(lsum);
    __syncthreads();  // every wave is done with its staging rows
    store_partial_tiles<S>(&sm.stage[0][0], acc, wave, lane);
    if (lane == 0) sm.lred[wave] = lsum;
    __syncthreads();
    const float mean_loss = (sm.lred[0] + sm.lred[1] + sm.lred[2] + sm.lred[3]) * (ce ? inv : inv);

    float g[S::NPT];
#pragma unroll
    for (int k = 0; k < S::NPT; ++k) g[k] = sum_partial_tiles<S>(&sm.stage[0][0], tp[k], 4);

    float gloss = mean_loss;
    if constexpr (kXgmi) {
      // all-reduce (sum) this model's gradient + loss over every rank through
      // the peers' xGMI-mapped receive buffers, inside the step (xgmi_core.h)
      xepoch += 1u;
      gloss = xgmi_allreduce_model<S::NPT>(a, model, P, g, mean_loss, xepoch, tid);
    }

    if (tid == 0 && a.loss_log) {
      const float lg = kXgmi ? gloss * a.hp.grad_scale : mean_loss;
      a.loss_log[(size_t)(t % a.loss_log_cap) * a.n_models + model] = lg;
    }

    if constexpr (MODE == DTP_MODE_GRAD) {
#pragma unroll
      for (int k = 0; k < S::NPT; ++k) {
        const int p = tid + k * kBlock;
        if (p < P) a.grad_out[(size_t)model * P + p] = g[k] * a.hp.grad_scale;
      }
      if (tid == 0) a.grad_out[(size_t)a.n_models * P + model] = mean_loss;
    } else if constexpr (kAdam) {
      const AdamScalars s = adam_scalars(a.hp, t + 1);
#pragma unroll
      for (int k = 0; k < S::NPT; ++k) {
        const int p = tid + k * kBlock;
        if (p < P) {
          float w = sm.w[lp[k]];
          adam_update(w, mr[k], vr[k], g[k] * a.hp.grad_scale, s);
          sm.w[lp[k]] = w;
        }
      }
    } else {
      const float lr = (float)a.hp.lr, mom = (float)a.hp.momentum, wd = (float)a.hp.weight_decay;
#pragma unroll
      for (int k = 0; k < S::NPT; ++k) {
        const int p = tid + k * kBlock;
        if (p < P) {
          float w = sm.w[lp[k]];
          sgd_update(w, mr[k], g[k] * a.hp.grad_scale, lr, mom, wd, t == 0);
          sm.w[lp[k]] = w;
        }
      }
    }
    __syncthreads();  // updated weights visible; reduction tiles consumed
  }

  if constexpr (kUpdate) {
    for (int p = tid; p < P; p += kBlock) gp[p] = sm.w[lds_pos<S>(p)];
#pragma unroll
    for (int k = 0; k < S::NPT; ++k) {
      const int p = tid + k * kBlock;
      if (p < P) {
        a.opt_m[(size_t)model * P + p] = mr[k];
        if (kAdam) a.opt_v[(size_t)model * P + p] = vr[k];
      }
    }
    if (tid == 0) a.step[model] = (int)(t0 + a.n_steps);
    if (kXgmi && tid == 0) a.epoch[model] = xepoch;
  }
}

// ------------------------------------------------------------------------------
// stage forward: one lane per sample, any number of workgroups
template <class S>
__global__ __launch_bounds__(kBlock) void mlp_stage_fwd_kernel(DtpStageArgs a) {
  __shared__ __align__(16) float sw[S::pad4(S::LP)];
  for (int p = threadIdx.x; p < S::P; p += kBlock) sw[lds_pos<S>(p)] = a.params[p];
  __syncthreads();
  const int b = blockIdx.x * kBlock + threadIdx.x;
  if (b >= a.batch) return;
  float h[S::NL + 1][16];
  static_for<0, S::IN>([&](auto IC) { h[0][decltype(IC)::value] = a.x[(size_t)b * S::IN + decltype(IC)::value]; });
  mlp_forward<S>(sw, h, a.slope);
  static_for<0, S::OUT>([&](auto JC) { a.out[(size_t)b * S::OUT + decltype(JC)::value] = h[S::NL][decltype(JC)::value]; });
  if (a.saved) {
    static_for<1, S::NL>([&](auto LC) {
      constexpr int l = decltype(LC)::value;
      static_for<0, S::H>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        a.saved[(size_t)b * S::SAVED + (l - 1) * S::H + i] = h[l][i];
      });
    });
  }
}

// stage backward: grid-stride over 256-sample chunks; per-wave MFMA dW tiles,
// LDS reduction, then one plain store (single block) or float atomics (multi block)
template <class S, bool WANT_DX>
__global__ __launch_bounds__(kBlock) void mlp_stage_bwd_kernel(DtpStageArgs a) {
  __shared__ __align__(16) struct {
    float w[S::pad4(S::LP)];
    float stage[4][2048];
  } sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int p = tid; p < S::P; p += kBlock) sm.w[lds_pos<S>(p)] = a.params[p];
  __syncthreads();
  f32x4 acc[S::NL];
#pragma unroll
  for (int l = 0; l < S::NL; ++l) acc[l] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c0 = blockIdx.x * kBlock; c0 < a.batch; c0 += gridDim.x * kBlock) {
    const int b = c0 + tid;
    const bool valid = b < a.batch;
    float h[S::NL + 1][16];
    static_for<0, S::IN>([&](auto IC) {
      constexpr int i = decltype(IC)::value;
      h[0][i] = valid ? a.x[(size_t)b * S::IN + i] : 0.f;
    });
    static_for<1, S::NL>([&](auto LC) {
      constexpr int l = decltype(LC)::value;
      static_for<0, S::H>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        h[l][i] = valid ? a.saved[(size_t)b * S::SAVED + (l - 1) * S::H + i] : 0.f;
      });
    });
    float dz[16];
    static_for<0, S::OUT>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      float go = valid ? a.grad_out[(size_t)b * S::OUT + j] : 0.f;
      if constexpr (S::FINAL_ACT) go *= leaky_grad_from_out(valid ? a.out[(size_t)b * S::OUT + j] : 0.f, a.slope);
      dz[j] = go;
    });
    float dx[16];
    mlp_backward<S, WANT_DX>(sm.w, h, dz, &sm.stage[wave][0], acc, a.slope, lane, dx);
    if constexpr (WANT_DX) {
      if (valid) {
        static_for<0, S::IN>([&](auto IC) {
          a.grad_in[(size_t)b * S::IN + decltype(IC)::value] = dx[decltype(IC)::value];
        });
      }
    }
  }
  __syncthreads();
  store_partial_tiles<S>(&sm.stage[0][0], acc, wave, lane);
  __syncthreads();
  for (int p = tid; p < S::P; p += kBlock) {
    const float g = sum_partial_tiles<S>(&sm.stage[0][0], tile_pos<S>(p), 4);
    if (gridDim.x == 1)
      a.grad_params[p] = g;
    else
      atomicAdd(&a.grad_params[p], g);
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
thread_local std::string g_err;
int set_err(int code, const std::string& m) {
  g_err = m;
  return code;
}
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_err(-3, std::string(what) + ": " + hipGetErrorString(e));
  return 0;
}

// (IN, H, NL, OUT): shapes the fused train-step kernel is instantiated for
#define DTP_TRAIN_SHAPES(X) \
  X(2, 10, 5, 1)            \
  X(2, 10, 3, 1)            \
  X(2, 10, 5, 2)            \
  X(2, 10, 5, 4)            \
  X(2, 15, 5, 1)            \
  X(2, 15, 5, 4)            \
  X(4, 15, 5, 4)

// (IN, H, NL, OUT, FINAL_ACT): every contiguous layer range of the toy model
// (layer-split stages) plus the train shapes as whole-model stages
#define DTP_STAGE_SHAPES(X) \
  X(2, 10, 5, 1, false)     \
  X(2, 10, 4, 10, true)     \
  X(10, 10, 4, 1, false)    \
  X(2, 10, 3, 10, true)     \
  X(10, 10, 3, 10, true)    \
  X(10, 10, 3, 1, false)    \
  X(2, 10, 2, 10, true)     \
  X(10, 10, 2, 10, true)    \
  X(10, 10, 2, 1, false)    \
  X(2, 10, 1, 10, true)     \
  X(10, 10, 1, 10, true)    \
  X(10, 10, 1, 1, false)    \
  X(2, 10, 3, 1, false)     \
  X(2, 10, 5, 2, false)     \
  X(2, 10, 5, 4, false)     \
  X(2, 15, 5, 1, false)     \
  X(2, 15, 5, 4, false)     \
  X(4, 15, 5, 4, false)

template <class S>
int launch_train(const DtpTrainArgs* a, int mode, hipStream_t st) {
  dim3 grid(a->n_models), block(dtp::kBlock);
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
int launch_stage_fwd(const DtpStageArgs* a, hipStream_t st) {
  if (a->batch <= 0) return 0;
  dim3 grid((a->batch + dtp::kBlock - 1) / dtp::kBlock), block(dtp::kBlock);
  hipLaunchKernelGGL((dtp::mlp_stage_fwd_kernel<S>), grid, block, 0, st, *a);
  return check_launch("mlp_stage_fwd_kernel");
}

template <class S>
int launch_stage_bwd(const DtpStageArgs* a, hipStream_t st) {
  if (a->batch <= 0) return 0;
  // one block reduces deterministically up to 4 chunks; larger batches spread
  // over more CUs and combine with float atomics into the zeroed grad buffer
  int nblk = (a->batch + 4 * dtp::kBlock - 1) / (4 * dtp::kBlock);
  if (nblk > 256) nblk = 256;
  dim3 grid(nblk), block(dtp::kBlock);
  if (a->grad_in)
    hipLaunchKernelGGL((dtp::mlp_stage_bwd_kernel<S, true>), grid, block, 0, st, *a);
  else
    hipLaunchKernelGGL((dtp::mlp_stage_bwd_kernel<S, false>), grid, block, 0, st, *a);
  return check_launch("mlp_stage_bwd_kernel");
}
}  // namespace

extern "C" {

int dtp_version(void) { return 1; }
const char* dtp_last_error(void) { return g_err.c_str(); }

int dtp_mlp_supported(int in, int h, int nl, int out, int final_act) {
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return 1;
  DTP_STAGE_SHAPES(X)
#undef X
  return 0;
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

int dtp_mlp_stage_fwd(const DtpStageArgs* a, int in, int h, int nl, int out, int final_act, void* stream) {
  hipStream_t st = (hipStream_t)stream;
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return launch_stage_fwd<dtp::Stage<I, H, N, O, F>>(a, st);
  DTP_STAGE_SHAPES(X)
#undef X
  return set_err(-2, "mlp stage shape not instantiated");
}

int dtp_mlp_stage_bwd(const DtpStageArgs* a, int in, int h, int nl, int out, int final_act, void* stream) {
  hipStream_t st = (hipStream_t)stream;
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return launch_stage_bwd<dtp::Stage<I, H, N, O, F>>(a, st);
  DTP_STAGE_SHAPES(X)
#undef X
  return set_err(-2, "mlp stage shape not instantiated");
}

int dtp_sampler_indices(const dtp::SamplerCfg* s, long long t0, int n_steps, int* out, void* stream) {
  if (!s || !out || s->batch <= 0 || n_steps <= 0) return set_err(-1, "bad sampler probe args");
  dim3 grid((s->batch + 255) / 256, n_steps), block(256);
  hipLaunchKernelGGL(dtp::sampler_probe_kernel, grid, block, 0, (hipStream_t)stream, *s, t0, n_steps, out);
  return check_launch("sampler_probe_kernel");
}

}  // extern "C"
