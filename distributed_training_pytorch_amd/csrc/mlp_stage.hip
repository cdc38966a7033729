// Layer-split stage kernels (autograd path): forward one lane per sample,
// backward = input-gradient VALU chain + MFMA weight-gradient reduction
// (mlp_core.h).  Equivalent of one MultiGPUModel stage of
// demo_one_model_multi_gpu.py:17-42 and of nn.Sequential fwd/bwd in
// toy_model_and_data.py:8-25.
#include <string>

#include "dtp_api.h"
#include "mlp_core.h"
#include "optim_core.h"

namespace dtp {
constexpr int kStage = 2 * kStgArr;

// stage forward: one lane per sample, any number of workgroups
template <class S>
DTP_DEV void stage_fwd_body(const DtpStageArgs& a, float* sw);

template <class S>
__global__ __launch_bounds__(kBlock) void mlp_stage_fwd_kernel(DtpStageArgs a) {
  __shared__ __align__(16) float sw[S::pad4(S::LP)];
  stage_fwd_body<S>(a, sw);
}

// several models of one shape in ONE launch (blockIdx.y = model): the Trainer demo's two
// models on the same batch (demo_pytorch_lightning.py: model_X(x), model_Y(x)); the stage
// arguments come straight from the kernarg segment (indexing the by-value parameter with
// blockIdx would copy it to scratch)
template <class S>
__global__ __launch_bounds__(kBlock) void mlp_stage_fwd_multi_kernel(DtpStageMulti) {
  __shared__ __align__(16) float sw[S::pad4(S::LP)];
  const DtpStageMulti* M = (const DtpStageMulti*)__builtin_amdgcn_kernarg_segment_ptr();
  const DtpStageArgs a = M->stage[blockIdx.y];
  stage_fwd_body<S>(a, sw);
}

template <class S>
DTP_DEV void stage_fwd_body(const DtpStageArgs& a, float* sw) {
  for (int p = threadIdx.x; p < S::P; p += kBlock) lds_store_param<S>(sw, p, a.params[p]);
  __syncthreads();
  const int b = blockIdx.x * kBlock + threadIdx.x;
  if (b >= a.batch) return;
  float h[S::NL + 1][16];
  static_for<0, S::IN>([&](auto IC) { h[0][decltype(IC)::value] = S::rnd(a.x[(size_t)b * S::IN + decltype(IC)::value]); });
  mlp_forward<S>(sw, h, a.slope);
  static_for<0, S::OUT>([&](auto JC) { a.out[(size_t)b * S::OUT + decltype(JC)::value] = h[S::NL][decltype(JC)::value]; });
  if (a.out_peer) {  // layer-split hand-off: the epilogue writes the next GPU's input directly
    static_for<0, S::OUT>([&](auto JC) {
      a.out_peer[(size_t)b * S::OUT + decltype(JC)::value] = h[S::NL][decltype(JC)::value];
    });
  }
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
// LDS reduction, then one plain store (single block) or float atomics (multi block).
// OPT: one block, and the flat optimizer's step over this stage's parameters fused into
// the store loop (the Trainer's module path: the backward of a toggled model's last
// autograd node and its optimizer step in ONE launch, ops/mlp.py "param-backward
// fusion"): the thread that sums dW_p also updates p, m[p], v[p] -- the weights were
// staged in LDS before, so no wave reads a global weight after it is updated.  The same
// adam_update / sgd_update as flat_optimizer_kernel: bitwise the unfused pair.
template <class S, bool WANT_DX, bool OPT>
DTP_DEV void stage_bwd_body(const DtpStageArgs& a, const DtpOptArgs& o) {
  __shared__ __align__(16) struct {
    float w[S::pad4(S::LP)];
    float stage[4][kStage];
  } sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long t = 0;
  if constexpr (OPT) t = o.step[0];  // read before the first barrier; advanced at the end by thread 0
  for (int p = tid; p < S::P; p += kBlock) lds_store_param<S>(sm.w, p, a.params[p]);
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
      h[0][i] = valid ? S::rnd(a.x[(size_t)b * S::IN + i]) : 0.f;
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
      float go = valid ? S::rnd(a.grad_out[(size_t)b * S::OUT + j]) : 0.f;
      if constexpr (S::FINAL_ACT) go = S::rnd(go * leaky_grad_from_out(valid ? a.out[(size_t)b * S::OUT + j] : 0.f, a.slope));
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
  if constexpr (OPT) {
    const bool zg = o.flags & DTP_OPT_ZERO_GRAD;
    const float gs = o.hp.grad_scale;
    if (o.kind == DTP_MODE_ADAM) {
      const AdamScalars sc = adam_scalars(o.hp, t + 1);
      for (int p = tid; p < S::P; p += kBlock) {
        const float g = sum_partial_tiles<S>(&sm.stage[0][0], tile_pos<S>(p), 4);
        const float gt = a.accumulate ? a.grad_params[p] + g : g;
        float w = o.params[p], mi = o.opt_m[p], vi = o.opt_v[p];
        adam_update(w, mi, vi, gt * gs, sc);
        o.params[p] = w;
        o.opt_m[p] = mi;
        o.opt_v[p] = vi;
        a.grad_params[p] = zg ? 0.f : gt;
      }
    } else {
      const float lr = (float)o.hp.lr, mom = (float)o.hp.momentum, wd = (float)o.hp.weight_decay;
      for (int p = tid; p < S::P; p += kBlock) {
        const float g = sum_partial_tiles<S>(&sm.stage[0][0], tile_pos<S>(p), 4);
        const float gt = a.accumulate ? a.grad_params[p] + g : g;
        float w = o.params[p], bi = o.opt_m[p];
        sgd_update(w, bi, gt * gs, lr, mom, wd, t == 0);
        o.params[p] = w;
        o.opt_m[p] = bi;
        a.grad_params[p] = zg ? 0.f : gt;
      }
    }
    if (tid == 0) o.step[0] = (int)(t + 1);
  } else {
    for (int p = tid; p < S::P; p += kBlock) {
      const float g = sum_partial_tiles<S>(&sm.stage[0][0], tile_pos<S>(p), 4);
      if (gridDim.x == 1)
        a.grad_params[p] = a.accumulate ? a.grad_params[p] + g : g;
      else
        atomicAdd(&a.grad_params[p], g);
    }
  }
}

template <class S, bool WANT_DX>
__global__ __launch_bounds__(kBlock) void mlp_stage_bwd_kernel(DtpStageArgs a) {
  stage_bwd_body<S, WANT_DX, false>(a, DtpOptArgs{});
}

// several models of one shape (blockIdx.y = model): model y's stage backward and the
// optimizer's row y in one block -- the module engine's ModelBank (both models' backwards
// and their one flat Adam: 3 launches -> 1).  Arguments from the kernarg segment, as in
// the forward's multi kernel.
template <class S>
__global__ __launch_bounds__(kBlock) void mlp_stage_bwd_opt_kernel(DtpStageMulti, DtpOptArgs O) {
  const DtpStageMulti* M = (const DtpStageMulti*)__builtin_amdgcn_kernarg_segment_ptr();  // the first argument
  const int y = blockIdx.y;
  const DtpStageArgs a = M->stage[y];
  DtpOptArgs o = O;
  const size_t off = (size_t)y * o.P;
  o.params += off;
  o.opt_m += off;
  if (o.opt_v) o.opt_v += off;
  o.step += y;
  o.grad += off;
  stage_bwd_body<S, false, true>(a, o);
}

}  // namespace dtp

namespace {
using dtp::check_launch;
using dtp::set_err;

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

// whole-model shapes that also have bf16-compute instances (autocast / precision='bf16')
#define DTP_STAGE_BF16_SHAPES(X) \
  X(2, 10, 5, 1, false)          \
  X(2, 10, 5, 4, false)

template <class S>
int launch_stage_fwd(const DtpStageArgs* a, hipStream_t st) {
  if (a->batch <= 0) return 0;
  dim3 grid((a->batch + dtp::kBlock - 1) / dtp::kBlock), block(dtp::kBlock);
  hipLaunchKernelGGL((dtp::mlp_stage_fwd_kernel<S>), grid, block, 0, st, *a);
  return check_launch("mlp_stage_fwd_kernel");
}

template <class S>
int launch_stage_fwd_multi(const DtpStageMulti* m, hipStream_t st) {
  int bmax = 0;
  for (int i = 0; i < m->n; ++i) bmax = m->stage[i].batch > bmax ? m->stage[i].batch : bmax;
  if (bmax <= 0) return 0;
  dim3 grid((bmax + dtp::kBlock - 1) / dtp::kBlock, m->n), block(dtp::kBlock);
  hipLaunchKernelGGL((dtp::mlp_stage_fwd_multi_kernel<S>), grid, block, 0, st, *m);
  return check_launch("mlp_stage_fwd_multi_kernel");
}

template <class S>
int launch_stage_bwd(const DtpStageArgs* a, hipStream_t st) {
  if (a->batch <= 0) return 0;
  // one block reduces deterministically up to 4 chunks; larger batches spread
  // over more CUs and combine with float atomics into the zeroed (or accumulated) grad buffer
  int nblk = (a->batch + 4 * dtp::kBlock - 1) / (4 * dtp::kBlock);
  if (nblk > 256) nblk = 256;
  dim3 grid(nblk), block(dtp::kBlock);
  if (a->grad_in)
    hipLaunchKernelGGL((dtp::mlp_stage_bwd_kernel<S, true>), grid, block, 0, st, *a);
  else
    hipLaunchKernelGGL((dtp::mlp_stage_bwd_kernel<S, false>), grid, block, 0, st, *a);
  return check_launch("mlp_stage_bwd_kernel");
}

// the fused form: one block per model (batch <= 4 x 256), whole-model fp32 stages, the
// optimizer's row i exactly model i's parameters and gradient (checked on the host too)
template <class S>
int launch_stage_bwd_opt(const DtpStageMulti* m, const DtpOptArgs* o, hipStream_t st) {
  if (m->n < 1 || m->n > DTP_STAGE_MULTI_MAX || o->n_models != m->n || o->P != S::P || o->shadow || o->loss_log ||
      (o->kind != DTP_MODE_ADAM && o->kind != DTP_MODE_SGD) || !o->opt_m || (o->kind == DTP_MODE_ADAM && !o->opt_v) ||
      !o->step)
    return set_err(-1, "stage_bwd_opt: the optimizer rows must be the stages' parameters and gradients");
  for (int i = 0; i < m->n; ++i) {
    const DtpStageArgs& a = m->stage[i];
    if (a.batch <= 0 || a.batch > 4 * dtp::kBlock || a.grad_in || a.bf16 || !a.grad_params ||
        o->params + (size_t)i * S::P != a.params || o->grad + (size_t)i * S::P != a.grad_params)
      return set_err(-1, "stage_bwd_opt: batch 1..1024, no input gradient, fp32, row i = stage i");
  }
  hipLaunchKernelGGL((dtp::mlp_stage_bwd_opt_kernel<S>), dim3(1, m->n), dim3(dtp::kBlock), 0, st, *m, *o);
  return check_launch("mlp_stage_bwd_opt_kernel");
}
}  // namespace

extern "C" {

int dtp_mlp_stage_bwd_opt(const DtpStageMulti* m, const DtpOptArgs* o, int in, int h, int nl, int out, int final_act,
                          void* stream) {
  if (!m || !o) return set_err(-1, "stage_bwd_opt: null arguments");
  hipStream_t st = (hipStream_t)stream;
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return launch_stage_bwd_opt<dtp::Stage<I, H, N, O, F>>(m, o, st);
  DTP_STAGE_SHAPES(X)
#undef X
  return set_err(-2, "mlp stage shape not instantiated");
}

int dtp_mlp_supported_bf16(int in, int h, int nl, int out, int final_act) {
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return 1;
  DTP_STAGE_BF16_SHAPES(X)
#undef X
  return 0;
}

int dtp_mlp_supported(int in, int h, int nl, int out, int final_act) {
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return 1;
  DTP_STAGE_SHAPES(X)
#undef X
  return 0;
}

int dtp_mlp_stage_fwd(const DtpStageArgs* a, int in, int h, int nl, int out, int final_act, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (a->bf16) {
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return launch_stage_fwd<dtp::Stage<I, H, N, O, F, true>>(a, st);
    DTP_STAGE_BF16_SHAPES(X)
#undef X
    return set_err(-2, "no bf16 instance of this mlp stage shape");
  }
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return launch_stage_fwd<dtp::Stage<I, H, N, O, F>>(a, st);
  DTP_STAGE_SHAPES(X)
#undef X
  return set_err(-2, "mlp stage shape not instantiated");
}

int dtp_mlp_stage_fwd_multi(const DtpStageMulti* m, int in, int h, int nl, int out, int final_act, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!m || m->n < 1 || m->n > DTP_STAGE_MULTI_MAX) return set_err(-1, "stage_fwd_multi: 1..4 models");
  for (int i = 0; i < m->n; ++i)
    if (m->stage[i].bf16 || m->stage[i].out_peer) return set_err(-1, "stage_fwd_multi: fp32, no peer output");
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return launch_stage_fwd_multi<dtp::Stage<I, H, N, O, F>>(m, st);
  DTP_STAGE_SHAPES(X)
#undef X
  return set_err(-2, "mlp stage shape not instantiated");
}

int dtp_mlp_stage_bwd(const DtpStageArgs* a, int in, int h, int nl, int out, int final_act, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (a->bf16) {
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return launch_stage_bwd<dtp::Stage<I, H, N, O, F, true>>(a, st);
    DTP_STAGE_BF16_SHAPES(X)
#undef X
    return set_err(-2, "no bf16 instance of this mlp stage shape");
  }
#define X(I, H, N, O, F) \
  if (in == I && h == H && nl == N && out == O && (bool)final_act == F) return launch_stage_bwd<dtp::Stage<I, H, N, O, F>>(a, st);
  DTP_STAGE_SHAPES(X)
#undef X
  return set_err(-2, "mlp stage shape not instantiated");
}

}  // extern "C"
