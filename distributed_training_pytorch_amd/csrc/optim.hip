// Flat optimizer over [n_models][P] parameters after an external (RCCL)
// gradient all-reduce: one launch updates every model (the reference runs
// ~7 elementwise kernels per parameter tensor x 10 tensors x 2 models,
// SURVEY.md §2.6 K11).  The DDP 1/W averaging and the loss bookkeeping are
// fused in, and so is the bf16 compute copy of the weights (`shadow`): the
// bf16-compute GEMM path reads its weight operands from it instead of casting the
// fp32 masters before every forward (2 B/parameter written here vs a 6 B/parameter
// cast pass and one launch per weight tensor).
#include <string>

#include "dtp_api.h"
#include "optim_core.h"

namespace dtp {

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kBlock) void flat_optimizer_kernel(DtpOptArgs a) {
  const int model = blockIdx.y;
  const long long t = a.step[model];
  float* p = a.params + (size_t)model * a.P;
  float* m = a.opt_m + (size_t)model * a.P;
  float* v = a.opt_v ? a.opt_v + (size_t)model * a.P : nullptr;
  const float* g = a.grad + (size_t)model * a.P;
  // DTP_OPT_ZERO_GRAD: the consumed gradient is zeroed in the same pass (the Trainer's
  // module path then needs no zero_grad fill launch before the next backward)
  const bool zg = a.flags & DTP_OPT_ZERO_GRAD;
  float* const gz = const_cast<float*>(g);
  __bf16* sh = a.shadow ? reinterpret_cast<__bf16*>(a.shadow) + (size_t)model * a.shadow_ld : nullptr;
  // float4 body: the four rows share their offset within 16 bytes (same [n][P] layout
  // on 16-byte aligned bases), so `head` scalar elements (0-3) bring every row to a
  // 16-byte boundary, the body runs 4 elements per thread and load, and at most 3
  // elements remain (the update is HBM-bound: 28 B per parameter). With an odd P the
  // second model's row starts off a 16-byte boundary: before the head peel it ran
  // the element-wise loop.
  const uintptr_t ph = (uintptr_t)p & 15;
  const bool vec = v && (((uintptr_t)m & 15) == ph) && (((uintptr_t)v & 15) == ph) && (((uintptr_t)g & 15) == ph) &&
                   (ph & 3) == 0 && (!sh || (ph == 0 && (a.P & 3) == 0 && ((uintptr_t)sh & 7) == 0));
  if (a.kind == DTP_MODE_ADAM && vec) {
    const AdamScalars s = adam_scalars(a.hp, t + 1);
    const int head = min((int)((16 - ph) & 15) >> 2, a.P);
    const int P4 = (a.P - head) >> 2, tail0 = head + 4 * P4;
    float4* p4 = reinterpret_cast<float4*>(p + head);
    float4* m4 = reinterpret_cast<float4*>(m + head);
    float4* v4 = reinterpret_cast<float4*>(v + head);
    const float4* g4 = reinterpret_cast<const float4*>(g + head);
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < P4; i += gridDim.x * kBlock) {
      float4 w = p4[i], mi = m4[i], vi = v4[i];
      const float4 gi = g4[i];
      if (zg) reinterpret_cast<float4*>(gz + head)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      adam_update(w.x, mi.x, vi.x, gi.x * a.hp.grad_scale, s);
      adam_update(w.y, mi.y, vi.y, gi.y * a.hp.grad_scale, s);
      adam_update(w.z, mi.z, vi.z, gi.z * a.hp.grad_scale, s);
      adam_update(w.w, mi.w, vi.w, gi.w * a.hp.grad_scale, s);
      p4[i] = w;
      m4[i] = mi;
      v4[i] = vi;
      if (sh) reinterpret_cast<bf16x4*>(sh)[i] = bf16x4{(__bf16)w.x, (__bf16)w.y, (__bf16)w.z, (__bf16)w.w};
    }
    // the head and tail elements (at most 6), one per thread of the first block
    const int e = blockIdx.x == 0 ? (int)threadIdx.x : 1 << 30;
    const int idx = e < head ? e : (e - head < a.P - tail0 ? tail0 + e - head : -1);
    if (idx >= 0) {
      float w = p[idx], mi = m[idx], vi = v[idx];
      const float gv = g[idx];
      if (zg) gz[idx] = 0.f;
      adam_update(w, mi, vi, gv * a.hp.grad_scale, s);
      p[idx] = w;
      m[idx] = mi;
      v[idx] = vi;
      if (sh) sh[idx] = (__bf16)w;
    }
  } else if (a.kind == DTP_MODE_ADAM && sh) {
    // unaligned rows (odd P: every bias-terminated MLP) with a shadow: two elements per
    // thread, so the shadow is written as one 4-byte bf16 pair per lane (the shadow's
    // rows are 512-byte aligned, ComputeShadow); single 2-byte stores per lane ran the
    // whole kernel 15 % slower
    const AdamScalars s = adam_scalars(a.hp, t + 1);
    const int P2 = (a.P + 1) >> 1;
    for (int j = blockIdx.x * kBlock + threadIdx.x; j < P2; j += gridDim.x * kBlock) {
      const int i = 2 * j;
      const bool two = i + 1 < a.P;
      float w0 = p[i], m0 = m[i], v0 = v[i];
      const float g0 = g[i];
      float w1 = 0.f, m1 = 0.f, v1 = 0.f, g1 = 0.f;
      if (two) w1 = p[i + 1], m1 = m[i + 1], v1 = v[i + 1], g1 = g[i + 1];
      if (zg) {
        gz[i] = 0.f;
        if (two) gz[i + 1] = 0.f;
      }
      adam_update(w0, m0, v0, g0 * a.hp.grad_scale, s);
      p[i] = w0;
      m[i] = m0;
      v[i] = v0;
      if (two) {
        adam_update(w1, m1, v1, g1 * a.hp.grad_scale, s);
        p[i + 1] = w1;
        m[i + 1] = m1;
        v[i + 1] = v1;
        *reinterpret_cast<bf16x2*>(sh + i) = bf16x2{(__bf16)w0, (__bf16)w1};
      } else {
        sh[i] = (__bf16)w0;
      }
    }
  } else if (a.kind == DTP_MODE_ADAM) {
    const AdamScalars s = adam_scalars(a.hp, t + 1);
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < a.P; i += gridDim.x * kBlock) {
      float w = p[i], mi = m[i], vi = v[i];
      const float gv = g[i];
      if (zg) gz[i] = 0.f;
      adam_update(w, mi, vi, gv * a.hp.grad_scale, s);
      p[i] = w;
      m[i] = mi;
      v[i] = vi;
    }
  } else {
    const float lr = (float)a.hp.lr, mom = (float)a.hp.momentum, wd = (float)a.hp.weight_decay;
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < a.P; i += gridDim.x * kBlock) {
      float w = p[i], bi = m[i];
      const float gv = g[i];
      if (zg) gz[i] = 0.f;
      sgd_update(w, bi, gv * a.hp.grad_scale, lr, mom, wd, t == 0);
      p[i] = w;
      m[i] = bi;
      if (sh) sh[i] = (__bf16)w;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (a.loss_log)
      a.loss_log[(size_t)(t % a.loss_log_cap) * a.n_models + model] = a.grad[(size_t)a.n_models * a.P + model] * a.loss_scale;
  }
  // the step counter is read by every block of this model: advance it only
  // after the grid is done -> done by the last block via a ticket would cost a
  // fence; instead the counter is advanced by a 1-block follow-up in the same
  // stream when gridDim.x > 1 (see launcher).
  if (gridDim.x == 1 && threadIdx.x == 0) a.step[model] = (int)(t + 1);
}

__global__ void advance_steps_kernel(int* step, int n) {
  const int i = threadIdx.x;
  if (i < n) step[i] += 1;
}

}  // namespace dtp

namespace {
thread_local std::string g_opt_err;
}

extern "C" int dtp_flat_optimizer(const DtpOptArgs* a, void* stream) {
  if (!a || a->P <= 0 || a->n_models <= 0) return -1;
  if (a->kind != DTP_MODE_ADAM && a->kind != DTP_MODE_SGD) return -2;
  hipStream_t st = (hipStream_t)stream;
  // small models (the toy's 371 parameters): one block per model loops over its
  // parameters and advances the step counter itself -- no follow-up launch
  int nblk = a->P <= 16 * dtp::kBlock ? 1 : (a->P + dtp::kBlock - 1) / dtp::kBlock;
  if (nblk > 1024) nblk = 1024;
  dim3 grid(nblk, a->n_models), block(dtp::kBlock);
  hipLaunchKernelGGL(dtp::flat_optimizer_kernel, grid, block, 0, st, *a);
  if (nblk > 1) hipLaunchKernelGGL(dtp::advance_steps_kernel, dim3(1), dim3(64), 0, st, a->step, a->n_models);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
