// Optimizer math shared by the fused train-step kernel and the flat optimizer
// kernel.  Mirrors torch.optim.Adam / torch.optim.SGD (defaults used by the
// reference: Adam(lr=1e-3), demo.py:80-81) element for element:
//   Adam:  m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
//          denom = sqrt(v)/sqrt(1-b2^t) + eps; p.addcdiv_(m, denom, -lr/(1-b1^t))
//   SGD :  buf = g (first step) | buf*mom + g;  p.add_(buf, -lr)
// with the scalar bias corrections formed in double, as torch does on the host.
#pragma once
#include "dtp_api.h"
#include "dtp_common.h"

namespace dtp {

struct AdamScalars {
  float step_size, bc2_sqrt, one_m_b1, b2, one_m_b2, eps, wd;
};

DTP_DEV AdamScalars adam_scalars(const DtpHyper& hp, long long t1) {
  AdamScalars s;
  const double bc1 = 1.0 - pow_int(hp.beta1, (uint64_t)t1);
  const double bc2 = 1.0 - pow_int(hp.beta2, (uint64_t)t1);
  s.step_size = (float)(hp.lr / bc1);
  s.bc2_sqrt = (float)sqrt(bc2);
  s.one_m_b1 = (float)(1.0 - hp.beta1);
  s.b2 = (float)hp.beta2;
  s.one_m_b2 = (float)(1.0 - hp.beta2);
  s.eps = (float)hp.eps;
  s.wd = (float)hp.weight_decay;
  return s;
}

// same, from carried powers b1t = beta1^t, b2t = beta2^t (t = the new step number)
DTP_DEV AdamScalars adam_scalars_from_pow(const DtpHyper& hp, double b1t, double b2t) {
  AdamScalars s;
  const double bc1 = 1.0 - b1t, bc2 = 1.0 - b2t;
  s.step_size = (float)(hp.lr / bc1);
  s.bc2_sqrt = (float)sqrt(bc2);
  s.one_m_b1 = (float)(1.0 - hp.beta1);
  s.b2 = (float)hp.beta2;
  s.one_m_b2 = (float)(1.0 - hp.beta2);
  s.eps = (float)hp.eps;
  s.wd = (float)hp.weight_decay;
  return s;
}

// the step-independent part of the scalars (step_size / bc2_sqrt filled by the caller)
DTP_DEV AdamScalars adam_consts(const DtpHyper& hp) {
  AdamScalars s;
  s.step_size = 0.f;
  s.bc2_sqrt = 1.f;
  s.one_m_b1 = (float)(1.0 - hp.beta1);
  s.b2 = (float)hp.beta2;
  s.one_m_b2 = (float)(1.0 - hp.beta2);
  s.eps = (float)hp.eps;
  s.wd = (float)hp.weight_decay;
  return s;
}

// Every fused multiply-add is spelled out (fmaf) and the translation units that
// use these helpers build with -ffp-contract=off (build.py), so the rounding of
// each update is fixed by the source, not by how the compiler scheduled the
// surrounding kernel: every kernel instance (FAST or generic, fused step or flat
// optimizer) produces bitwise the same update.
// DTP_ADAM_FAST (default): sqrt(v) from the hardware square root, and each division as
// a reciprocal estimate, a product and one residual correction (fma) -- within an ulp or
// two of the correctly rounded results (the torch.optim.Adam comparisons of the GPU tests
// hold at their tolerances, down to rtol 1e-6 for the flat optimizer), and a short
// dependency chain: the precise forms (v_div_scale / fmas / fixup, the scaled sqrt
// refinement) were ~30 dependent VALU ops per parameter and 0.16 us of the 4.3 us fused
// step (profiles/r4_adam/).  -DDTP_ADAM_FAST=0 restores torch's exact division / sqrt.
#ifndef DTP_ADAM_FAST
#define DTP_ADAM_FAST 1
#endif

// a / b for a normal, positive b: reciprocal estimate, product, one residual correction
DTP_DEV float div_nr(float a, float b) {
  const float r = __builtin_amdgcn_rcpf(b);
  const float q = a * r;
  return fmaf(fmaf(-b, q, a), r, q);
}

DTP_DEV void adam_update(float& p, float& m, float& v, float g, const AdamScalars& s) {
  if (s.wd != 0.f) g = fmaf(s.wd, p, g);
  m = fmaf(s.one_m_b1, g - m, m);                  // m.lerp_(g, 1 - b1)
  v = fmaf(s.one_m_b2 * g, g, v * s.b2);           // v.mul_(b2).addcmul_(g, g, 1 - b2)
#if DTP_ADAM_FAST
  const float denom = div_nr(__builtin_amdgcn_sqrtf(v), s.bc2_sqrt) + s.eps;
  p = fmaf(-s.step_size, div_nr(m, denom), p);
#else
  const float denom = sqrtf(v) / s.bc2_sqrt + s.eps;
  p = fmaf(-s.step_size, m / denom, p);            // p.addcdiv_(m, denom, -step_size)
#endif
}

DTP_DEV void sgd_update(float& p, float& buf, float g, float lr, float mom, float wd, bool first) {
  if (wd != 0.f) g = fmaf(wd, p, g);
  if (mom != 0.f) {
    buf = first ? g : fmaf(buf, mom, g);
    g = buf;
  }
  p = fmaf(-lr, g, p);
}

}  // namespace dtp
