// C ABI of libdtp.so (consumed from Python through ctypes; every struct here
// has a mirror in distributed_training_pytorch_amd/_native.py — keep in sync).
#pragma once
#include <stdint.h>
#include "sampler.h"

extern "C" {

// ---- fused train step (fwd + loss + bwd [+ optimizer]) for n_models MLPs ----
enum DtpTrainMode : int {
  DTP_MODE_GRAD = 0,       // write local mean-loss gradients (+ loss) into grad_out; no update
  DTP_MODE_ADAM = 1,       // fused Adam update (single rank, or grads already global)
  DTP_MODE_SGD = 2,        // fused SGD(+momentum) update
  DTP_MODE_XGMI_ADAM = 3,  // in-kernel xGMI all-reduce across ranks, then Adam
  DTP_MODE_XGMI_SGD = 4,   // in-kernel xGMI all-reduce across ranks, then SGD
};

enum DtpLoss : int { DTP_LOSS_MSE = 0, DTP_LOSS_CE = 1 };

struct DtpHyper {
  double lr, beta1, beta2, eps, weight_decay, momentum;
  float slope;        // LeakyReLU negative slope
  float grad_scale;   // applied to the summed gradient before the update (1/world for DDP averaging)
};

struct DtpTrainArgs {
  const float* X;       // [n][IN] dataset inputs (device resident)
  const float* Y;       // [n][OUT] targets (MSE) or [n] class ids stored as float (CE)
  const int* idx;       // SAMPLER_EXPLICIT: [n_steps][batch] dataset indices
  float* params;        // [n_models][P]
  float* opt_m;         // [n_models][P] Adam exp_avg / SGD momentum buffer
  float* opt_v;         // [n_models][P] Adam exp_avg_sq
  int* step;            // [n_models] optimizer step counters (device side)
  float* grad_out;      // MODE_GRAD: [n_models][P] gradients then [n_models] mean losses
  float* loss_log;      // [loss_log_cap][n_models] mean loss per step (nullable)
  int* status;          // [16] error / timeout words (xGMI mode), nullable
  float* const* peers;  // MODE_XGMI_*: [world] device pointers of every rank's receive buffer
  unsigned* epoch;      // MODE_XGMI_*: [n_models] exchange epoch counters (device)
  float* wsp;           // [n_models][dtp_mlp_workspace_floats] scalar-weight workspace (scratch)
  int loss_log_cap;
  int n_models;
  int n_steps;
  int loss;             // DtpLoss
  int cache_data;       // stage the dataset in LDS (persistent multi-step runs)
  int timeout_us;       // bound on every cross-GPU spin (xGMI)
  int bf16;             // bf16 compute instance (fp32 master weights / Adam), toy shapes
  int host_t0;          // >= 0: the step number of the first step (= the device counters), else read them
  dtp::SamplerCfg smp;
  DtpHyper hp;
  // Adam bias-correction scalars {lr / (1 - b1^t), sqrt(1 - b2^t)} of step t at [t], formed on
  // the host in f64 (torch's math); [len - 1] holds the saturated values (every later t).
  // Nullable: the kernel forms them itself.  Used with host_t0 >= 0 (the persistent engine).
  const float* adam_tab;  // [adam_tab_len][2]
  int adam_tab_len;
  int xbuf_bytes;  // MODE_XGMI_*: bytes of each rank's receive buffer (0: unchecked)
  // split-batch step (grp_core.h): the engine's own exchange buffer, epoch counters and
  // timeout words; groups = workgroups per model.  Filled by dtp_train_engine_create; on
  // input groups is the caller's request: 0 the measured policy, 1 on, -1 off.
  void* grp_buf;
  unsigned* grp_epoch;
  int* grp_status;
  int groups;
  int pad3_;
};

int dtp_version(void);
const char* dtp_last_error(void);
int dtp_mlp_supported(int in, int h, int nl, int out, int final_act);
int dtp_mlp_supported_bf16(int in, int h, int nl, int out, int final_act);
int dtp_mlp_param_count(int in, int h, int nl, int out);
int dtp_mlp_workspace_floats(int in, int h, int nl, int out);
int dtp_mlp_train_bf16_supported(int in, int h, int nl, int out);
int dtp_mlp_train(const DtpTrainArgs* a, int in, int h, int nl, int out, int mode, void* stream);
int dtp_mlp_train_profile(const DtpTrainArgs* a, void* stream);
int dtp_mlp_train_profile_lanes(const DtpTrainArgs* a, int lanes, void* stream);
// lanes per sample of the step instance these arguments select (mlp_lanes.h), 0: none
int dtp_mlp_train_lanes(const DtpTrainArgs* a, int in, int h, int nl, int out, int mode);
long long dtp_xgmi_fused_buffer_bytes(int P, int n_models, int world);

// ---- stage forward / backward (autograd path, layer-split pipeline) ----
struct DtpStageArgs {
  const float* x;         // [B][IN]
  const float* params;    // [P]
  float* out;             // [B][OUT]  (forward output; read by backward when FINAL_ACT)
  float* saved;           // [B][(NL-1)*H] hidden activations
  const float* grad_out;  // [B][OUT]  (backward)
  float* grad_in;         // [B][IN]   (backward, nullable)
  float* grad_params;     // [P]       (backward; must be zeroed when the grid has >1 block and !accumulate)
  float* out_peer;        // [B][OUT]  forward: second copy of the output stored straight into
                          //           the next stage's GPU (peer-mapped over xGMI), nullable
  int batch;
  float slope;
  int accumulate;  // backward: add into grad_params (a persistent .grad view) instead of overwriting it
  int bf16;        // bf16 compute (Stage<..., BF>: bf16 operands, fp32 accumulation and weight gradients)
};

int dtp_mlp_stage_fwd(const DtpStageArgs* a, int in, int h, int nl, int out, int final_act, void* stream);
// up to DTP_STAGE_MULTI_MAX models of one shape forward in ONE launch
#define DTP_STAGE_MULTI_MAX 4
struct DtpStageMulti {
  DtpStageArgs stage[DTP_STAGE_MULTI_MAX];
  int n;
  int pad_;
};
int dtp_mlp_stage_fwd_multi(const DtpStageMulti* m, int in, int h, int nl, int out, int final_act, void* stream);
int dtp_mlp_stage_bwd(const DtpStageArgs* a, int in, int h, int nl, int out, int final_act, void* stream);

// ---- persistent layer-split pipeline stage (split_train.hip) ----
// One stage of a model split by layers over several GPUs, resident for n_steps
// iterations: the stage's activation goes to the next stage and the input gradient
// back to the previous one as epoch-tagged granules stored straight into the
// neighbour GPU's receive buffer (peer-mapped over xGMI); the stage's weight
// gradient is (optionally) all-reduced over the data-parallel ranks in-kernel and
// the optimizer is fused.
struct DtpSplitStageArgs {
  const float* X;         // [n][IN of the model]  dataset inputs (first stage)
  const float* Y;         // [n][OUT of the model] targets (last stage)
  float* params;          // [P] this stage's parameters (torch order)
  float* opt_m;           // [P] Adam exp_avg / SGD momentum
  float* opt_v;           // [P] Adam exp_avg_sq
  int* step;              // [1] optimizer step counter (device)
  float* loss_log;        // [loss_log_cap] global mean loss per step (last stage), nullable
  int* status;            // [16]: [0,1] stage-link timeout flag / epoch, [2,3] data-parallel exchange
  void* act_in;           // receive buffer of the incoming activation (not the first stage), local
  void* act_out;          // the next stage's act_in, peer-mapped (not the last stage)
  void* grad_in;          // receive buffer of the incoming output gradient (not the last stage), local
  void* grad_out;         // the previous stage's grad_in, peer-mapped (not the first stage)
  float* const* dp_peers; // [dp_world] this stage's exchange buffers on every DP rank (dp_world > 1)
  int loss_log_cap;
  int n_steps;
  int timeout_us;
  int cache_data;
  int dp_world;
  int dp_rank;
  int optim;              // DTP_MODE_ADAM or DTP_MODE_SGD
  int link_local;         // bit 0: the previous stage, bit 1: the next stage is on this GPU;
                          // bit 2: every neighbour stage runs in this launch (split_lanes.hip plain links)
                          // (device-scope link: plain device memory, sc1); else system scope
  dtp::SamplerCfg smp;
  DtpHyper hp;            // grad_scale = 1 / dp_world
  // split-batch stages (split_lanes.hip, members > 1 on one rank): the stage's on-chip
  // member exchange buffer ([2][members][slot16] granules, zeroed), nullable
  void* grp_buf;
};

#define DTP_SPLIT_MAX_LOCAL 8
// the stages placed on one GPU, launched together (one workgroup each)
struct DtpSplitLaunch {
  DtpSplitStageArgs stage[DTP_SPLIT_MAX_LOCAL];
  int shape_id[DTP_SPLIT_MAX_LOCAL];  // dtp_split_shape_id of each stage
  int n;
  int members;  // split_lanes.hip: workgroups per stage (the stage's batch in member slices); else unused
};

int dtp_split_launch(const DtpSplitLaunch* L, void* stream);
int dtp_split_shape_id(int in, int h, int nl, int out, int final_act, int first);
long long dtp_split_link_bytes(int width, int batch);
int dtp_split_stage_supported(int in, int h, int nl, int out, int final_act, int first);
// split-batch stages: every stage's batch over L->members workgroups of the 4-lanes schedule
int dtp_split_lanes_launch(const DtpSplitLaunch* L, void* stream);
int dtp_split_lanes_supported(int in, int h, int nl, int out, int final_act, int first);
long long dtp_split_lanes_grp_bytes(int P, int members);

// ---- flat optimizers over [n_models][P] (after an external all-reduce) ----
struct DtpOptArgs {
  float* params;
  float* opt_m;
  float* opt_v;
  int* step;          // [n_models]
  const float* grad;  // [n_models][P] (+ [n_models] losses when loss_log != null)
  float* loss_log;
  int loss_log_cap;
  int n_models;
  int P;
  int kind;           // DTP_MODE_ADAM or DTP_MODE_SGD
  float loss_scale;   // applied to the all-reduced losses (1/world)
  int flags;          // DTP_OPT_ZERO_GRAD: write 0 over every gradient element once read
  DtpHyper hp;
  void* shadow;       // [n_models][shadow_ld] bf16 copy of the updated params, or null
  long long shadow_ld;  // row stride of shadow in elements (>= P)
};

#define DTP_OPT_ZERO_GRAD 1
int dtp_flat_optimizer(const DtpOptArgs* a, void* stream);

// ---- MFMA GEMM with fused Linear epilogues (gemm.hip) ----
#define DTP_DT_F32 0
#define DTP_DT_BF16 1
struct DtpGemmArgs {
  const void* A;      // A(m,k) = A[m*lda+k] (trans_a=0) or A[k*lda+m] (trans_a=1)
  const void* B;      // B(n,k) = B[n*ldb+k] (trans_b=0) or B[k*ldb+n] (trans_b=1)
  void* C;            // [M][ldc], out_dtype
  const float* bias;  // [N] or null
  const void* aux;    // [M][ldaux] (dtype): multiply by LeakyReLU'(aux) (backward through the previous layer)
  long long lda, ldb, ldc, ldaux;
  int M, N, K;
  int dtype;       // DTP_DT_* of A, B, aux
  int out_dtype;   // DTP_DT_* of C
  int trans_a, trans_b;
  int act;         // 1: LeakyReLU(slope) on the result
  int accumulate;  // 1: C += result
  int splitk;      // >1: K split over blocks, f32 atomics into C
  float alpha, slope;
  int vec_a, vec_b;  // set by dtp_gemm (16-byte loads allowed)
  int force_big;     // tests: take the 256x256 bf16 kernel for any layout it supports
  int fast;          // LDS-DMA 256x256 bf16 kernel: 0 auto, 1 whenever its preconditions hold, -1 never
  int pad_;
  void* work;              // split-K partial sums of the 8-phase kernel (splitk = 0: dtp_gemm picks)
  long long work_bytes;
};

int dtp_gemm(const DtpGemmArgs* a, void* stream);
// bytes of DtpGemmArgs::work the call would use with splitk = 0 (0: no split-K plan)
long long dtp_gemm_workspace(const DtpGemmArgs* a);
// out[n] (+)= sum_m X[m*ld+n]  (bias gradients)
int dtp_colsum(const void* X, long long ld, int M, int N, int dtype, float* out, int accumulate, void* stream);

// sampler probe (tests): dataset indices of steps [t0, t0+n_steps), row-major [n_steps][batch], -1 padded
int dtp_sampler_indices(const dtp::SamplerCfg* s, long long t0, int n_steps, int* out, void* stream);

}  // extern "C"
