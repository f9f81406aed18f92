// Host-callable launchers for the multi-tensor ops (implemented in csrc/mta/*.hip).
// This header is torch-free so the device translation units compile fast; the pybind layer
// (csrc/bindings/*.cpp) converts at::Tensor lists into an MtaMeta and calls these.
#pragma once
#include <hip/hip_runtime.h>
#include "apex_amd/mta.h"

namespace apex_amd {

struct Launch {
  hipStream_t stream;
  int max_blocks;  // persistent-grid cap (CUs x resident blocks)
};

// out = in * scale; noop |= !finite(in)   (reference csrc/multi_tensor_scale_kernel.cu:30-111)
// copy a host-built work table to the device through kernel arguments (capture-safe)
void mta_upload_bytes(void* dst, const void* src, size_t bytes, hipStream_t s);

void mt_scale(const MtaMeta& m, int in_t, int out_t, int* noop, DevScalar scale, const Launch& L);
// out = a*x + b*y; arg_to_check: -1 both, 0 x, 1 y   (reference csrc/multi_tensor_axpby_kernel.cu:28-126)
void mt_axpby(const MtaMeta& m, int x_t, int y_t, int out_t, int* noop, float a, float b, int arg_to_check,
              const Launch& L);
// noop |= any(!finite(x))  (fast overflow probe used by sync-free amp)
void mt_check_finite(const MtaMeta& m, int t, int* noop, const Launch& L);

// Norm family.  mode: 0 = L2, 1 = max-abs.  Writes total[0] and, if per_tensor, per_tensor[t].
// out list (depth 2) gets in*scale when out_t >= 0 (l2norm_scale).  skip_on_noop: l2norm_mp.
// blend (norm_out / NovoGrad): per_tensor[t] = sqrt(alpha*old^2 + beta*sumsq) or alpha*old + beta*max.
void mt_norm(const MtaMeta& m, int in_t, int out_t, int* noop, float* total, float* per_tensor, int mode,
             bool skip_on_noop, DevScalar scale, bool blend, float alpha, float beta, const Launch& L);

struct AdamArgs {
  float beta1, beta2, eps, weight_decay;
  DevScalar lr;
  DevScalar inv_scale;      // grads are multiplied by this (fused unscale); 1 if already unscaled
  const float* step_dev;    // device step (after increment) -> bias correction on device; else host
  float bc1, bc2;           // host bias corrections (used when step_dev == nullptr)
  int bias_correction;
  int mode;                 // 0: L2 (Adam), 1: decoupled (AdamW)
  bool skip_on_noop;        // sync-free amp: skip the whole step when *noop != 0
};
// lists: g, p, m, v [, p_model_out]
void mt_adam(const MtaMeta& m, int g_t, int p_t, int out_t, int* noop, const AdamArgs& a, const Launch& L);
// Inverse of one fp32-master Adam step (lists g, p, m, v [, model out]); skipped when *noop.
void mt_adam_undo(const MtaMeta& m, int g_t, int out_t, int* noop, const AdamArgs& a, const Launch& L);

struct SgdArgs {
  float wd, momentum, dampening;
  DevScalar lr;
  DevScalar scale;          // grad scale (reference `scale` arg; 1/loss_scale for fused unscale)
  bool nesterov, first_run, wd_after_momentum;
};
// lists: g, w, mom [, w_model_out]; always skips when *noop != 0 (reference :46)
void mt_sgd(const MtaMeta& m, int g_t, int w_t, int out_t, int* noop, const SgdArgs& a, const Launch& L);

// lists: g, p, h  (reference csrc/multi_tensor_adagrad.cu)
void mt_adagrad(const MtaMeta& m, int t, int* noop, float lr, float eps, int mode, float wd, const Launch& L);

struct NovoArgs {
  float beta1, beta2, beta3, bc1, bc2, eps, lr, weight_decay;
  int mode;
  const float* grad_norms;  // per tensor (already blended)
};
// lists: g, p, m
void mt_novograd(const MtaMeta& m, int t, int* noop, const NovoArgs& a, const Launch& L);

struct LambArgs {
  float beta1, beta2, beta3, eps, weight_decay;
  DevScalar lr;
  const float* step_dev;    // device step (lamb_mp) or null -> bc1/bc2
  float bc1, bc2;
  int bias_correction;
  int mode;                 // 0: L2 on grad, 1: decoupled
  const float* global_grad_norm;
  DevScalar max_grad_norm;
  DevScalar inv_scale;
  bool use_nvlamb;
  bool skip_on_noop;
  float* param_norm;        // [ntensors] out of stage 1
  float* update_norm;       // [ntensors] out of stage 1
};
// Stage 1 (fused with both per-tensor norms): lists g, p, m, v; writes update into g.
void mt_lamb_stage1(const MtaMeta& m, int g_t, int p_t, int* noop, const LambArgs& a, const Launch& L);
// Stage 2: lists update, p [, p_model_out]
void mt_lamb_stage2(const MtaMeta& m, int u_t, int p_t, int out_t, int* noop, const LambArgs& a,
                    const Launch& L);

// Legacy two-kernel LAMB (reference csrc/multi_tensor_lamb_stage_1.cu / _2.cu)
void mt_lamb_legacy_stage1(const MtaMeta& m, int g_t, int p_t, int* noop, const float* per_tensor_decay,
                           float beta1, float beta2, float beta3, float bc1, float bc2, float eps,
                           const float* global_grad_norm, float max_global_grad_norm, const Launch& L,
                           const float* step_dev = nullptr, int bias_correction = 1);
// lists p, update [, model out (16-bit or fp8 copy of the updated p)]
// step_dev / lr_dev non-null: capturable form — skipped entirely while *noop != 0, bias
// corrections from the device step count, learning rate read on the device
void mt_lamb_legacy_stage2(const MtaMeta& m, int p_t, int u_t, int out_t, int* noop,
                           const float* per_tensor_param_norm, const float* per_tensor_update_norm, float lr,
                           float weight_decay, bool use_nvlamb, const Launch& L, const float* lr_dev = nullptr);

// Dynamic loss-scale update, fully on device (sync-free amp).  state = {scale, inv_scale_used,
// unskipped, skipped_total}; skip_flag <- dynamic && overflow.
void amp_update_scale(const int* overflow, int* skip_flag, float* state, float growth_factor, float backoff,
                      int growth_interval, float min_scale, float max_scale, bool dynamic, hipStream_t s);

// contrib: Adam with per-tensor hyper-params / e5m2 copies (DistributedFusedAdam)
void mt_cast(const MtaMeta& m, int in_t, int out_t, int* noop, const Launch& L);

}  // namespace apex_amd
