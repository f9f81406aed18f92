// pybind surface of the multi-tensor ops.  Function names and argument orders follow the
// reference's amp_C module (csrc/amp_C_frontend.cpp:147-174) so existing callers of
// `multi_tensor_applier(amp_C.multi_tensor_adam, ...)` work unchanged; the *_capturable /
// *_fused variants are MI355X additions (device-resident lr/step/scale, sync-free skip).
#include "common.h"

namespace apex_amd {

using TL = std::vector<std::vector<at::Tensor>>;

static int* noop_ptr(const at::Tensor& noop) {
  TORCH_CHECK(noop.is_cuda() && noop.scalar_type() == at::kInt && noop.numel() >= 1,
              "noop_flag must be a 1-element int32 GPU tensor");
  return noop.data_ptr<int>();
}

static bool prepare(const TL& tl) {
  if (tl.empty() || tl[0].empty()) return false;
  return true;
}

void multi_tensor_scale(int chunk_size, at::Tensor noop, TL tl, double scale) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 2, "multi_tensor_scale expects 2 lists");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  mt_scale(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), noop_ptr(noop),
           DevScalar{(float)scale, nullptr}, make_launch(tl[0][0]));
}

// scale read from a device tensor (sync-free unscale)
void multi_tensor_scale_t(int chunk_size, at::Tensor noop, TL tl, at::Tensor scale) {
  if (!prepare(tl)) return;
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  mt_scale(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), noop_ptr(noop),
           dev_scalar(scale, 1.f), make_launch(tl[0][0]));
}

void multi_tensor_axpby(int chunk_size, at::Tensor noop, TL tl, double a, double b, int64_t arg_to_check) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 3, "multi_tensor_axpby expects 3 lists");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  mt_axpby(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()),
           dtype_code(tl[2][0].scalar_type()), noop_ptr(noop), (float)a, (float)b, (int)arg_to_check,
           make_launch(tl[0][0]));
}

void multi_tensor_check_finite(int chunk_size, at::Tensor noop, TL tl) {
  if (!prepare(tl)) return;
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  TL one{tl[0]};
  auto m = mta_meta(one, chunk_size);
  mt_check_finite(m, dtype_code(tl[0][0].scalar_type()), noop_ptr(noop), make_launch(tl[0][0]));
}

static std::tuple<at::Tensor, at::Tensor> norm_impl(int chunk_size, at::Tensor noop, const TL& tl, bool per_tensor,
                                                    int mode, bool skip, const c10::optional<at::Tensor>& scale_t,
                                                    float scale) {
  auto opts = at::TensorOptions().dtype(at::kFloat).device(noop.device());
  if (!prepare(tl)) return {at::zeros({1}, opts), at::zeros({0}, opts)};
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  auto total = at::empty({1}, opts);
  auto pt = per_tensor ? at::empty({(int64_t)tl[0].size()}, opts) : at::empty({0}, opts);
  const int out_t = tl.size() > 1 ? dtype_code(tl[1][0].scalar_type()) : -1;
  mt_norm(m, dtype_code(tl[0][0].scalar_type()), out_t, noop_ptr(noop), total.data_ptr<float>(),
          per_tensor ? pt.data_ptr<float>() : nullptr, mode, skip, dev_scalar(scale_t, scale), false, 0.f, 0.f,
          make_launch(tl[0][0]));
  return {total, pt};
}

std::tuple<at::Tensor, at::Tensor> multi_tensor_l2norm(int chunk_size, at::Tensor noop, TL tl,
                                                       c10::optional<bool> per_tensor) {
  TL one;
  if (!tl.empty()) one.push_back(tl[0]);
  return norm_impl(chunk_size, noop, one, per_tensor.value_or(false), 0, false, c10::nullopt, 1.f);
}

std::tuple<at::Tensor, at::Tensor> multi_tensor_l2norm_mp(int chunk_size, at::Tensor noop, TL tl,
                                                          c10::optional<bool> per_tensor) {
  TL one;
  if (!tl.empty()) one.push_back(tl[0]);
  return norm_impl(chunk_size, noop, one, per_tensor.value_or(false), 0, true, c10::nullopt, 1.f);
}

std::tuple<at::Tensor, at::Tensor> multi_tensor_maxnorm(int chunk_size, at::Tensor noop, TL tl,
                                                        c10::optional<bool> per_tensor) {
  TL one;
  if (!tl.empty()) one.push_back(tl[0]);
  return norm_impl(chunk_size, noop, one, per_tensor.value_or(false), 1, false, c10::nullopt, 1.f);
}

std::tuple<at::Tensor, at::Tensor> multi_tensor_l2norm_scale(int chunk_size, at::Tensor noop, TL tl, double scale,
                                                             c10::optional<bool> per_tensor) {
  TORCH_CHECK(tl.size() == 2, "multi_tensor_l2norm_scale expects 2 lists");
  return norm_impl(chunk_size, noop, tl, per_tensor.value_or(false), 0, false, c10::nullopt, (float)scale);
}

// per-tensor norm blended into `out` (reference multi_tensor_norm_out_cuda; norm_type 0 = inf, else L2)
void multi_tensor_norm_out(int chunk_size, at::Tensor noop, TL tl, at::Tensor out, double alpha, double beta,
                           int64_t norm_type) {
  if (!prepare(tl)) return;
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  TL one{tl[0]};
  auto m = mta_meta(one, chunk_size);
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() == (int64_t)tl[0].size(),
              "norm_out: out must be float32 [ntensors]");
  mt_norm(m, dtype_code(tl[0][0].scalar_type()), -1, noop_ptr(noop), nullptr, out.data_ptr<float>(),
          norm_type == 0 ? 1 : 0, false, DevScalar{1.f, nullptr}, true, (float)alpha, (float)beta,
          make_launch(tl[0][0]));
}

void multi_tensor_adam(int chunk_size, at::Tensor noop, TL tl, double lr, double beta1, double beta2, double eps,
                       int64_t step, int64_t mode, int64_t bias_correction, double weight_decay) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 4 || tl.size() == 5, "multi_tensor_adam expects 4 (g,p,m,v) or 5 lists");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  AdamArgs a{};
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.weight_decay = (float)weight_decay;
  a.lr = DevScalar{(float)lr, nullptr};
  a.inv_scale = DevScalar{1.f, nullptr};
  a.step_dev = nullptr;
  a.bias_correction = (int)bias_correction;
  a.bc1 = bias_correction ? (float)(1.0 - std::pow(beta1, (double)step)) : 1.f;
  a.bc2 = bias_correction ? (float)(1.0 - std::pow(beta2, (double)step)) : 1.f;
  a.mode = (int)mode;
  a.skip_on_noop = false;
  const int out_t = tl.size() == 5 ? dtype_code(tl[4][0].scalar_type()) : -1;
  mt_adam(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), out_t, noop_ptr(noop), a,
          make_launch(tl[0][0]));
}

// Sync-free / capturable Adam: lr, step, inv_scale on device; skips the whole step when
// noop (the amp skip flag) is set.  lists: g, p(fp32), m, v [, p_model]
void multi_tensor_adam_capturable(int chunk_size, at::Tensor noop, TL tl, at::Tensor lr, double beta1, double beta2,
                                  double eps, at::Tensor step, int64_t mode, int64_t bias_correction,
                                  double weight_decay, c10::optional<at::Tensor> inv_scale) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 4 || tl.size() == 5, "multi_tensor_adam_capturable expects 4 or 5 lists");
  TORCH_CHECK(step.scalar_type() == at::kFloat && step.is_cuda(), "step must be a float32 GPU tensor");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  AdamArgs a{};
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.weight_decay = (float)weight_decay;
  a.lr = dev_scalar(lr, 0.f);
  a.inv_scale = dev_scalar(inv_scale, 1.f);
  a.step_dev = step.data_ptr<float>();
  a.bias_correction = (int)bias_correction;
  a.bc1 = a.bc2 = 1.f;
  a.mode = (int)mode;
  a.skip_on_noop = true;
  const int out_t = tl.size() == 5 ? dtype_code(tl[4][0].scalar_type()) : -1;
  mt_adam(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), out_t, noop_ptr(noop), a,
          make_launch(tl[0][0]));
}

void multi_tensor_adam_undo(int chunk_size, at::Tensor noop, TL tl, at::Tensor lr, double beta1, double beta2,
                            double eps, at::Tensor step, int64_t mode, int64_t bias_correction, double weight_decay,
                            c10::optional<at::Tensor> inv_scale) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 4 || tl.size() == 5, "multi_tensor_adam_undo expects 4 or 5 lists");
  TORCH_CHECK(tl[1][0].scalar_type() == at::kFloat, "multi_tensor_adam_undo: fp32 master params required");
  TORCH_CHECK(step.scalar_type() == at::kFloat && step.is_cuda(), "step must be a float32 GPU tensor");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  AdamArgs a{};
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.weight_decay = (float)weight_decay;
  a.lr = dev_scalar(lr, 0.f);
  a.inv_scale = dev_scalar(inv_scale, 1.f);
  a.step_dev = step.data_ptr<float>();
  a.bias_correction = (int)bias_correction;
  a.bc1 = a.bc2 = 1.f;
  a.mode = (int)mode;
  a.skip_on_noop = true;
  const int out_t = tl.size() == 5 ? dtype_code(tl[4][0].scalar_type()) : -1;
  mt_adam_undo(m, dtype_code(tl[0][0].scalar_type()), out_t, noop_ptr(noop), a, make_launch(tl[0][0]));
}

void multi_tensor_sgd(int chunk_size, at::Tensor noop, TL tl, double wd, double momentum, double dampening,
                      double lr, bool nesterov, bool first_run, bool wd_after_momentum, double scale) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 3 || tl.size() == 4, "multi_tensor_sgd expects 3 or 4 lists");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  SgdArgs a{};
  a.wd = (float)wd;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.lr = DevScalar{(float)lr, nullptr};
  a.scale = DevScalar{(float)scale, nullptr};
  a.nesterov = nesterov;
  a.first_run = first_run;
  a.wd_after_momentum = wd_after_momentum;
  const int out_t = tl.size() == 4 ? dtype_code(tl[3][0].scalar_type()) : -1;
  mt_sgd(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), out_t, noop_ptr(noop), a,
         make_launch(tl[0][0]));
}

void multi_tensor_sgd_capturable(int chunk_size, at::Tensor noop, TL tl, double wd, double momentum,
                                 double dampening, at::Tensor lr, bool nesterov, bool first_run,
                                 bool wd_after_momentum, c10::optional<at::Tensor> scale) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 3 || tl.size() == 4, "multi_tensor_sgd expects 3 or 4 lists");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  SgdArgs a{};
  a.wd = (float)wd;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.lr = dev_scalar(lr, 0.f);
  a.scale = dev_scalar(scale, 1.f);
  a.nesterov = nesterov;
  a.first_run = first_run;
  a.wd_after_momentum = wd_after_momentum;
  const int out_t = tl.size() == 4 ? dtype_code(tl[3][0].scalar_type()) : -1;
  mt_sgd(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), out_t, noop_ptr(noop), a,
         make_launch(tl[0][0]));
}

void multi_tensor_adagrad(int chunk_size, at::Tensor noop, TL tl, double lr, double eps, int64_t mode,
                          double weight_decay) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 3, "multi_tensor_adagrad expects 3 lists");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  mt_adagrad(m, dtype_code(tl[0][0].scalar_type()), noop_ptr(noop), (float)lr, (float)eps, (int)mode,
             (float)weight_decay, make_launch(tl[0][0]));
}

void multi_tensor_novograd(int chunk_size, at::Tensor noop, TL tl, at::Tensor grad_norms, double lr, double beta1,
                           double beta2, double eps, int64_t step, int64_t bias_correction, double weight_decay,
                           int64_t grad_averaging, int64_t mode, int64_t norm_type) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 3, "multi_tensor_novograd expects 3 lists");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  // blend the new per-tensor grad norms into grad_norms (alpha = beta2, beta = 1 - beta2)
  multi_tensor_norm_out(chunk_size, noop, TL{tl[0]}, grad_norms, beta2, 1.0 - beta2, norm_type);
  auto m = mta_meta(tl, chunk_size);
  NovoArgs a{};
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.beta3 = grad_averaging == 1 ? (float)(1.0 - beta1) : 1.f;
  a.bc1 = bias_correction ? (float)(1.0 - std::pow(beta1, (double)step)) : 1.f;
  a.bc2 = bias_correction ? (float)std::sqrt(1.0 - std::pow(beta2, (double)step)) : 1.f;
  a.eps = (float)eps;
  a.lr = (float)lr;
  a.weight_decay = (float)weight_decay;
  a.mode = (int)mode;
  a.grad_norms = grad_norms.data_ptr<float>();
  mt_novograd(m, dtype_code(tl[0][0].scalar_type()), noop_ptr(noop), a, make_launch(tl[0][0]));
}

static void lamb_impl(int chunk_size, at::Tensor noop, const TL& tl, DevScalar lr, double beta1, double beta2,
                      double eps, const float* step_dev, double step_host, int64_t bias_correction, double wd,
                      int64_t grad_averaging, int64_t mode, at::Tensor global_grad_norm, DevScalar max_grad_norm,
                      bool use_nvlamb, bool skip, DevScalar inv_scale) {
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  const int nt = (int)tl[0].size();
  auto opts = at::TensorOptions().dtype(at::kFloat).device(tl[0][0].device());
  auto norms = at::empty({2, nt}, opts);
  LambArgs a{};
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.beta3 = grad_averaging == 1 ? (float)(1.0 - beta1) : 1.f;
  a.eps = (float)eps;
  a.weight_decay = (float)wd;
  a.lr = lr;
  a.step_dev = step_dev;
  a.bias_correction = (int)bias_correction;
  a.bc1 = bias_correction ? (float)(1.0 - std::pow(beta1, step_host)) : 1.f;
  a.bc2 = bias_correction ? (float)(1.0 - std::pow(beta2, step_host)) : 1.f;
  a.mode = (int)mode;
  TORCH_CHECK(global_grad_norm.scalar_type() == at::kFloat && global_grad_norm.is_cuda(),
              "global_grad_norm must be a float32 GPU tensor");
  a.global_grad_norm = global_grad_norm.data_ptr<float>();
  a.max_grad_norm = max_grad_norm;
  a.inv_scale = inv_scale;
  a.use_nvlamb = use_nvlamb;
  a.skip_on_noop = skip;
  a.param_norm = norms.data_ptr<float>();
  a.update_norm = norms.data_ptr<float>() + nt;
  const auto L = make_launch(tl[0][0]);
  TL s1{tl[0], tl[1], tl[2], tl[3]};
  auto m1 = mta_meta(s1, chunk_size);
  mt_lamb_stage1(m1, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), noop_ptr(noop), a, L);
  TL s2{tl[0], tl[1]};
  if (tl.size() == 5) s2.push_back(tl[4]);
  auto m2 = mta_meta(s2, chunk_size);
  const int out_t = tl.size() == 5 ? dtype_code(tl[4][0].scalar_type()) : -1;
  mt_lamb_stage2(m2, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), out_t, noop_ptr(noop),
                 a, L);
}

void multi_tensor_lamb(int chunk_size, at::Tensor noop, TL tl, double lr, double beta1, double beta2, double eps,
                       int64_t step, int64_t bias_correction, double weight_decay, int64_t grad_averaging,
                       int64_t mode, at::Tensor global_grad_norm, double max_grad_norm,
                       c10::optional<bool> use_nvlamb) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 4, "multi_tensor_lamb expects 4 lists");
  lamb_impl(chunk_size, noop, tl, DevScalar{(float)lr, nullptr}, beta1, beta2, eps, nullptr, (double)step,
            bias_correction, weight_decay, grad_averaging, mode, global_grad_norm,
            DevScalar{(float)max_grad_norm, nullptr}, use_nvlamb.value_or(false), false, DevScalar{1.f, nullptr});
}

// reference multi_tensor_lamb_mp: device lr/step, found_inf (skip), inv_scale (fused unscale),
// optional 5th list = low-precision model params written back.
void multi_tensor_lamb_mp(int chunk_size, at::Tensor noop, TL tl, at::Tensor lr, double beta1, double beta2,
                          double eps, at::Tensor step, int64_t bias_correction, double weight_decay,
                          int64_t grad_averaging, int64_t mode, at::Tensor global_grad_norm,
                          at::Tensor max_grad_norm, c10::optional<bool> use_nvlamb, at::Tensor found_inf,
                          at::Tensor inv_scale) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 4 || tl.size() == 5, "multi_tensor_lamb_mp expects 4 or 5 lists");
  at::Tensor stepf = step.scalar_type() == at::kFloat ? step : step.to(at::kFloat);
  at::Tensor fi = found_inf.scalar_type() == at::kInt ? found_inf : found_inf.to(at::kInt);
  // found_inf doubles as the skip flag; noop still receives overflow reports
  at::Tensor skipflag = fi;
  (void)noop;
  lamb_impl(chunk_size, skipflag, tl, dev_scalar(lr, 0.f), beta1, beta2, eps, stepf.data_ptr<float>(), 1.0,
            bias_correction, weight_decay, grad_averaging, mode, global_grad_norm, dev_scalar(max_grad_norm, 0.f),
            use_nvlamb.value_or(false), true, dev_scalar(inv_scale, 1.f));
}

void multi_tensor_lamb_stage1_cuda(int chunk_size, at::Tensor noop, TL tl, at::Tensor per_tensor_decay,
                                   int64_t step, double beta1, double beta2, double eps, at::Tensor global_grad_norm,
                                   double max_global_grad_norm, c10::optional<double> beta3) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 5, "multi_tensor_lamb_stage1 expects 5 lists (g, p, m, v, update)");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  const float bc1 = (float)(1.0 - std::pow(beta1, (double)step));
  const float bc2 = (float)(1.0 - std::pow(beta2, (double)step));
  mt_lamb_legacy_stage1(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), noop_ptr(noop),
                        per_tensor_decay.data_ptr<float>(), (float)beta1, (float)beta2,
                        (float)beta3.value_or(1.0 - beta1), bc1, bc2, (float)eps,
                        global_grad_norm.data_ptr<float>(), (float)max_global_grad_norm, make_launch(tl[0][0]));
}

void multi_tensor_lamb_stage2_cuda(int chunk_size, at::Tensor noop, TL tl, at::Tensor per_tensor_param_norm,
                                   at::Tensor per_tensor_update_norm, double lr, double weight_decay,
                                   c10::optional<bool> use_nvlamb) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 2 || tl.size() == 3, "multi_tensor_lamb_stage2 expects 2 or 3 lists (p, update[, out])");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  const int out_t = tl.size() == 3 ? dtype_code(tl[2][0].scalar_type()) : -1;
  mt_lamb_legacy_stage2(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), out_t,
                        noop_ptr(noop),
                        per_tensor_param_norm.data_ptr<float>(), per_tensor_update_norm.data_ptr<float>(), (float)lr,
                        (float)weight_decay, use_nvlamb.value_or(false), make_launch(tl[0][0]));
}

// capturable legacy pair (DistributedFusedLAMB): `skip` int32 device flag gates both launches,
// step / lr are fp32 device scalars — no host value per step, no sync
void multi_tensor_lamb_stage1_capturable(int chunk_size, at::Tensor skip, TL tl, at::Tensor per_tensor_decay,
                                         at::Tensor step, bool bias_correction, double beta1, double beta2,
                                         double eps, at::Tensor global_grad_norm, double max_global_grad_norm,
                                         double beta3) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 5, "multi_tensor_lamb_stage1_capturable expects 5 lists (g, p, m, v, update)");
  TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kFloat && step.numel() == 1, "step: fp32 [1] device tensor");
  TORCH_CHECK(skip.is_cuda() && skip.scalar_type() == at::kInt && skip.numel() >= 1, "skip: int32 device flag");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  mt_lamb_legacy_stage1(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), noop_ptr(skip),
                        per_tensor_decay.data_ptr<float>(), (float)beta1, (float)beta2, (float)beta3, 1.f, 1.f,
                        (float)eps, global_grad_norm.data_ptr<float>(), (float)max_global_grad_norm,
                        make_launch(tl[0][0]), step.data_ptr<float>(), bias_correction ? 1 : 0);
}

void multi_tensor_lamb_stage2_capturable(int chunk_size, at::Tensor skip, TL tl, at::Tensor per_tensor_param_norm,
                                         at::Tensor per_tensor_update_norm, at::Tensor lr, double weight_decay,
                                         bool use_nvlamb) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 2 || tl.size() == 3, "multi_tensor_lamb_stage2_capturable expects 2 or 3 lists");
  TORCH_CHECK(lr.is_cuda() && lr.scalar_type() == at::kFloat && lr.numel() == 1, "lr: fp32 [1] device tensor");
  TORCH_CHECK(skip.is_cuda() && skip.scalar_type() == at::kInt && skip.numel() >= 1, "skip: int32 device flag");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  const int out_t = tl.size() == 3 ? dtype_code(tl[2][0].scalar_type()) : -1;
  mt_lamb_legacy_stage2(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), out_t,
                        noop_ptr(skip), per_tensor_param_norm.data_ptr<float>(),
                        per_tensor_update_norm.data_ptr<float>(), 0.f, (float)weight_decay, use_nvlamb,
                        make_launch(tl[0][0]), lr.data_ptr<float>());
}

void multi_tensor_cast(int chunk_size, at::Tensor noop, TL tl) {
  if (!prepare(tl)) return;
  TORCH_CHECK(tl.size() == 2, "multi_tensor_cast expects 2 lists");
  const c10::hip::HIPGuard g(tl[0][0].get_device());
  auto m = mta_meta(tl, chunk_size);
  mt_cast(m, dtype_code(tl[0][0].scalar_type()), dtype_code(tl[1][0].scalar_type()), noop_ptr(noop),
          make_launch(tl[0][0]));
}

// state = float32[4] {scale, inv_scale_used, unskipped, skipped_total}
void amp_update_scale_(at::Tensor overflow, at::Tensor skip_flag, at::Tensor state, double growth_factor,
                       double backoff_factor, int64_t growth_interval, double min_scale, double max_scale,
                       bool dynamic) {
  TORCH_CHECK(state.scalar_type() == at::kFloat && state.numel() >= 4, "state must be float32[4]");
  const c10::hip::HIPGuard g(state.get_device());
  amp_update_scale(overflow.data_ptr<int>(), skip_flag.data_ptr<int>(), state.data_ptr<float>(), (float)growth_factor,
                   (float)backoff_factor, (int)growth_interval, (float)min_scale, (float)max_scale, dynamic,
                   cur_stream());
}

void mta_cache_clear();
int64_t mta_cache_size();

void bind_amp_C(pybind11::module_& root) {
  auto m = root.def_submodule("amp_C", "multi-tensor ops (HIP, gfx950)");
  m.def("multi_tensor_scale", &multi_tensor_scale, "out = in*scale with overflow check");
  m.def("multi_tensor_scale_t", &multi_tensor_scale_t, "out = in*scale (device scale tensor)");
  m.def("multi_tensor_axpby", &multi_tensor_axpby, "out = a*x + b*y");
  m.def("multi_tensor_check_finite", &multi_tensor_check_finite, "noop |= any non-finite");
  m.def("multi_tensor_l2norm", &multi_tensor_l2norm, "L2 norm (total, per tensor)", pybind11::arg("chunk_size"),
        pybind11::arg("noop_flag"), pybind11::arg("tensor_lists"), pybind11::arg("per_tensor") = c10::nullopt);
  m.def("multi_tensor_l2norm_mp", &multi_tensor_l2norm_mp, "L2 norm; no-op when noop_flag set",
        pybind11::arg("chunk_size"), pybind11::arg("noop_flag"), pybind11::arg("tensor_lists"),
        pybind11::arg("per_tensor") = c10::nullopt);
  m.def("multi_tensor_maxnorm", &multi_tensor_maxnorm, "max-abs norm", pybind11::arg("chunk_size"),
        pybind11::arg("noop_flag"), pybind11::arg("tensor_lists"), pybind11::arg("per_tensor") = c10::nullopt);
  m.def("multi_tensor_l2norm_scale", &multi_tensor_l2norm_scale, "L2 norm of input + scaled copy",
        pybind11::arg("chunk_size"), pybind11::arg("noop_flag"), pybind11::arg("tensor_lists"), pybind11::arg("scale"),
        pybind11::arg("per_tensor") = c10::nullopt);
  m.def("multi_tensor_norm_out", &multi_tensor_norm_out, "blend per-tensor norms into out");
  m.def("multi_tensor_adam", &multi_tensor_adam, "Adam/AdamW");
  m.def("multi_tensor_adam_capturable", &multi_tensor_adam_capturable, "Adam with device lr/step/inv_scale");
  m.def("multi_tensor_sgd", &multi_tensor_sgd, "SGD + momentum");
  m.def("multi_tensor_sgd_capturable", &multi_tensor_sgd_capturable, "SGD with device lr/scale");
  m.def("multi_tensor_adagrad", &multi_tensor_adagrad, "Adagrad");
  m.def("multi_tensor_novograd", &multi_tensor_novograd, "NovoGrad");
  m.def("multi_tensor_lamb", &multi_tensor_lamb, "LAMB", pybind11::arg("chunk_size"), pybind11::arg("noop_flag"),
        pybind11::arg("tensor_lists"), pybind11::arg("lr"), pybind11::arg("beta1"), pybind11::arg("beta2"),
        pybind11::arg("epsilon"), pybind11::arg("step"), pybind11::arg("bias_correction"),
        pybind11::arg("weight_decay"), pybind11::arg("grad_averaging"), pybind11::arg("mode"),
        pybind11::arg("global_grad_norm"), pybind11::arg("max_grad_norm"),
        pybind11::arg("use_nvlamb_python") = c10::nullopt);
  m.def("multi_tensor_lamb_mp", &multi_tensor_lamb_mp, "LAMB with device lr/step, found_inf and inv_scale");
  m.def("multi_tensor_adam_undo", &multi_tensor_adam_undo, "invert the last Adam step in place");
  m.def("multi_tensor_lamb_stage1_cuda", &multi_tensor_lamb_stage1_cuda, "legacy LAMB stage 1",
        pybind11::arg("chunk_size"), pybind11::arg("noop_flag"), pybind11::arg("tensor_lists"),
        pybind11::arg("per_tensor_decay"), pybind11::arg("step"), pybind11::arg("beta1"), pybind11::arg("beta2"),
        pybind11::arg("epsilon"), pybind11::arg("global_grad_norm"), pybind11::arg("max_global_grad_norm"),
        pybind11::arg("beta3") = c10::nullopt);
  m.def("multi_tensor_lamb_stage2_cuda", &multi_tensor_lamb_stage2_cuda, "legacy LAMB stage 2");
  m.def("multi_tensor_lamb_stage1_capturable", &multi_tensor_lamb_stage1_capturable,
        "legacy LAMB stage 1, skip-gated, device step");
  m.def("multi_tensor_lamb_stage2_capturable", &multi_tensor_lamb_stage2_capturable,
        "legacy LAMB stage 2, skip-gated, device lr");
  m.def("multi_tensor_cast", &multi_tensor_cast, "out = in (dtype conversion)");
  m.def("amp_update_scale_", &amp_update_scale_, "device-side dynamic loss scale update");
  m.def("mta_cache_clear", &mta_cache_clear, "drop cached multi-tensor work tables");
  m.def("mta_cache_size", &mta_cache_size, "number of cached multi-tensor work tables");
}

}  // namespace apex_amd
