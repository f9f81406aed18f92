// pybind surface of the fused NHWC batch norm: submodule ``_C.bn_nhwc`` used by
// apex.contrib.groupbn.BatchNorm2d_NHWC and apex.models' fused ResNet blocks.  Tensors are the
// dense [M, C] views of NHWC activations (the python layer builds them zero-copy).
#include "common.h"
#include "apex_amd/bn_nhwc_api.h"

namespace apex_amd {

namespace {

using OT = c10::optional<at::Tensor>;
bool has(const OT& t) { return t.has_value() && t->defined(); }
const float* fptr(const OT& t) { return has(t) ? t->data_ptr<float>() : nullptr; }
float* fptr_mut(const OT& t) { return has(t) ? t->data_ptr<float>() : nullptr; }

void check2d(const at::Tensor& x, const char* what) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.is_contiguous(), "bn_nhwc: ", what, " must be a contiguous [M, C] GPU tensor");
  TORCH_CHECK(x.size(1) % 8 == 0, "bn_nhwc: C must be a multiple of 8");
  TORCH_CHECK(((uintptr_t)x.data_ptr() & 15u) == 0, "bn_nhwc: ", what, " must be 16-byte aligned");
}

void check_param(const OT& t, int64_t c) {
  if (!has(t)) return;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() == c && t->is_contiguous(),
              "bn_nhwc: weight/bias/running stats must be contiguous fp32 [C]");
}

std::vector<at::Tensor> fwd_train(at::Tensor x, OT z, OT w, OT b, OT running_mean, OT running_var, double momentum,
                                  double eps, bool relu, bool want_mask) {
  TORCH_CHECK(!want_mask || relu, "bn_nhwc: the ReLU bit mask needs relu=True");
  check2d(x, "input");
  const c10::hip::HIPGuard g(x.get_device());
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  for (const OT* p : {&w, &b, &running_mean, &running_var}) check_param(*p, c);
  if (has(z)) {
    check2d(*z, "z");
    TORCH_CHECK(z->sizes() == x.sizes() && z->scalar_type() == x.scalar_type(), "bn_nhwc: z must match input");
  }
  const int cus = device_cus(x.get_device());
  int64_t wsf = 0;
  const int gy = bn_nhwc_plan(m, c, cus, &wsf);
  auto fo = x.options().dtype(at::kFloat);
  auto ws = at::empty({wsf}, fo);
  auto save_mean = at::empty({c}, fo), save_invstd = at::empty({c}, fo), coef = at::empty({2, c}, fo);
  auto y = at::empty_like(x);
  const int dt = dtype_code(x.scalar_type());
  bn_nhwc_stats(x.data_ptr(), dt, m, c, fptr(w), fptr(b), (float)eps, (float)momentum, fptr_mut(running_mean),
                fptr_mut(running_var), save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                coef.data_ptr<float>(), ws.data_ptr<float>(), gy, cus, cur_stream());
  at::Tensor mask;
  if (want_mask) mask = at::empty({m * c / 8}, x.options().dtype(at::kByte));
  bn_nhwc_apply(x.data_ptr(), dt, has(z) ? z->data_ptr() : nullptr, coef.data_ptr<float>(), relu, y.data_ptr(), m, c,
                cus, cur_stream(), want_mask ? mask.data_ptr<uint8_t>() : nullptr);
  return {y, save_mean, save_invstd, coef, mask};
}

// y = relu(bn(x) + bn_z(z)): a residual block whose shortcut is itself conv -> BN (downsampling
// blocks).  Statistics of both inputs, then ONE apply pass for the pair.
std::vector<at::Tensor> fwd_train_dual(at::Tensor x, at::Tensor z, OT w, OT b, OT running_mean, OT running_var,
                                       double momentum, double eps, OT wz, OT bz, OT running_mean_z,
                                       OT running_var_z, double momentum_z, double eps_z, bool want_mask) {
  check2d(x, "input");
  check2d(z, "z");
  TORCH_CHECK(z.sizes() == x.sizes() && z.scalar_type() == x.scalar_type(), "bn_nhwc dual: z must match input");
  const c10::hip::HIPGuard g(x.get_device());
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  for (const OT* p : {&w, &b, &running_mean, &running_var, &wz, &bz, &running_mean_z, &running_var_z})
    check_param(*p, c);
  const int cus = device_cus(x.get_device());
  int64_t wsf = 0;
  const int gy = bn_nhwc_plan(m, c, cus, &wsf);
  auto fo = x.options().dtype(at::kFloat);
  auto ws = at::empty({wsf}, fo);
  auto sm = at::empty({c}, fo), si = at::empty({c}, fo), coef = at::empty({2, c}, fo);
  auto smz = at::empty({c}, fo), siz = at::empty({c}, fo), coefz = at::empty({2, c}, fo);
  const int dt = dtype_code(x.scalar_type());
  bn_nhwc_stats(x.data_ptr(), dt, m, c, fptr(w), fptr(b), (float)eps, (float)momentum, fptr_mut(running_mean),
                fptr_mut(running_var), sm.data_ptr<float>(), si.data_ptr<float>(), coef.data_ptr<float>(),
                ws.data_ptr<float>(), gy, cus, cur_stream());
  bn_nhwc_stats(z.data_ptr(), dt, m, c, fptr(wz), fptr(bz), (float)eps_z, (float)momentum_z, fptr_mut(running_mean_z),
                fptr_mut(running_var_z), smz.data_ptr<float>(), siz.data_ptr<float>(), coefz.data_ptr<float>(),
                ws.data_ptr<float>(), gy, cus, cur_stream());
  at::Tensor mask;
  if (want_mask) mask = at::empty({m * c / 8}, x.options().dtype(at::kByte));
  auto y = at::empty_like(x);
  bn_nhwc_apply_dual(x.data_ptr(), z.data_ptr(), dt, coef.data_ptr<float>(), coefz.data_ptr<float>(), y.data_ptr(),
                     m, c, cus, cur_stream(), want_mask ? mask.data_ptr<uint8_t>() : nullptr);
  return {y, sm, si, coef, smz, siz, coefz, mask};
}

// stem: training BN statistics of x [N, C, H, W] (channels_last), then relu(bn(x)) max-pooled in
// the same pass that normalizes; returns (pooled [N, C, OH, OW] channels_last, 1-byte argmax
// indices, save_mean, save_invstd, coef)
std::vector<at::Tensor> fwd_train_relu_maxpool(at::Tensor x4, OT w, OT b, OT running_mean, OT running_var,
                                               double momentum, double eps, std::vector<int64_t> k,
                                               std::vector<int64_t> st, std::vector<int64_t> pad) {
  TORCH_CHECK(x4.is_cuda() && x4.dim() == 4 && x4.is_contiguous(at::MemoryFormat::ChannelsLast),
              "bn_nhwc apply+pool: channels_last 4-D GPU input expected");
  TORCH_CHECK(k.size() == 2 && st.size() == 2 && pad.size() == 2, "bn_nhwc apply+pool: 2-D window expected");
  const c10::hip::HIPGuard g(x4.get_device());
  const int n = (int)x4.size(0), c = (int)x4.size(1), h = (int)x4.size(2), wd = (int)x4.size(3);
  at::Tensor x = x4.permute({0, 2, 3, 1}).reshape({-1, c});
  check2d(x, "input");
  for (const OT* p : {&w, &b, &running_mean, &running_var}) check_param(*p, c);
  const int64_t m = x.size(0);
  const int cus = device_cus(x.get_device());
  int64_t wsf = 0;
  const int gy = bn_nhwc_plan(m, c, cus, &wsf);
  auto fo = x.options().dtype(at::kFloat);
  auto ws = at::empty({wsf}, fo);
  auto sm = at::empty({c}, fo), si = at::empty({c}, fo), coef = at::empty({2, c}, fo);
  const int dt = dtype_code(x.scalar_type());
  bn_nhwc_stats(x.data_ptr(), dt, m, c, fptr(w), fptr(b), (float)eps, (float)momentum, fptr_mut(running_mean),
                fptr_mut(running_var), sm.data_ptr<float>(), si.data_ptr<float>(), coef.data_ptr<float>(),
                ws.data_ptr<float>(), gy, cus, cur_stream());
  const int oh = (h + 2 * (int)pad[0] - (int)k[0]) / (int)st[0] + 1;
  const int ow = (wd + 2 * (int)pad[1] - (int)k[1]) / (int)st[1] + 1;
  auto opts = x4.options().memory_format(at::MemoryFormat::ChannelsLast);
  auto y = at::empty({n, c, oh, ow}, opts);
  auto idx = at::empty({n, c, oh, ow}, opts.dtype(at::kByte));
  bn_nhwc_apply_relu_maxpool(x.data_ptr(), dt, coef.data_ptr<float>(), n, h, wd, c, (int)k[0], (int)k[1], (int)st[0],
                             (int)st[1], (int)pad[0], (int)pad[1], oh, ow, y.data_ptr(), idx.data_ptr<uint8_t>(), cus,
                             cur_stream());
  return {y, idx, sm, si, coef};
}

at::Tensor fwd_eval(at::Tensor x, OT z, OT w, OT b, at::Tensor running_mean, at::Tensor running_var, double eps,
                    bool relu) {
  check2d(x, "input");
  const c10::hip::HIPGuard g(x.get_device());
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  for (const OT* p : {&w, &b}) check_param(*p, c);
  check_param(running_mean, c);
  check_param(running_var, c);
  auto coef = at::empty({2, c}, x.options().dtype(at::kFloat));
  bn_nhwc_coef_from_stats(running_mean.data_ptr<float>(), running_var.data_ptr<float>(), true, fptr(w), fptr(b),
                          (float)eps, c, coef.data_ptr<float>(), cur_stream());
  auto y = at::empty_like(x);
  bn_nhwc_apply(x.data_ptr(), dtype_code(x.scalar_type()), has(z) ? z->data_ptr() : nullptr, coef.data_ptr<float>(),
                relu, y.data_ptr(), m, c, device_cus(x.get_device()), cur_stream());
  return y;
}

std::vector<at::Tensor> bwd(at::Tensor dy_, at::Tensor x, OT z, OT w, at::Tensor save_mean, at::Tensor save_invstd,
                            at::Tensor coef_fwd, bool relu, bool need_dz, OT dy2_, OT mask_) {
  check2d(x, "input");
  const c10::hip::HIPGuard g(x.get_device());
  at::Tensor dy = dy_.contiguous();
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "bn_nhwc: grad must match input");
  // second gradient of a forked output (both branches of a residual block consumed it): summed
  // in the reduction pass, which then writes the masked sum for the apply pass
  at::Tensor dy2;
  if (has(dy2_)) {
    dy2 = dy2_->contiguous();
    TORCH_CHECK(dy2.sizes() == x.sizes() && dy2.scalar_type() == x.scalar_type(), "bn_nhwc: grad2 must match input");
    if (!relu) {
      dy = dy + dy2;
      dy2 = at::Tensor();
    }
  }
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  const int cus = device_cus(x.get_device());
  int64_t wsf = 0;
  const int gy = bn_nhwc_plan(m, c, cus, &wsf);
  auto fo = x.options().dtype(at::kFloat);
  auto ws = at::empty({wsf}, fo);
  auto gw = at::empty({c}, fo), gb = at::empty({c}, fo), coef_bwd = at::empty({3, c}, fo);
  const bool has_z = has(z);
  // ReLU bit mask from the forward: the masked gradient is written by the reduction pass and the
  // apply pass reads it, so z is never touched
  const bool bits = has(mask_);
  if (bits)
    TORCH_CHECK(relu && mask_->scalar_type() == at::kByte && mask_->numel() * 8 == m * c && mask_->is_contiguous(),
                "bn_nhwc: mask must be a contiguous uint8 [M*C/8] tensor of a relu forward");
  // the residual branch needs the masked gradient itself (grad_z); without it the mask is
  // recomputed in registers by both passes
  at::Tensor dz;
  if (relu && (need_dz || dy2.defined() || bits)) dz = at::empty_like(x);
  const int dt = dtype_code(x.scalar_type());
  bn_nhwc_bwd_reduce(dy.data_ptr(), x.data_ptr(), dt, has_z ? z->data_ptr() : nullptr, coef_fwd.data_ptr<float>(),
                     relu, save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(), fptr(w), gw.data_ptr<float>(),
                     gb.data_ptr<float>(), coef_bwd.data_ptr<float>(), dz.defined() ? dz.data_ptr() : nullptr, m, c,
                     ws.data_ptr<float>(), gy, cus, cur_stream(), dy2.defined() ? dy2.data_ptr() : nullptr,
                     bits ? mask_->data_ptr<uint8_t>() : nullptr);
  auto dx = at::empty_like(x);
  if (dz.defined()) {
    bn_nhwc_bwd_apply(dz.data_ptr(), true, x.data_ptr(), dt, nullptr, coef_fwd.data_ptr<float>(), relu,
                      coef_bwd.data_ptr<float>(), dx.data_ptr(), m, c, cus, cur_stream());
  } else {
    bn_nhwc_bwd_apply(dy.data_ptr(), false, x.data_ptr(), dt, has_z ? z->data_ptr() : nullptr,
                      coef_fwd.data_ptr<float>(), relu, coef_bwd.data_ptr<float>(), dx.data_ptr(), m, c, cus,
                      cur_stream());
    if (need_dz) dz = dy;  // no ReLU: d(z) = dy
  }
  if (!need_dz) dz = at::Tensor();
  return {dx, dz, gw, gb};
}

// ---- bn_group > 1: the python layer exchanges the payloads between the two halves ----------

// forward, step 1: [mean(C) | M2(C) | count] of this rank's batch
at::Tensor fwd_group_local(at::Tensor x) {
  check2d(x, "input");
  const c10::hip::HIPGuard g(x.get_device());
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  const int cus = device_cus(x.get_device());
  int64_t wsf = 0;
  const int gy = bn_nhwc_plan(m, c, cus, &wsf);
  auto fo = x.options().dtype(at::kFloat);
  auto ws = at::empty({wsf}, fo);
  auto payload = at::empty({2 * (int64_t)c + 1}, fo);
  bn_nhwc_stats_local(x.data_ptr(), dtype_code(x.scalar_type()), m, c, payload.data_ptr<float>(),
                      ws.data_ptr<float>(), gy, cus, cur_stream());
  return payload;
}

// forward, step 2: merge the group's [world, 2C+1] payloads, then normalize (+z, +ReLU, +mask)
std::vector<at::Tensor> fwd_group_finish(at::Tensor x, OT z, at::Tensor gathered, OT w, OT b, OT running_mean,
                                         OT running_var, double momentum, double eps, bool relu, bool want_mask) {
  TORCH_CHECK(!want_mask || relu, "bn_nhwc: the ReLU bit mask needs relu=True");
  check2d(x, "input");
  const c10::hip::HIPGuard g(x.get_device());
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  for (const OT* p : {&w, &b, &running_mean, &running_var}) check_param(*p, c);
  TORCH_CHECK(gathered.is_cuda() && gathered.scalar_type() == at::kFloat && gathered.is_contiguous() &&
                  gathered.dim() == 2 && gathered.size(1) == 2 * (int64_t)c + 1,
              "bn_nhwc: gathered statistics must be a contiguous fp32 [world, 2C+1] GPU tensor");
  if (has(z)) {
    check2d(*z, "z");
    TORCH_CHECK(z->sizes() == x.sizes() && z->scalar_type() == x.scalar_type(), "bn_nhwc: z must match input");
  }
  auto fo = x.options().dtype(at::kFloat);
  auto save_mean = at::empty({c}, fo), save_invstd = at::empty({c}, fo), coef = at::empty({2, c}, fo);
  auto inv_count = at::empty({1}, fo);
  bn_nhwc_stats_merge(gathered.data_ptr<float>(), (int)gathered.size(0), c, fptr(w), fptr(b), (float)eps,
                      (float)momentum, fptr_mut(running_mean), fptr_mut(running_var), save_mean.data_ptr<float>(),
                      save_invstd.data_ptr<float>(), coef.data_ptr<float>(), inv_count.data_ptr<float>(),
                      cur_stream());
  at::Tensor mask;
  if (want_mask) mask = at::empty({m * c / 8}, x.options().dtype(at::kByte));
  auto y = at::empty_like(x);
  bn_nhwc_apply(x.data_ptr(), dtype_code(x.scalar_type()), has(z) ? z->data_ptr() : nullptr, coef.data_ptr<float>(),
                relu, y.data_ptr(), m, c, device_cus(x.get_device()), cur_stream(),
                want_mask ? mask.data_ptr<uint8_t>() : nullptr);
  return {y, save_mean, save_invstd, coef, mask, inv_count};
}

// backward, step 1: local [sum_dy | sum_dy_xmu] payload, local grad_w / grad_b and (when the
// ReLU is fused) the masked gradient the apply pass reads
std::vector<at::Tensor> bwd_group_local(at::Tensor dy_, at::Tensor x, OT z, OT w, at::Tensor save_mean,
                                        at::Tensor save_invstd, at::Tensor coef_fwd, bool relu, OT dy2_, OT mask_) {
  check2d(x, "input");
  const c10::hip::HIPGuard g(x.get_device());
  at::Tensor dy = dy_.contiguous();
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "bn_nhwc: grad must match input");
  at::Tensor dy2;
  if (has(dy2_)) {
    dy2 = dy2_->contiguous();
    TORCH_CHECK(dy2.sizes() == x.sizes() && dy2.scalar_type() == x.scalar_type(), "bn_nhwc: grad2 must match input");
    if (!relu) {
      dy = dy + dy2;
      dy2 = at::Tensor();
    }
  }
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  const int cus = device_cus(x.get_device());
  int64_t wsf = 0;
  const int gy = bn_nhwc_plan(m, c, cus, &wsf);
  auto fo = x.options().dtype(at::kFloat);
  auto ws = at::empty({wsf}, fo);
  auto gw = at::empty({c}, fo), gb = at::empty({c}, fo), payload = at::empty({2 * (int64_t)c}, fo);
  const bool bits = has(mask_);
  if (bits)
    TORCH_CHECK(relu && mask_->scalar_type() == at::kByte && mask_->numel() * 8 == m * c && mask_->is_contiguous(),
                "bn_nhwc: mask must be a contiguous uint8 [M*C/8] tensor of a relu forward");
  // with a fused ReLU the masked gradient is always materialized here (it is grad_z of a
  // residual layer and the apply pass's input), so the second half never needs z
  at::Tensor dym;
  if (relu) dym = at::empty_like(x);
  bn_nhwc_bwd_reduce(dy.data_ptr(), x.data_ptr(), dtype_code(x.scalar_type()), has(z) ? z->data_ptr() : nullptr,
                     coef_fwd.data_ptr<float>(), relu, save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                     fptr(w), gw.data_ptr<float>(), gb.data_ptr<float>(), nullptr,
                     dym.defined() ? dym.data_ptr() : nullptr, m, c, ws.data_ptr<float>(), gy, cus, cur_stream(),
                     dy2.defined() ? dy2.data_ptr() : nullptr, bits ? mask_->data_ptr<uint8_t>() : nullptr,
                     payload.data_ptr<float>());
  return {payload, gw, gb, dym.defined() ? dym : dy};
}

// backward, step 2: dx from the group's sums (`sums` [rows, 2C], summed in row order)
at::Tensor bwd_group_finish(at::Tensor dy_masked, at::Tensor x, at::Tensor sums, at::Tensor inv_count, OT w,
                            at::Tensor save_mean, at::Tensor save_invstd, at::Tensor coef_fwd) {
  check2d(x, "input");
  check2d(dy_masked, "grad");
  const c10::hip::HIPGuard g(x.get_device());
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kFloat && sums.is_contiguous() &&
                  sums.numel() % (2 * (int64_t)c) == 0 && sums.numel() > 0,
              "bn_nhwc: group sums must be a contiguous fp32 [rows, 2C] GPU tensor");
  auto coef_bwd = at::empty({3, c}, x.options().dtype(at::kFloat));
  bn_nhwc_bwd_coef_group(sums.data_ptr<float>(), (int)(sums.numel() / (2 * (int64_t)c)), c,
                         inv_count.data_ptr<float>(), save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                         fptr(w), coef_bwd.data_ptr<float>(), cur_stream());
  auto dx = at::empty_like(x);
  bn_nhwc_bwd_apply(dy_masked.data_ptr(), true, x.data_ptr(), dtype_code(x.scalar_type()), nullptr,
                    coef_fwd.data_ptr<float>(), false, coef_bwd.data_ptr<float>(), dx.data_ptr(), m, c,
                    device_cus(x.get_device()), cur_stream());
  return dx;
}

// group statistics without the apply: merge the [world, 2C+1] payloads -> (save_mean,
// save_invstd, coef [2C], inv_count [1]), running stats updated (the fused bottleneck node
// applies the coefficients inside its convolutions)
std::vector<at::Tensor> stats_group_merge(at::Tensor gathered, OT w, OT b, OT running_mean, OT running_var,
                                          double momentum, double eps) {
  TORCH_CHECK(gathered.is_cuda() && gathered.scalar_type() == at::kFloat && gathered.is_contiguous() &&
                  gathered.dim() == 2 && gathered.size(1) % 2 == 1,
              "bn_nhwc: gathered statistics must be a contiguous fp32 [world, 2C+1] GPU tensor");
  const int c = (int)(gathered.size(1) / 2);
  for (const OT* p : {&w, &b, &running_mean, &running_var}) check_param(*p, c);
  const c10::hip::HIPGuard g(gathered.get_device());
  auto fo = gathered.options();
  auto save_mean = at::empty({c}, fo), save_invstd = at::empty({c}, fo), coef = at::empty({2 * c}, fo);
  auto inv_count = at::empty({1}, fo);
  bn_nhwc_stats_merge(gathered.data_ptr<float>(), (int)gathered.size(0), c, fptr(w), fptr(b), (float)eps,
                      (float)momentum, fptr_mut(running_mean), fptr_mut(running_var), save_mean.data_ptr<float>(),
                      save_invstd.data_ptr<float>(), coef.data_ptr<float>(), inv_count.data_ptr<float>(),
                      cur_stream());
  return {save_mean, save_invstd, coef, inv_count};
}

// group backward from [2, G, C] reduction partials (sum_dy | sum_dy_xmu, e.g. a conv epilogue's):
// (payload [2C], local grad_w, local grad_b)
std::vector<at::Tensor> bwd_part_local(at::Tensor part, at::Tensor save_invstd) {
  TORCH_CHECK(part.is_cuda() && part.dim() == 3 && part.size(0) == 2 && part.is_contiguous() &&
                  part.scalar_type() == at::kFloat,
              "bn_nhwc bwd_part_local: part must be the [2, G, C] fp32 partials");
  const int c = (int)part.size(2);
  check_param(save_invstd, c);
  const c10::hip::HIPGuard g(part.get_device());
  auto fo = part.options();
  auto payload = at::empty({2 * (int64_t)c}, fo), gw = at::empty({c}, fo), gb = at::empty({c}, fo);
  bn_nhwc_bwd_local(part.data_ptr<float>(), (int)part.size(1), c, save_invstd.data_ptr<float>(), gw.data_ptr<float>(),
                    gb.data_ptr<float>(), payload.data_ptr<float>(), cur_stream());
  return {payload, gw, gb};
}

// group backward: coef_bwd [3C] from the group's exchanged sums ([rows, 2C], summed in row order)
at::Tensor bwd_group_coef(at::Tensor sums, at::Tensor inv_count, at::Tensor save_mean, at::Tensor save_invstd, OT w) {
  const int c = (int)save_mean.numel();
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kFloat && sums.is_contiguous() &&
                  sums.numel() % (2 * (int64_t)c) == 0 && sums.numel() > 0,
              "bn_nhwc: group sums must be a contiguous fp32 [rows, 2C] GPU tensor");
  check_param(w, c);
  const c10::hip::HIPGuard g(sums.get_device());
  auto coef = at::empty({3 * (int64_t)c}, sums.options());
  bn_nhwc_bwd_coef_group(sums.data_ptr<float>(), (int)(sums.numel() / (2 * (int64_t)c)), c, inv_count.data_ptr<float>(),
                         save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(), fptr(w), coef.data_ptr<float>(),
                         cur_stream());
  return coef;
}

// statistics only: (save_mean, save_invstd, coef[2, C]) of x, running stats updated in place
std::vector<at::Tensor> stats(at::Tensor x, OT w, OT b, OT running_mean, OT running_var, double momentum, double eps) {
  check2d(x, "input");
  const c10::hip::HIPGuard g(x.get_device());
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  for (const OT* p : {&w, &b, &running_mean, &running_var}) check_param(*p, c);
  const int cus = device_cus(x.get_device());
  int64_t wsf = 0;
  const int gy = bn_nhwc_plan(m, c, cus, &wsf);
  auto fo = x.options().dtype(at::kFloat);
  auto ws = at::empty({wsf}, fo);
  auto sm = at::empty({c}, fo), si = at::empty({c}, fo), coef = at::empty({2, c}, fo);
  bn_nhwc_stats(x.data_ptr(), dtype_code(x.scalar_type()), m, c, fptr(w), fptr(b), (float)eps, (float)momentum,
                fptr_mut(running_mean), fptr_mut(running_var), sm.data_ptr<float>(), si.data_ptr<float>(),
                coef.data_ptr<float>(), ws.data_ptr<float>(), gy, cus, cur_stream());
  return {sm, si, coef};
}

// apply only, with precomputed coefficients: y = act(x * coef[0] + coef[1] (+ z)) (+ ReLU bit mask);
// with z2 / coef_z the downsampling pair y = relu(bn(x) + bn_z(z))
std::vector<at::Tensor> apply(at::Tensor x, OT z, at::Tensor coef, bool relu, bool want_mask, OT coef_z) {
  check2d(x, "input");
  TORCH_CHECK(!want_mask || relu, "bn_nhwc apply: the ReLU bit mask needs relu=True");
  const c10::hip::HIPGuard g(x.get_device());
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() == 2 * (int64_t)c,
              "bn_nhwc apply: coef must be contiguous fp32 [2C]");
  if (has(z)) {
    check2d(*z, "z");
    TORCH_CHECK(z->sizes() == x.sizes() && z->scalar_type() == x.scalar_type(), "bn_nhwc apply: z must match x");
  }
  at::Tensor mask;
  if (want_mask) mask = at::empty({m * c / 8}, x.options().dtype(at::kByte));
  auto y = at::empty_like(x);
  const int cus = device_cus(x.get_device());
  if (has(coef_z)) {
    TORCH_CHECK(has(z) && relu && coef_z->scalar_type() == at::kFloat && coef_z->numel() == 2 * (int64_t)c,
                "bn_nhwc apply: the dual form needs z, relu and coef_z [2C]");
    bn_nhwc_apply_dual(x.data_ptr(), z->data_ptr(), dtype_code(x.scalar_type()), coef.data_ptr<float>(),
                       coef_z->data_ptr<float>(), y.data_ptr(), m, c, cus, cur_stream(),
                       want_mask ? mask.data_ptr<uint8_t>() : nullptr);
  } else {
    bn_nhwc_apply(x.data_ptr(), dtype_code(x.scalar_type()), has(z) ? z->data_ptr() : nullptr, coef.data_ptr<float>(),
                  relu, y.data_ptr(), m, c, cus, cur_stream(), want_mask ? mask.data_ptr<uint8_t>() : nullptr);
  }
  return {y, mask};
}

// reduction only (the ReLU mask recomputed from x, nothing written): (coef [5, C] = coef_bwd [3, C]
// followed by coef_fwd [2, C], grad_w, grad_b) — the operand of a consumer that applies
// dx = A (mask ? dy : 0) + B x + K itself (the 1x1 dgrad's recomputed-mask prologue)
std::vector<at::Tensor> bwd_coef(at::Tensor dy_, at::Tensor x, OT w, at::Tensor save_mean, at::Tensor save_invstd,
                                 at::Tensor coef_fwd) {
  check2d(x, "input");
  const c10::hip::HIPGuard g(x.get_device());
  at::Tensor dy = dy_.contiguous();
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "bn_nhwc: grad must match input");
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  TORCH_CHECK(coef_fwd.is_contiguous() && coef_fwd.scalar_type() == at::kFloat && coef_fwd.numel() == 2 * (int64_t)c,
              "bn_nhwc bwd_coef: coef_fwd must be fp32 [2C]");
  const int cus = device_cus(x.get_device());
  int64_t wsf = 0;
  const int gy = bn_nhwc_plan(m, c, cus, &wsf);
  auto fo = x.options().dtype(at::kFloat);
  auto ws = at::empty({wsf}, fo);
  auto gw = at::empty({c}, fo), gb = at::empty({c}, fo), coef = at::empty({5, c}, fo);
  bn_nhwc_bwd_reduce(dy.data_ptr(), x.data_ptr(), dtype_code(x.scalar_type()), nullptr, coef_fwd.data_ptr<float>(), true,
                     save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(), fptr(w), gw.data_ptr<float>(),
                     gb.data_ptr<float>(), coef.data_ptr<float>(), nullptr, m, c, ws.data_ptr<float>(), gy, cus,
                     cur_stream(), nullptr, nullptr);
  coef.narrow(0, 3, 2).view({-1}).copy_(coef_fwd.view({-1}));
  return {coef, gw, gb};
}

// backward reduction only: (dy_masked, coef_bwd[3, C], grad_w, grad_b).  The dx pass is left to
// the consumer (bwd_apply below, or a convolution whose operand prologue computes
// dx = coef_bwd[0] * dy_masked + coef_bwd[1] * x + coef_bwd[2] on load).
std::vector<at::Tensor> bwd_reduce(at::Tensor dy_, at::Tensor x, OT w, at::Tensor save_mean, at::Tensor save_invstd,
                                   at::Tensor coef_fwd, bool relu, OT mask_) {
  check2d(x, "input");
  const c10::hip::HIPGuard g(x.get_device());
  at::Tensor dy = dy_.contiguous();
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "bn_nhwc: grad must match input");
  const int64_t m = x.size(0);
  const int c = (int)x.size(1);
  const int cus = device_cus(x.get_device());
  int64_t wsf = 0;
  const int gy = bn_nhwc_plan(m, c, cus, &wsf);
  auto fo = x.options().dtype(at::kFloat);
  auto ws = at::empty({wsf}, fo);
  auto gw = at::empty({c}, fo), gb = at::empty({c}, fo), coef_bwd = at::empty({3, c}, fo);
  const bool bits = has(mask_);
  if (bits)
    TORCH_CHECK(relu && mask_->scalar_type() == at::kByte && mask_->numel() * 8 == m * c && mask_->is_contiguous(),
                "bn_nhwc: mask must be a contiguous uint8 [M*C/8] tensor of a relu forward");
  at::Tensor dm = relu ? at::empty_like(x) : dy;
  bn_nhwc_bwd_reduce(dy.data_ptr(), x.data_ptr(), dtype_code(x.scalar_type()), nullptr, coef_fwd.data_ptr<float>(), relu,
                     save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(), fptr(w), gw.data_ptr<float>(),
                     gb.data_ptr<float>(), coef_bwd.data_ptr<float>(), relu ? dm.data_ptr() : nullptr, m, c,
                     ws.data_ptr<float>(), gy, cus, cur_stream(), nullptr, bits ? mask_->data_ptr<uint8_t>() : nullptr);
  return {dm, coef_bwd, gw, gb};
}

// dx = coef_bwd[0] * dy_masked + coef_bwd[1] * x + coef_bwd[2]
at::Tensor bwd_apply(at::Tensor dy_masked, at::Tensor x, at::Tensor coef_fwd, at::Tensor coef_bwd) {
  check2d(x, "input");
  check2d(dy_masked, "grad");
  const c10::hip::HIPGuard g(x.get_device());
  auto dx = at::empty_like(x);
  bn_nhwc_bwd_apply(dy_masked.data_ptr(), true, x.data_ptr(), dtype_code(x.scalar_type()), nullptr,
                    coef_fwd.data_ptr<float>(), false, coef_bwd.data_ptr<float>(), dx.data_ptr(), x.size(0),
                    (int)x.size(1), device_cus(x.get_device()), cur_stream());
  return dx;
}

}  // namespace

void bind_bn_nhwc(pybind11::module_& root) {
  auto m = root.def_submodule("bn_nhwc", "gfx950 fused NHWC batch norm (+add+ReLU)");
  m.def("fwd_train", &fwd_train, pybind11::arg("x"), pybind11::arg("z"), pybind11::arg("w"), pybind11::arg("b"),
        pybind11::arg("running_mean"), pybind11::arg("running_var"), pybind11::arg("momentum"), pybind11::arg("eps"),
        pybind11::arg("relu"), pybind11::arg("want_mask") = false);
  m.def("fwd_eval", &fwd_eval);
  m.def("stats", &stats);
  m.def("bwd_reduce", &bwd_reduce);
  m.def("bwd_apply", &bwd_apply);
  m.def("bwd_coef", &bwd_coef);
  m.def("apply", &apply, pybind11::arg("x"), pybind11::arg("z"), pybind11::arg("coef"), pybind11::arg("relu"),
        pybind11::arg("want_mask") = false, pybind11::arg("coef_z") = c10::nullopt);
  m.def("fwd_train_dual", &fwd_train_dual);
  m.def("fwd_train_relu_maxpool", &fwd_train_relu_maxpool);
  m.def("bwd", &bwd, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("z"), pybind11::arg("w"),
        pybind11::arg("save_mean"), pybind11::arg("save_invstd"), pybind11::arg("coef_fwd"), pybind11::arg("relu"),
        pybind11::arg("need_dz"), pybind11::arg("dy2") = c10::nullopt, pybind11::arg("mask") = c10::nullopt);
  m.def("fwd_group_local", &fwd_group_local);
  m.def("fwd_group_finish", &fwd_group_finish);
  m.def("bwd_group_local", &bwd_group_local, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("z"),
        pybind11::arg("w"), pybind11::arg("save_mean"), pybind11::arg("save_invstd"), pybind11::arg("coef_fwd"),
        pybind11::arg("relu"), pybind11::arg("dy2") = c10::nullopt, pybind11::arg("mask") = c10::nullopt);
  m.def("bwd_group_finish", &bwd_group_finish);
  m.def("stats_group_merge", &stats_group_merge);
  m.def("bwd_part_local", &bwd_part_local);
  m.def("bwd_group_coef", &bwd_group_coef);
}

}  // namespace apex_amd
