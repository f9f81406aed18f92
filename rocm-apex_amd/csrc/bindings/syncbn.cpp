// pybind surface of the batch-norm kernels: submodule ``_C.syncbn`` with the reference's
// function names (csrc/syncbn.cpp:8-109).  c_last entry points take a contiguous tensor whose
// LAST dim is the channel (the python layer hands torch channels_last activations in as a
// permuted zero-copy [N, H, W, C] view); NCHW entry points take [N, C, *] contiguous.
// Fused-ReLU extensions (z / bias / fuse_relu on the backward kernels) let the backward mask
// dy in registers instead of materialising the masked gradient.
#include "common.h"
#include "apex_amd/syncbn_api.h"

namespace apex_amd {

namespace {

using OT = c10::optional<at::Tensor>;

bool has(const OT& t) { return t.has_value() && t->defined(); }

BnShape shape_of(const at::Tensor& x, bool c_last) {
  TORCH_CHECK(x.is_cuda(), "syncbn: input must be a GPU tensor");
  TORCH_CHECK(x.is_contiguous(), "syncbn: input must be contiguous (c_last: channel as the last dim)");
  BnShape sh;
  sh.c_last = c_last;
  if (c_last) {
    sh.c = (int)x.size(-1);
    sh.n = sh.c ? x.numel() / sh.c : 0;
    sh.s = 1;
  } else {
    TORCH_CHECK(x.dim() >= 2, "syncbn: expected [N, C, ...]");
    sh.n = x.size(0);
    sh.c = (int)x.size(1);
    sh.s = (sh.n && sh.c) ? x.numel() / (sh.n * sh.c) : 0;
  }
  return sh;
}

BnParams params(const at::Tensor& mean, const at::Tensor& inv_std, const OT& w, const OT& b, int c) {
  TORCH_CHECK(mean.scalar_type() == at::kFloat && inv_std.scalar_type() == at::kFloat, "syncbn: fp32 stats expected");
  TORCH_CHECK(mean.numel() == c && inv_std.numel() == c, "syncbn: stats size mismatch");
  BnParams p;
  p.mean = mean.data_ptr<float>();
  p.inv_std = inv_std.data_ptr<float>();
  p.w = has(w) ? w->data_ptr() : nullptr;
  p.b = has(b) ? b->data_ptr() : nullptr;
  p.w_t = has(w) ? dtype_code(w->scalar_type()) : (has(b) ? dtype_code(b->scalar_type()) : -1);
  if (has(w) && has(b)) TORCH_CHECK(w->scalar_type() == b->scalar_type(), "syncbn: weight/bias dtype mismatch");
  if (has(w)) TORCH_CHECK(w->numel() == c && w->is_contiguous(), "syncbn: weight size mismatch");
  if (has(b)) TORCH_CHECK(b->numel() == c && b->is_contiguous(), "syncbn: bias size mismatch");
  return p;
}

FusedRelu relu_of(bool on, const OT& z, const at::Tensor& x) {
  FusedRelu r;
  r.on = on;
  if (has(z)) {
    TORCH_CHECK(z->sizes() == x.sizes() && z->scalar_type() == x.scalar_type() && z->is_contiguous(),
                "syncbn: z must match the input");
    r.z = z->data_ptr();
  }
  return r;
}

std::vector<at::Tensor> welford(const at::Tensor& x, bool c_last) {
  const c10::hip::HIPGuard g(x.get_device());
  const BnShape sh = shape_of(x, c_last);
  auto fo = x.options().dtype(at::kFloat);
  auto mean = at::empty({sh.c}, fo), var = at::empty({sh.c}, fo);
  const int cus = device_cus(x.get_device());
  auto ws = at::empty({bn_workspace_floats(sh, cus)}, fo);
  bn_welford(x.data_ptr(), dtype_code(x.scalar_type()), sh, mean.data_ptr<float>(), var.data_ptr<float>(),
             ws.data_ptr<float>(), cus, cur_stream());
  return {mean, var};
}

at::Tensor forward(const at::Tensor& x, const OT& z, const at::Tensor& mean, const at::Tensor& inv_std, const OT& w,
                   const OT& b, bool relu, bool c_last) {
  const c10::hip::HIPGuard g(x.get_device());
  const BnShape sh = shape_of(x, c_last);
  auto y = at::empty_like(x);
  bn_forward(x.data_ptr(), dtype_code(x.scalar_type()), params(mean, inv_std, w, b, sh.c), relu_of(relu, z, x),
             y.data_ptr(), sh, device_cus(x.get_device()), cur_stream());
  return y;
}

std::vector<at::Tensor> reduce(const at::Tensor& dy_, const at::Tensor& x, const at::Tensor& mean,
                               const at::Tensor& inv_std, const OT& w, const OT& z, const OT& b, bool relu,
                               bool c_last) {
  const c10::hip::HIPGuard g(x.get_device());
  const BnShape sh = shape_of(x, c_last);
  at::Tensor dy = dy_.contiguous();
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "syncbn: grad must match input");
  auto fo = x.options().dtype(at::kFloat);
  auto sum_dy = at::empty({sh.c}, fo), sum_dy_xmu = at::empty({sh.c}, fo);
  at::Tensor gw, gb;
  if (has(w)) {
    gw = at::empty({sh.c}, w->options());
    gb = at::empty({sh.c}, w->options());
  }
  const int cus = device_cus(x.get_device());
  auto ws = at::empty({bn_workspace_floats(sh, cus)}, fo);
  BnParams p = params(mean, inv_std, w, b, sh.c);
  bn_reduce(dy.data_ptr(), x.data_ptr(), dtype_code(x.scalar_type()), p, relu_of(relu, z, x),
            sum_dy.data_ptr<float>(), sum_dy_xmu.data_ptr<float>(), has(w) ? gw.data_ptr() : nullptr,
            has(w) ? gb.data_ptr() : nullptr, sh, ws.data_ptr<float>(), cus, cur_stream());
  return {sum_dy, sum_dy_xmu, gw, gb};
}

at::Tensor backward(const at::Tensor& dy_, const at::Tensor& x, const at::Tensor& mean, const at::Tensor& inv_std,
                    const OT& w, const at::Tensor& sum_dy, const at::Tensor& sum_dy_xmu, const at::Tensor& count,
                    const OT& z, const OT& b, bool relu, bool c_last) {
  const c10::hip::HIPGuard g(x.get_device());
  const BnShape sh = shape_of(x, c_last);
  at::Tensor dy = dy_.contiguous();
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "syncbn: grad must match input");
  TORCH_CHECK(count.scalar_type() == at::kInt && count.is_cuda(), "syncbn: count must be an int32 GPU tensor");
  TORCH_CHECK(sum_dy.scalar_type() == at::kFloat && sum_dy_xmu.scalar_type() == at::kFloat, "syncbn: fp32 sums");
  auto dx = at::empty_like(x);
  at::Tensor cnt = count.contiguous();
  bn_backward(dy.data_ptr(), x.data_ptr(), dtype_code(x.scalar_type()), params(mean, inv_std, w, b, sh.c),
              relu_of(relu, z, x), sum_dy.data_ptr<float>(), sum_dy_xmu.data_ptr<float>(), cnt.data_ptr<int>(),
              (int)cnt.numel(), dx.data_ptr(), sh, device_cus(x.get_device()), cur_stream());
  return dx;
}

}  // namespace

void bind_syncbn(pybind11::module_& root) {
  namespace py = pybind11;
  auto m = root.def_submodule("syncbn", "gfx950 batch-norm statistics / apply kernels (SyncBatchNorm)");
  m.def("welford_mean_var", [](at::Tensor x) { return welford(x, false); });
  m.def("welford_mean_var_c_last", [](at::Tensor x) { return welford(x, true); });
  m.def("welford_parallel", [](at::Tensor mean_all, at::Tensor var_all, at::Tensor count_all, double eps) {
    TORCH_CHECK(mean_all.dim() == 2 && var_all.sizes() == mean_all.sizes(), "welford_parallel: [world, C] expected");
    const c10::hip::HIPGuard g(mean_all.get_device());
    auto ma = mean_all.contiguous().to(at::kFloat), va = var_all.contiguous().to(at::kFloat);
    auto ca = count_all.contiguous().to(at::kInt);
    const int world = (int)ma.size(0), c = (int)ma.size(1);
    TORCH_CHECK(ca.numel() == world, "welford_parallel: count size mismatch");
    auto fo = ma.options();
    auto mean = at::empty({c}, fo), var_u = at::empty({c}, fo), inv_std = at::empty({c}, fo);
    bn_welford_parallel(ma.data_ptr<float>(), va.data_ptr<float>(), ca.data_ptr<int>(), world, c, (float)eps,
                        mean.data_ptr<float>(), var_u.data_ptr<float>(), inv_std.data_ptr<float>(), cur_stream());
    return std::vector<at::Tensor>{mean, var_u, inv_std};
  });
  m.def("batchnorm_forward", [](at::Tensor x, at::Tensor mean, at::Tensor inv_std, OT w, OT b) {
    return forward(x, c10::nullopt, mean, inv_std, w, b, false, false);
  });
  m.def("batchnorm_forward_c_last", [](at::Tensor x, OT z, at::Tensor mean, at::Tensor inv_std, OT w, OT b,
                                       bool fuse_relu) { return forward(x, z, mean, inv_std, w, b, fuse_relu, true); },
        py::arg("input"), py::arg("z"), py::arg("mean"), py::arg("inv_std"), py::arg("weight"), py::arg("shift"),
        py::arg("fuse_relu") = false);
  m.def("relu_bw_c_last", [](at::Tensor dy, at::Tensor x, OT z, at::Tensor mean, at::Tensor inv_std, OT w, OT b) {
    const c10::hip::HIPGuard g(x.get_device());
    const BnShape sh = shape_of(x, true);
    at::Tensor d = dy.contiguous();
    auto out = at::empty_like(x);
    bn_relu_backward(d.data_ptr(), x.data_ptr(), dtype_code(x.scalar_type()), params(mean, inv_std, w, b, sh.c),
                     relu_of(true, z, x), out.data_ptr(), sh, device_cus(x.get_device()), cur_stream());
    return out;
  });
  m.def("reduce_bn", [](at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor inv_std, OT w) {
    return reduce(dy, x, mean, inv_std, w, c10::nullopt, c10::nullopt, false, false);
  });
  m.def("reduce_bn_c_last",
        [](at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor inv_std, OT w, OT z, OT b, bool fuse_relu) {
          return reduce(dy, x, mean, inv_std, w, z, b, fuse_relu, true);
        },
        py::arg("grad_output"), py::arg("input"), py::arg("mean"), py::arg("inv_std"), py::arg("weight"),
        py::arg("z") = c10::nullopt, py::arg("shift") = c10::nullopt, py::arg("fuse_relu") = false);
  m.def("batchnorm_backward", [](at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor inv_std, OT w,
                                 at::Tensor sum_dy, at::Tensor sum_dy_xmu, at::Tensor count) {
    return backward(dy, x, mean, inv_std, w, sum_dy, sum_dy_xmu, count, c10::nullopt, c10::nullopt, false, false);
  });
  m.def("batchnorm_backward_c_last",
        [](at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor inv_std, OT w, at::Tensor sum_dy,
           at::Tensor sum_dy_xmu, at::Tensor count, OT z, OT b, bool fuse_relu) {
          return backward(dy, x, mean, inv_std, w, sum_dy, sum_dy_xmu, count, z, b, fuse_relu, true);
        },
        py::arg("grad_output"), py::arg("input"), py::arg("mean"), py::arg("inv_std"), py::arg("weight"),
        py::arg("sum_dy"), py::arg("sum_dy_xmu"), py::arg("count"), py::arg("z") = c10::nullopt,
        py::arg("shift") = c10::nullopt, py::arg("fuse_relu") = false);
}

}  // namespace apex_amd
