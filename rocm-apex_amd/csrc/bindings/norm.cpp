// pybind surface of the normalisation kernels: submodule ``_C.fused_layer_norm_cuda`` with the
// reference's function names (csrc/layer_norm_cuda.cpp:259-266) plus RMSNorm entry points.
#include "common.h"
#include "apex_amd/norm_api.h"

namespace apex_amd {

namespace {

void n1_n2(const at::Tensor& x, at::IntArrayRef shape, int64_t& n1, int& n2) {
  const int64_t nd = (int64_t)shape.size();
  TORCH_CHECK(nd >= 1 && x.dim() >= nd, "layer_norm: normalized_shape must be a suffix of the input shape");
  int64_t m = 1;
  for (int64_t i = 0; i < nd; ++i) {
    TORCH_CHECK(x.size(x.dim() - nd + i) == shape[i], "layer_norm: input shape ", x.sizes(),
                " does not end with normalized_shape ", shape);
    m *= shape[i];
  }
  TORCH_CHECK(m <= INT32_MAX, "layer_norm: normalized size too large");
  n2 = (int)m;
  n1 = m ? x.numel() / m : 0;
}

void check_w(const c10::optional<at::Tensor>& w, at::IntArrayRef shape, const at::Tensor& x) {
  if (!w.has_value() || !w->defined()) return;
  TORCH_CHECK(w->sizes().equals(shape), "layer_norm: weight/bias shape must equal normalized_shape");
  TORCH_CHECK(w->device() == x.device(), "layer_norm: weight on a different device");
  TORCH_CHECK(w->is_contiguous(), "layer_norm: weight must be contiguous");
}

const void* ptr_or_null(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
}

std::vector<at::Tensor> fwd_impl(const at::Tensor& input, at::IntArrayRef shape, const c10::optional<at::Tensor>& gamma,
                                 const c10::optional<at::Tensor>& beta, double eps, bool rms,
                                 c10::optional<at::ScalarType> out_dtype) {
  TORCH_CHECK(input.is_cuda(), "layer_norm: input must be a GPU tensor");
  const c10::hip::HIPGuard g(input.get_device());
  at::Tensor x = input.contiguous();
  int64_t n1;
  int n2;
  n1_n2(x, shape, n1, n2);
  check_w(gamma, shape, x);
  check_w(beta, shape, x);
  const bool has_w = gamma.has_value() && gamma->defined();
  if (beta.has_value() && beta->defined())
    TORCH_CHECK(has_w && beta->scalar_type() == gamma->scalar_type(), "layer_norm: bias needs a weight of its dtype");
  const at::ScalarType ot = out_dtype.has_value() ? *out_dtype : x.scalar_type();
  const at::ScalarType wt = has_w ? gamma->scalar_type() : x.scalar_type();
  auto y = at::empty(x.sizes(), x.options().dtype(ot));
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = rms ? at::empty({0}, fopt) : at::empty({n1}, fopt);
  auto invvar = at::empty({n1}, fopt);
  NormFwdArgs a;
  a.x = x.data_ptr();
  a.gamma = ptr_or_null(gamma);
  a.beta = ptr_or_null(beta);
  a.y = y.data_ptr();
  a.mean = rms ? nullptr : mean.data_ptr<float>();
  a.invvar = invvar.data_ptr<float>();
  a.n1 = n1;
  a.n2 = n2;
  a.eps = (float)eps;
  a.in_t = dtype_code(x.scalar_type());
  a.w_t = dtype_code(wt);
  a.out_t = dtype_code(ot);
  a.rms = rms;
  norm_fwd(a, device_cus(x.get_device()), cur_stream());
  if (rms) return {y, invvar};
  return {y, mean, invvar};
}

std::vector<at::Tensor> bwd_impl(const at::Tensor& dout, const c10::optional<at::Tensor>& mean, const at::Tensor& invvar,
                                 const at::Tensor& input, at::IntArrayRef shape, const c10::optional<at::Tensor>& gamma,
                                 bool has_beta, double /*eps*/, bool rms,
                                 const c10::optional<at::Tensor>& dres = c10::nullopt) {
  TORCH_CHECK(input.is_cuda(), "layer_norm: input must be a GPU tensor");
  const c10::hip::HIPGuard g(input.get_device());
  at::Tensor x = input.contiguous();
  at::Tensor dy = dout.contiguous();
  int64_t n1;
  int n2;
  n1_n2(x, shape, n1, n2);
  TORCH_CHECK(dy.numel() == x.numel(), "layer_norm backward: grad shape mismatch");
  TORCH_CHECK(invvar.scalar_type() == at::kFloat && invvar.numel() == n1, "layer_norm backward: bad invvar");
  if (!rms)
    TORCH_CHECK(mean.has_value() && mean->scalar_type() == at::kFloat && mean->numel() == n1,
                "layer_norm backward: bad mean");
  check_w(gamma, shape, x);
  const bool has_w = gamma.has_value() && gamma->defined();
  const at::ScalarType wt = has_w ? gamma->scalar_type() : x.scalar_type();
  auto dx = at::empty(x.sizes(), x.options());
  at::Tensor dgamma, dbeta, ws;
  const int cus = device_cus(x.get_device());
  if (has_w) {
    dgamma = at::empty(shape, x.options().dtype(wt));
    if (has_beta) dbeta = at::empty(shape, x.options().dtype(wt));
    ws = at::empty({norm_bwd_workspace_floats(n1, n2, cus)}, x.options().dtype(at::kFloat));
  }
  NormBwdArgs a;
  a.dy = dy.data_ptr();
  a.x = x.data_ptr();
  a.mean = rms ? nullptr : mean->data_ptr<float>();
  a.invvar = invvar.data_ptr<float>();
  a.gamma = ptr_or_null(gamma);
  a.dx = dx.data_ptr();
  a.dgamma = has_w ? dgamma.data_ptr() : nullptr;
  a.dbeta = (has_w && has_beta) ? dbeta.data_ptr() : nullptr;
  a.workspace = has_w ? ws.data_ptr<float>() : nullptr;
  a.n1 = n1;
  a.n2 = n2;
  a.in_t = dtype_code(x.scalar_type());
  a.w_t = dtype_code(wt);
  a.out_t = dtype_code(dy.scalar_type());
  a.rms = rms;
  at::Tensor dr;
  if (dres.has_value() && dres->defined()) {
    dr = dres->contiguous();
    TORCH_CHECK(dr.is_cuda() && dr.numel() == x.numel() && dr.scalar_type() == dy.scalar_type(),
                "layer_norm backward: residual gradient must match the output gradient");
    a.dres = dr.data_ptr();
  }
  TORCH_CHECK(a.out_t == a.in_t || a.out_t == a.w_t, "layer_norm backward: grad dtype must be input or weight dtype");
  norm_bwd(a, cus, cur_stream());
  return {dx, dgamma, dbeta};
}

}  // namespace

void bind_norm(pybind11::module_& root) {
  auto m = root.def_submodule("fused_layer_norm_cuda", "gfx950 LayerNorm / RMSNorm (register-resident rows)");
  m.def("forward_affine",
        [](at::Tensor x, std::vector<int64_t> shape, at::Tensor gamma, c10::optional<at::Tensor> beta, double eps,
           c10::optional<at::ScalarType> out_dtype) { return fwd_impl(x, shape, gamma, beta, eps, false, out_dtype); },
        pybind11::arg("input"), pybind11::arg("normalized_shape"), pybind11::arg("gamma"), pybind11::arg("beta"),
        pybind11::arg("epsilon"), pybind11::arg("out_dtype") = c10::nullopt);
  m.def("forward_affine_mixed_dtypes",
        [](at::Tensor x, std::vector<int64_t> shape, at::Tensor gamma, c10::optional<at::Tensor> beta, double eps) {
          return fwd_impl(x, shape, gamma, beta, eps, false, gamma.scalar_type());
        });
  m.def("forward", [](at::Tensor x, std::vector<int64_t> shape, double eps) {
    return fwd_impl(x, shape, c10::nullopt, c10::nullopt, eps, false, c10::nullopt);
  });
  m.def("backward_affine",
        [](at::Tensor dout, at::Tensor mean, at::Tensor invvar, at::Tensor x, std::vector<int64_t> shape,
           at::Tensor gamma, c10::optional<at::Tensor> beta, double eps, c10::optional<at::Tensor> dres) {
          return bwd_impl(dout, mean, invvar, x, shape, gamma, beta.has_value() && beta->defined(), eps, false, dres);
        },
        pybind11::arg("dout"), pybind11::arg("mean"), pybind11::arg("invvar"), pybind11::arg("input"),
        pybind11::arg("normalized_shape"), pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("epsilon"),
        pybind11::arg("dres") = c10::nullopt);
  m.def("backward", [](at::Tensor dout, at::Tensor mean, at::Tensor invvar, at::Tensor x, std::vector<int64_t> shape,
                       double eps) {
    return bwd_impl(dout, mean, invvar, x, shape, c10::nullopt, false, eps, false)[0];
  });
  m.def("rms_forward_affine",
        [](at::Tensor x, std::vector<int64_t> shape, at::Tensor gamma, double eps,
           c10::optional<at::ScalarType> out_dtype) { return fwd_impl(x, shape, gamma, c10::nullopt, eps, true, out_dtype); },
        pybind11::arg("input"), pybind11::arg("normalized_shape"), pybind11::arg("gamma"), pybind11::arg("epsilon"),
        pybind11::arg("out_dtype") = c10::nullopt);
  m.def("rms_forward_affine_mixed_dtypes", [](at::Tensor x, std::vector<int64_t> shape, at::Tensor gamma, double eps) {
    return fwd_impl(x, shape, gamma, c10::nullopt, eps, true, gamma.scalar_type());
  });
  m.def("rms_forward", [](at::Tensor x, std::vector<int64_t> shape, double eps) {
    return fwd_impl(x, shape, c10::nullopt, c10::nullopt, eps, true, c10::nullopt);
  });
  m.def("rms_backward_affine", [](at::Tensor dout, at::Tensor invvar, at::Tensor x, std::vector<int64_t> shape,
                                  at::Tensor gamma, double eps) {
    auto r = bwd_impl(dout, c10::nullopt, invvar, x, shape, gamma, false, eps, true);
    return std::vector<at::Tensor>{r[0], r[1]};
  });
  m.def("rms_backward", [](at::Tensor dout, at::Tensor invvar, at::Tensor x, std::vector<int64_t> shape, double eps) {
    return bwd_impl(dout, c10::nullopt, invvar, x, shape, c10::nullopt, false, eps, true)[0];
  });
}

}  // namespace apex_amd
