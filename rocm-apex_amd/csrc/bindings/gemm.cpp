// pybind surface of the MFMA GEMM:
//   _C.gemm.matmul(...)          generic C = op(A) op(B) (+ epilogue), any of the 4 major-ness combos
//   _C.gemm.column_sum(x)        bias gradients
//   _C.fused_dense_cuda.*        the reference's module (csrc/fused_dense.cpp:20-190):
//       linear_bias_forward / linear_bias_backward / linear_gelu_linear_forward / _backward
// Every GEMM of a Linear layer (forward, input gradient, weight gradient) is one launch of the
// same kernel family; no operand is transposed in memory.
#include "common.h"
#include "apex_amd/gemm_api.h"

namespace apex_amd {

namespace {

using OT = c10::optional<at::Tensor>;
bool has(const OT& t) { return t.has_value() && t->defined(); }

// C[M][N] = A(M x K) B(K x N); see gemm_api.h for the major-ness conventions.
at::Tensor run_gemm(const at::Tensor& a, bool a_kmajor, const at::Tensor& b, bool b_kmajor, int64_t m, int64_t n,
                    int64_t k, int epilogue, const OT& bias, const OT& aux_in, at::Tensor* aux_out,
                    at::Tensor* colsum_out = nullptr, at::ScalarType colsum_t = at::kFloat) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda(), "gemm: GPU tensors expected");
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous(), "gemm: contiguous operands expected");
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), "gemm: operand dtype mismatch");
  auto c = at::empty({m, n}, a.options());
  GemmArgs g{};
  g.a = a.data_ptr();
  g.b = b.data_ptr();
  g.c = c.data_ptr();
  g.m = (int)m;
  g.n = (int)n;
  g.k = (int)k;
  g.a_kmajor = a_kmajor;
  g.b_kmajor = b_kmajor;
  g.lda = a_kmajor ? k : m;
  g.ldb = b_kmajor ? k : n;
  g.ldc = n;
  g.dtype = dtype_code(a.scalar_type());
  g.epilogue = epilogue;
  at::Tensor bias_c, aux_c;
  if (has(bias)) {
    bias_c = bias->contiguous().to(a.scalar_type());
    TORCH_CHECK(bias_c.numel() == n, "gemm: bias size mismatch");
    g.bias = bias_c.data_ptr();
  }
  if (has(aux_in)) {
    aux_c = aux_in->contiguous();
    TORCH_CHECK(aux_c.numel() == m * n && aux_c.scalar_type() == a.scalar_type(), "gemm: aux_in mismatch");
    g.aux_in = aux_c.data_ptr();
  }
  if (aux_out != nullptr) {
    *aux_out = at::empty({m, n}, a.options());
    g.aux_out = aux_out->data_ptr();
  }
  TORCH_CHECK(gemm_supported(g), "gemm: unsupported shape/alignment/dtype (need fp16/bf16, K, N multiples of 8, "
              "16-byte aligned operands)");
  const int cus = device_cus(a.get_device());
  at::Tensor ws;  // split-K partials (weight gradients with few output tiles); caching allocator
  const int64_t wsf = gemm_splitk_workspace_floats(g, cus);
  const char* sk = std::getenv("APEX_AMD_SPLITK");  // =off disables (A/B timing)
  if (wsf > 0 && !(sk != nullptr && sk[0] == 'o')) {
    ws = at::empty({wsf}, a.options().dtype(at::kFloat));
    g.splitk_ws = ws.data_ptr<float>();
  }
  at::Tensor cpart;
  const bool fused_cs = colsum_out != nullptr && gemm_colsum_fusable(g, cus);
  if (fused_cs) {
    // column sums of C in the epilogue: one fp32 row per 256-row tile, then a fixed-order fold
    cpart = at::empty({(m + 255) / 256, n}, a.options().dtype(at::kFloat));
    g.colpart = cpart.data_ptr<float>();
  }
  gemm_mfma(g, cus, cur_stream());
  if (colsum_out != nullptr) {
    *colsum_out = at::empty({n}, a.options().dtype(colsum_t));
    if (fused_cs) {
      column_sum_finalize(cpart.data_ptr<float>(), (int)cpart.size(0), (int)n, colsum_out->data_ptr(),
                          dtype_code(colsum_t), cur_stream());
    } else {
      auto cws = at::empty({column_sum_workspace_floats(m, (int)n, cus)}, a.options().dtype(at::kFloat));
      column_sum(c.data_ptr(), dtype_code(c.scalar_type()), m, (int)n, n, colsum_out->data_ptr(), dtype_code(colsum_t),
                 cws.data_ptr<float>(), cus, cur_stream());
    }
  }
  return c;
}

at::Tensor colsum(const at::Tensor& x2d, at::ScalarType out_t) {
  const c10::hip::HIPGuard g(x2d.get_device());
  at::Tensor x = x2d.contiguous();
  const int64_t m = x.size(0), n = x.size(1);
  auto out = at::empty({n}, x.options().dtype(out_t));
  const int cus = device_cus(x.get_device());
  auto ws = at::empty({column_sum_workspace_floats(m, n, cus)}, x.options().dtype(at::kFloat));
  column_sum(x.data_ptr(), dtype_code(x.scalar_type()), m, (int)n, n, out.data_ptr(), dtype_code(out_t),
             ws.data_ptr<float>(), cus, cur_stream());
  return out;
}

at::Tensor as2d(const at::Tensor& t) {
  at::Tensor c = t.contiguous();
  return c.view({-1, c.size(-1)});
}

// ---- Linear building blocks (x [M, K], W [N, K]) ----
at::Tensor linear_fwd(const at::Tensor& x2, const at::Tensor& w, const OT& bias, int epi, at::Tensor* aux) {
  return run_gemm(x2, true, w.contiguous(), true, x2.size(0), w.size(0), x2.size(1), epi, bias, c10::nullopt, aux);
}
// dx[M, K] = dy[M, N] W[N, K]   (epilogue may multiply by an activation derivative of aux_in)
at::Tensor linear_dgrad(const at::Tensor& dy2, const at::Tensor& w, int epi, const OT& aux_in) {
  return run_gemm(dy2, true, w.contiguous(), false, dy2.size(0), w.size(1), dy2.size(1), epi, c10::nullopt, aux_in,
                  nullptr);
}
// dW[N, K] = dy[M, N]^T x[M, K]
at::Tensor linear_wgrad(const at::Tensor& dy2, const at::Tensor& x2) {
  return run_gemm(dy2, false, x2, false, dy2.size(1), x2.size(1), dy2.size(0), kEpiNone, c10::nullopt, c10::nullopt,
                  nullptr);
}

}  // namespace

void bind_lt(pybind11::module_& root);  // lt_epilogue.cpp

void bind_gemm(pybind11::module_& root) {
  bind_lt(root);
  namespace py = pybind11;
  auto g = root.def_submodule("gemm", "gfx950 MFMA GEMM with fused epilogues");
  g.attr("EPI_NONE") = (int)kEpiNone;
  g.attr("EPI_GELU") = (int)kEpiGelu;
  g.attr("EPI_RELU") = (int)kEpiRelu;
  g.attr("EPI_SIGMOID") = (int)kEpiSigmoid;
  g.attr("EPI_DGELU") = (int)kEpiDGelu;
  g.attr("EPI_DRELU") = (int)kEpiDRelu;
  g.attr("EPI_DSIGMOID") = (int)kEpiDSigmoid;
  g.def("matmul",
        [](at::Tensor a, bool a_kmajor, at::Tensor b, bool b_kmajor, int64_t m, int64_t n, int64_t k, int epilogue,
           OT bias, OT aux_in, bool want_aux) {
          const c10::hip::HIPGuard guard(a.get_device());
          at::Tensor aux;
          auto c = run_gemm(a.contiguous(), a_kmajor, b.contiguous(), b_kmajor, m, n, k, epilogue, bias, aux_in,
                            want_aux ? &aux : nullptr);
          return std::make_tuple(c, aux);
        },
        py::arg("a"), py::arg("a_kmajor"), py::arg("b"), py::arg("b_kmajor"), py::arg("m"), py::arg("n"),
        py::arg("k"), py::arg("epilogue") = (int)kEpiNone, py::arg("bias") = c10::nullopt,
        py::arg("aux_in") = c10::nullopt, py::arg("want_aux") = false);
  g.def("linear", [](at::Tensor x, at::Tensor w, OT bias, int epi, bool want_aux) {
    const c10::hip::HIPGuard guard(x.get_device());
    at::Tensor aux;
    auto y = linear_fwd(as2d(x), w, bias, epi, want_aux ? &aux : nullptr);
    return std::make_tuple(y, aux);
  });
  g.def("linear_dgrad", [](at::Tensor dy, at::Tensor w, int epi, OT aux_in) {
    const c10::hip::HIPGuard guard(dy.get_device());
    return linear_dgrad(as2d(dy), w, epi, aux_in);
  });
  g.def("linear_wgrad", [](at::Tensor dy, at::Tensor x) {
    const c10::hip::HIPGuard guard(dy.get_device());
    return linear_wgrad(as2d(dy), as2d(x));
  });
  g.def("linear_dgrad_bgrad", [](at::Tensor dy, at::Tensor w, int epi, at::Tensor aux_in,
                                 c10::optional<at::ScalarType> out_dtype) {
    // (dz, db): dz = (dy W) * act'(aux_in) with db = column sums of the stored dz in the GEMM's
    // epilogue (the reference's DGELU_BGRAD, csrc/fused_dense_cuda.cu:977) — no pass over dz
    const c10::hip::HIPGuard guard(dy.get_device());
    at::Tensor d = as2d(dy), db;
    auto dz = run_gemm(d, true, w.contiguous(), false, d.size(0), w.size(1), d.size(1), epi, c10::nullopt, aux_in,
                       nullptr, &db, out_dtype.value_or(d.scalar_type()));
    return std::make_tuple(dz, db);
  }, py::arg("dy"), py::arg("w"), py::arg("epilogue"), py::arg("aux_in"), py::arg("out_dtype") = c10::nullopt);
  g.def("dgelu_column_sum", [](at::Tensor dy, at::Tensor aux, c10::optional<at::ScalarType> out_dtype) {
    // (dz, db): dz = dy * gelu_tanh'(aux), db = column sums of dz — one pass
    const c10::hip::HIPGuard guard(dy.get_device());
    at::Tensor d = as2d(dy), a = as2d(aux);
    TORCH_CHECK(d.sizes() == a.sizes() && d.scalar_type() == a.scalar_type(), "dgelu_column_sum: shape mismatch");
    const int64_t m = d.size(0), n = d.size(1);
    auto dz = at::empty_like(d);
    const at::ScalarType ot = out_dtype.value_or(d.scalar_type());
    auto db = at::empty({n}, d.options().dtype(ot));
    const int cus = device_cus(d.get_device());
    auto ws = at::empty({column_sum_workspace_floats(m, n, cus)}, d.options().dtype(at::kFloat));
    dgelu_column_sum(d.data_ptr(), a.data_ptr(), dz.data_ptr(), dtype_code(d.scalar_type()), m, (int)n, db.data_ptr(),
                     dtype_code(ot), ws.data_ptr<float>(), cus, cur_stream());
    return std::make_tuple(dz, db);
  }, pybind11::arg("dy"), pybind11::arg("aux"), pybind11::arg("out_dtype") = c10::nullopt);
  g.def("gelu", [](at::Tensor z) {
    // y = gelu_tanh(z) (the tanh approximation of the reference's cuBLASLt GELU epilogue)
    const c10::hip::HIPGuard guard(z.get_device());
    at::Tensor zc = z.contiguous();
    auto y = at::empty_like(zc);
    gelu_tanh_forward(zc.data_ptr(), y.data_ptr(), dtype_code(zc.scalar_type()), zc.numel(), device_cus(zc.get_device()),
                      cur_stream());
    return y;
  });
  g.def("column_sum", [](at::Tensor x, c10::optional<at::ScalarType> out_dtype) {
    return colsum(as2d(x), out_dtype.value_or(x.scalar_type()));
  }, py::arg("x"), py::arg("out_dtype") = c10::nullopt);

  auto fd = root.def_submodule("fused_dense_cuda", "fused dense (GEMM + bias [+ GeLU]) on gfx950 MFMA");
  fd.def("linear_bias_forward", [](at::Tensor input, at::Tensor weight, OT bias) {
    const c10::hip::HIPGuard guard(input.get_device());
    return linear_fwd(as2d(input), weight, bias, kEpiNone, nullptr);
  });
  fd.def("linear_bias_backward", [](at::Tensor input, at::Tensor weight, at::Tensor grad_output) {
    const c10::hip::HIPGuard guard(input.get_device());
    auto x2 = as2d(input), dy2 = as2d(grad_output);
    auto dx = linear_dgrad(dy2, weight, kEpiNone, c10::nullopt);
    auto dw = linear_wgrad(dy2, x2);
    auto db = colsum(dy2, weight.scalar_type());
    return std::vector<at::Tensor>{dx, dw, db};
  });
  fd.def("linear_gelu_linear_forward",
         [](at::Tensor input, at::Tensor w1, at::Tensor b1, at::Tensor w2, at::Tensor b2) {
           const c10::hip::HIPGuard guard(input.get_device());
           at::Tensor gelu_in;
           auto out1 = linear_fwd(as2d(input), w1, b1, kEpiGelu, &gelu_in);
           auto out2 = linear_fwd(out1, w2, b2, kEpiNone, nullptr);
           return std::vector<at::Tensor>{out1, out2, gelu_in};
         });
  fd.def("linear_gelu_linear_backward", [](at::Tensor input, at::Tensor gelu_in, at::Tensor output1, at::Tensor w1,
                                           at::Tensor w2, at::Tensor grad_output) {
    const c10::hip::HIPGuard guard(input.get_device());
    auto x2 = as2d(input), dy2 = as2d(grad_output);
    auto dw2 = linear_wgrad(dy2, output1);
    auto db2 = colsum(dy2, w2.scalar_type());
    // (dy W2) * gelu'(pre-activation), its column sums (db1) in the same epilogue
    at::Tensor db1;
    auto dh = run_gemm(dy2, true, w2.contiguous(), false, dy2.size(0), w2.size(1), dy2.size(1), kEpiDGelu,
                       c10::nullopt, gelu_in, nullptr, &db1, w1.scalar_type());
    auto dw1 = linear_wgrad(dh, x2);
    auto dx = linear_dgrad(dh, w1, kEpiNone, c10::nullopt);
    return std::vector<at::Tensor>{dx, dw1, db1, dw2, db2};
  });
}

}  // namespace apex_amd
