// pybind surface: submodule ``_C.xentropy_cuda`` (reference apex/contrib/csrc/xentropy/
// interface.cpp:5-52: forward(input, labels, smoothing, half_to_float) -> [losses,
// max_log_sum_exp]; backward(grad_loss, logits, max_log_sum_exp, labels, smoothing)).
// The padding-index masking the reference does in python is folded into the kernels here.
#include "common.h"

namespace apex_amd {

void xentropy_fwd(const void* logits, int dt, const int64_t* labels, float* losses, float* lse, int64_t rows,
                  int classes, float smoothing, int64_t padding_idx, bool use_pad, hipStream_t s);
void xentropy_bwd(const float* grad_loss, const void* logits, int dt, const float* lse, const int64_t* labels,
                  void* grad, int64_t rows, int classes, float smoothing, int64_t padding_idx, bool use_pad,
                  hipStream_t s);

namespace {

std::vector<at::Tensor> fwd(const at::Tensor& input, const at::Tensor& labels_, double smoothing, bool half_to_float,
                            c10::optional<int64_t> padding_idx) {
  TORCH_CHECK(input.is_cuda() && input.dim() == 2, "xentropy: [rows, classes] GPU logits expected");
  const c10::hip::HIPGuard g(input.get_device());
  at::Tensor x = input.contiguous();
  at::Tensor labels = labels_.contiguous().to(at::kLong);
  TORCH_CHECK(labels.numel() == x.size(0), "xentropy: one label per row");
  auto fo = x.options().dtype(at::kFloat);
  auto losses = at::empty({x.size(0)}, fo), lse = at::empty({x.size(0)}, fo);
  xentropy_fwd(x.data_ptr(), dtype_code(x.scalar_type()), labels.data_ptr<int64_t>(), losses.data_ptr<float>(),
               lse.data_ptr<float>(), x.size(0), (int)x.size(1), (float)smoothing, padding_idx.value_or(0),
               padding_idx.has_value(), cur_stream());
  if (!half_to_float && x.scalar_type() != at::kFloat) losses = losses.to(x.scalar_type());
  return {losses, lse};
}

at::Tensor bwd(const at::Tensor& grad_loss, const at::Tensor& logits, const at::Tensor& lse, const at::Tensor& labels_,
               double smoothing, c10::optional<int64_t> padding_idx) {
  const c10::hip::HIPGuard g(logits.get_device());
  at::Tensor x = logits.contiguous();
  at::Tensor gl = grad_loss.contiguous().to(at::kFloat);
  at::Tensor ls = lse.contiguous().to(at::kFloat);
  at::Tensor labels = labels_.contiguous().to(at::kLong);
  auto grad = at::empty_like(x);
  xentropy_bwd(gl.data_ptr<float>(), x.data_ptr(), dtype_code(x.scalar_type()), ls.data_ptr<float>(),
               labels.data_ptr<int64_t>(), grad.data_ptr(), x.size(0), (int)x.size(1), (float)smoothing,
               padding_idx.value_or(0), padding_idx.has_value(), cur_stream());
  return grad;
}

}  // namespace

void bind_xentropy(pybind11::module_& root) {
  namespace py = pybind11;
  auto m = root.def_submodule("xentropy_cuda", "gfx950 softmax cross-entropy with label smoothing");
  m.def("forward", &fwd, py::arg("input"), py::arg("labels"), py::arg("smoothing"), py::arg("half_to_float"),
        py::arg("padding_idx") = c10::nullopt);
  m.def("backward", &bwd, py::arg("grad_loss"), py::arg("logits"), py::arg("max_log_sum_exp"), py::arg("labels"),
        py::arg("smoothing"), py::arg("padding_idx") = c10::nullopt);
}

}  // namespace apex_amd
