// pybind surface of the fused softmax kernels.  Submodule names and signatures follow the
// reference's Megatron extensions (csrc/megatron/scaled_masked_softmax.cpp:84-95,
// csrc/megatron/scaled_upper_triang_masked_softmax.cpp:65-70) plus an unmasked
// ``scaled_softmax_cuda``.  Unlike the reference, backward does not overwrite the incoming
// gradient (it may be shared by autograd) and key lengths up to 16384 stay on the fast path.
#include "common.h"
#include "apex_amd/softmax_api.h"

namespace apex_amd {

namespace {

void check_in(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda(), "softmax: input must be a GPU tensor");
  const auto t = x.scalar_type();
  TORCH_CHECK(t == at::kHalf || t == at::kBFloat16 || t == at::kFloat, "softmax: fp16/bf16/fp32 input expected");
}

at::Tensor fwd(const at::Tensor& input, const c10::optional<at::Tensor>& mask, double scale, int mode) {
  check_in(input);
  const c10::hip::HIPGuard g(input.get_device());
  at::Tensor x = input.contiguous();
  SoftmaxFwdArgs a{};
  if (mode == kMaskCausal) {
    TORCH_CHECK(x.dim() == 3, "scaled_upper_triang_masked_softmax: expected [attn_batches, sq, sk]");
    TORCH_CHECK(x.size(1) == x.size(2), "causal mask is only for self attention (sq == sk)");
    a.sq = (int)x.size(1);
    a.heads = 1;
  } else if (mode == kMaskPad) {
    TORCH_CHECK(x.dim() == 4, "scaled_masked_softmax: expected [b, np, sq, sk]");
    TORCH_CHECK(mask.has_value() && mask->defined(), "scaled_masked_softmax: mask required");
    const auto& m = *mask;
    TORCH_CHECK(m.dim() == 4 && m.size(1) == 1 && m.size(2) == x.size(2) && m.size(3) == x.size(3),
                "scaled_masked_softmax: mask must be [b or 1, 1, sq, sk]");
    TORCH_CHECK(m.size(0) == 1 || m.size(0) == x.size(0), "scaled_masked_softmax: mask batch must be 1 or b");
    a.sq = (int)x.size(2);
    a.heads = (int)x.size(1);
    a.pad_batches = (int)m.size(0);
  } else {
    TORCH_CHECK(x.dim() >= 2, "scaled_softmax: expected >= 2-D input");
    a.sq = x.dim() >= 2 ? (int)x.size(-2) : 1;
    a.heads = 1;
  }
  at::Tensor mk;
  if (mode == kMaskPad) {
    mk = mask->to(at::kByte).contiguous();
    a.mask = mk.data_ptr<uint8_t>();
  }
  auto y = at::empty_like(x);
  a.x = x.data_ptr();
  a.y = y.data_ptr();
  a.sk = (int)x.size(-1);
  a.rows = a.sk ? x.numel() / a.sk : 0;
  a.scale = (float)scale;
  a.mode = mode;
  a.dtype = dtype_code(x.scalar_type());
  if (a.pad_batches == 0) a.pad_batches = 1;
  softmax_fwd(a, cur_stream());
  return y;
}

at::Tensor bwd(const at::Tensor& grad, const at::Tensor& probs, double scale) {
  check_in(probs);
  const c10::hip::HIPGuard g(probs.get_device());
  at::Tensor dy = grad.contiguous().to(probs.scalar_type());
  at::Tensor y = probs.contiguous();
  TORCH_CHECK(dy.sizes() == y.sizes(), "softmax backward: shape mismatch");
  auto dx = at::empty_like(y);
  SoftmaxBwdArgs a{};
  a.dy = dy.data_ptr();
  a.y = y.data_ptr();
  a.dx = dx.data_ptr();
  a.sk = (int)y.size(-1);
  a.rows = a.sk ? y.numel() / a.sk : 0;
  a.scale = (float)scale;
  a.dtype = dtype_code(y.scalar_type());
  softmax_bwd(a, cur_stream());
  return dx;
}

}  // namespace

void bind_softmax(pybind11::module_& root) {
  auto m1 = root.def_submodule("scaled_masked_softmax_cuda", "scale + padding mask + softmax (gfx950)");
  m1.def("forward", [](at::Tensor x, at::Tensor mask, double scale) { return fwd(x, mask, scale, kMaskPad); });
  m1.def("backward", [](at::Tensor g, at::Tensor y, double scale) { return bwd(g, y, scale); });
  // every row is independent here, so any batching works; kept for the reference's API
  m1.def("get_batch_per_block", [](int64_t, int64_t, int64_t, int64_t) { return (int64_t)1; });

  auto m2 = root.def_submodule("scaled_upper_triang_masked_softmax_cuda", "scale + causal mask + softmax (gfx950)");
  m2.def("forward", [](at::Tensor x, double scale) { return fwd(x, c10::nullopt, scale, kMaskCausal); });
  m2.def("backward", [](at::Tensor g, at::Tensor y, double scale) { return bwd(g, y, scale); });

  auto m3 = root.def_submodule("scaled_softmax_cuda", "scale + softmax (gfx950)");
  m3.def("forward", [](at::Tensor x, double scale) { return fwd(x, c10::nullopt, scale, kMaskNone); });
  m3.def("backward", [](at::Tensor g, at::Tensor y, double scale) { return bwd(g, y, scale); });
}

}  // namespace apex_amd
