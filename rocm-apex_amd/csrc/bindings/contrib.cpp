// pybind surface of contrib kernels:
//   _C.transducer_joint_cuda.forward / backward   (reference apex/contrib/csrc/transducer/transducer_joint.cpp)
//   _C.transducer_loss_cuda.forward / backward    (reference apex/contrib/csrc/transducer/transducer_loss.cpp)
#include "common.h"
#include "apex_amd/transducer_api.h"
#include "apex_amd/pool_api.h"

namespace apex_amd {

void bias_dropout_add_fwd(const void* x, const void* bias, const void* res, void* out, int64_t n, int h, int dtype,
                          float p, uint64_t seed, uint64_t offset, int cus, hipStream_t s, const int64_t* step);
void bias_dropout_add_bwd(const void* g, void* dx, int64_t n, int dtype, float p, uint64_t seed, uint64_t offset, int cus,
                          hipStream_t s, const int64_t* step);

void* peer_alloc(size_t bytes, int* kind);
void peer_free(void* p);
std::string peer_handle(void* p);
void* peer_open(const std::string& handle);
void peer_close(void* p);
int peer_max_group();
void peer_allgather(const float* local, int n, int nmax, float* const* bufs, int me, int group, uint32_t epoch,
                    float* out, int* err, double timeout_s, hipStream_t s);

namespace {

// ---- peer memory (hipIpc over xGMI) exchange: csrc/comm/peer.hip ----
pybind11::tuple pm_alloc(int64_t bytes) {
  int kind = 0;
  void* p = peer_alloc((size_t)bytes, &kind);
  return pybind11::make_tuple((int64_t)(uintptr_t)p, kind);
}
void pm_free(int64_t p) { peer_free((void*)(uintptr_t)p); }
pybind11::bytes pm_handle(int64_t p) { return pybind11::bytes(peer_handle((void*)(uintptr_t)p)); }
int64_t pm_open(const std::string& h) { return (int64_t)(uintptr_t)peer_open(h); }
void pm_close(int64_t p) { peer_close((void*)(uintptr_t)p); }

// out[group][n] = every member's `local` [n] (fp32), exchanged through the members' buffers
void pm_allgather(const at::Tensor& local, const std::vector<int64_t>& bufs, int64_t nmax, int64_t me,
                  int64_t epoch, at::Tensor& out, at::Tensor& err, double timeout_s) {
  TORCH_CHECK(local.is_cuda() && local.scalar_type() == at::kFloat && local.is_contiguous(), "peer: fp32 local");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() &&
                  out.numel() == (int64_t)bufs.size() * local.numel(), "peer: out must be [group, n] fp32");
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt, "peer: err must be an int32 GPU tensor");
  const c10::hip::HIPGuard guard(local.get_device());
  std::vector<float*> ptrs;
  for (int64_t b : bufs) ptrs.push_back((float*)(uintptr_t)b);
  peer_allgather(local.data_ptr<float>(), (int)local.numel(), (int)nmax, ptrs.data(), (int)me, (int)bufs.size(),
                 (uint32_t)epoch, out.data_ptr<float>(), err.data_ptr<int>(), timeout_s, cur_stream());
}

// out = residual + dropout(x + bias) with a regenerable counter-hash mask (csrc/transformer/bias_dropout_add.hip)
const int64_t* step_ptr(const c10::optional<at::Tensor>& step) {
  if (!step.has_value() || !step->defined()) return nullptr;
  TORCH_CHECK(step->is_cuda() && step->scalar_type() == at::kLong && step->numel() >= 1,
              "rng_step must be an int64 GPU tensor");
  return step->data_ptr<int64_t>();
}

at::Tensor bda_forward(const at::Tensor& x, const c10::optional<at::Tensor>& bias, const at::Tensor& residual, double p,
                       int64_t seed, int64_t offset, const c10::optional<at::Tensor>& rng_step) {
  TORCH_CHECK(x.is_cuda() && x.sizes() == residual.sizes() && x.scalar_type() == residual.scalar_type(),
              "bias_dropout_add: x and residual must be same-shape GPU tensors");
  const c10::hip::HIPGuard guard(x.get_device());
  at::Tensor xc = x.contiguous(), rc = residual.contiguous();
  at::Tensor bc;
  const int h = (int)x.size(-1);
  if (bias.has_value() && bias->defined()) {
    bc = bias->contiguous().to(x.scalar_type());
    TORCH_CHECK(bc.numel() == h, "bias_dropout_add: bias must have the hidden size");
  }
  at::Tensor out = at::empty_like(xc);
  bias_dropout_add_fwd(xc.data_ptr(), bc.defined() ? bc.data_ptr() : nullptr, rc.data_ptr(), out.data_ptr(), xc.numel(),
                       h, dtype_code(x.scalar_type()), (float)p, (uint64_t)seed, (uint64_t)offset,
                       device_cus(x.get_device()), cur_stream(), step_ptr(rng_step));
  return out;
}

at::Tensor bda_backward(const at::Tensor& g, double p, int64_t seed, int64_t offset,
                        const c10::optional<at::Tensor>& rng_step) {
  const c10::hip::HIPGuard guard(g.get_device());
  at::Tensor gc = g.contiguous();
  at::Tensor dx = at::empty_like(gc);
  bias_dropout_add_bwd(gc.data_ptr(), dx.data_ptr(), gc.numel(), dtype_code(g.scalar_type()), (float)p, (uint64_t)seed,
                       (uint64_t)offset, device_cus(g.get_device()), cur_stream(), step_ptr(rng_step));
  return dx;
}

at::Tensor as_int(const at::Tensor& t) { return t.to(at::kInt).contiguous(); }

struct JointHold {
  JointArgs a{};
  at::Tensor f, g, fl, gl, bo;
};

void joint_setup(JointHold& j, const at::Tensor& f, const at::Tensor& g, const at::Tensor& f_len,
                 const at::Tensor& g_len, const at::Tensor& batch_offset, bool pack_output) {
  TORCH_CHECK(f.is_cuda() && g.is_cuda() && f.dim() == 3 && g.dim() == 3, "transducer joint: f [B,T,H], g [B,U,H]");
  TORCH_CHECK(f.scalar_type() == g.scalar_type(), "transducer joint: dtype mismatch");
  j.f = f.contiguous();
  j.g = g.contiguous();
  j.fl = as_int(f_len);
  j.gl = as_int(g_len);
  JointArgs& a = j.a;
  a.f = j.f.data_ptr();
  a.g = j.g.data_ptr();
  a.f_len = j.fl.data_ptr<int>();
  a.g_len = j.gl.data_ptr<int>();
  a.B = (int)f.size(0);
  a.T = (int)f.size(1);
  a.U = (int)g.size(1);
  a.H = (int)f.size(2);
  a.packed = pack_output;
  if (pack_output) {
    j.bo = batch_offset.to(at::kLong).contiguous();
    a.batch_offset = j.bo.data_ptr<int64_t>();
  }
  a.dtype = dtype_code(f.scalar_type());
}

std::vector<at::Tensor> joint_forward(at::Tensor f, at::Tensor g, at::Tensor f_len, at::Tensor g_len,
                                      at::Tensor batch_offset, int64_t packed_batch, int64_t opt, bool pack_output,
                                      bool relu, bool dropout, double dropout_prob, int64_t tile_size, int64_t seed,
                                      int64_t offset) {
  (void)opt;
  (void)tile_size;
  const c10::hip::HIPGuard guard(f.get_device());
  JointHold j;
  joint_setup(j, f, g, f_len, g_len, batch_offset, pack_output);
  auto shape = pack_output ? std::vector<int64_t>{packed_batch, j.a.H}
                           : std::vector<int64_t>{j.a.B, j.a.T, j.a.U, j.a.H};
  auto out = at::empty(shape, f.options());
  at::Tensor mask;
  if (relu || dropout) {
    mask = at::empty(shape, f.options().dtype(at::kByte));
    j.a.mask = mask.data_ptr<uint8_t>();
  }
  j.a.out = out.data_ptr();
  j.a.relu = relu;
  j.a.dropout = dropout;
  j.a.p_drop = (float)dropout_prob;
  j.a.seed = (uint64_t)seed;
  j.a.offset = (uint64_t)offset;
  transducer_joint_fwd(j.a, cur_stream());
  return {out, mask};
}

std::vector<at::Tensor> joint_backward(std::vector<at::Tensor> inp, at::Tensor f_len, at::Tensor g_len,
                                       at::Tensor batch_offset, int64_t max_f_len, int64_t max_g_len, bool pack_output,
                                       double scale, at::Tensor f_like, at::Tensor g_like) {
  const c10::hip::HIPGuard guard(inp[0].get_device());
  JointHold j;
  joint_setup(j, f_like, g_like, f_len, g_len, batch_offset, pack_output);
  TORCH_CHECK(j.a.T == max_f_len && j.a.U == max_g_len, "transducer joint bwd: shape mismatch");
  at::Tensor grad = inp[0].contiguous();
  at::Tensor mask;
  if (inp.size() > 1) {
    mask = inp[1].to(at::kByte).contiguous();
    j.a.mask = mask.data_ptr<uint8_t>();
  }
  auto fg = at::empty({j.a.B, j.a.T, j.a.H}, grad.options());
  auto gg = at::empty({j.a.B, j.a.U, j.a.H}, grad.options());
  transducer_joint_bwd(j.a, grad.data_ptr(), fg.data_ptr(), gg.data_ptr(), (float)scale, cur_stream());
  return {fg, gg};
}

struct LossHold {
  LossArgs a{};
  at::Tensor x, label, fl, yl, bo;
};

void loss_setup(LossHold& h, const at::Tensor& x, const at::Tensor& label, const at::Tensor& f_len,
                const at::Tensor& y_len, const at::Tensor& batch_offset, int64_t max_f_len, int64_t blank,
                bool packed) {
  h.x = x.contiguous();
  h.label = as_int(label);
  h.fl = as_int(f_len);
  h.yl = as_int(y_len);
  LossArgs& a = h.a;
  a.x = h.x.data_ptr();
  a.label = h.label.data_ptr<int>();
  a.f_len = h.fl.data_ptr<int>();
  a.y_len = h.yl.data_ptr<int>();
  a.B = (int)f_len.size(0);
  a.T = (int)max_f_len;
  a.U = (int)h.label.size(1) + 1;
  a.V = x.size(-1);
  a.blank = (int)blank;
  a.packed = packed;
  if (packed) {
    h.bo = batch_offset.to(at::kLong).contiguous();
    a.batch_offset = h.bo.data_ptr<int64_t>();
  } else {
    TORCH_CHECK(x.dim() == 4 && x.size(1) == max_f_len && x.size(2) == a.U, "transducer loss: x must be [B, T, U+1, V]");
  }
  a.dtype = dtype_code(x.scalar_type());
}

std::vector<at::Tensor> loss_forward(at::Tensor x, at::Tensor label, at::Tensor f_len, at::Tensor y_len,
                                     at::Tensor batch_offset, int64_t max_f_len, int64_t blank_idx, int64_t opt,
                                     bool packed_input) {
  (void)opt;
  const c10::hip::HIPGuard guard(x.get_device());
  LossHold h;
  loss_setup(h, x, label, f_len, y_len, batch_offset, max_f_len, blank_idx, packed_input);
  auto fo = x.options().dtype(at::kFloat);
  auto alpha = at::empty({h.a.B, h.a.T, h.a.U}, fo);
  auto beta = at::empty({h.a.B, h.a.T, h.a.U}, fo);
  auto loss = at::empty({h.a.B}, fo);
  h.a.alpha = alpha.data_ptr<float>();
  h.a.beta = beta.data_ptr<float>();
  h.a.loss = loss.data_ptr<float>();
  transducer_loss_fwd(h.a, cur_stream());
  return {alpha, beta, loss.to(x.scalar_type())};
}

at::Tensor loss_backward(at::Tensor x, at::Tensor loss_grad, at::Tensor alpha, at::Tensor beta, at::Tensor f_len,
                         at::Tensor y_len, at::Tensor label, at::Tensor batch_offset, int64_t max_f_len,
                         int64_t blank_idx, int64_t opt, bool fuse_softmax_backward, bool packed_input) {
  (void)opt;
  const c10::hip::HIPGuard guard(x.get_device());
  LossHold h;
  loss_setup(h, x, label, f_len, y_len, batch_offset, max_f_len, blank_idx, packed_input);
  at::Tensor a_c = alpha.contiguous(), b_c = beta.contiguous();
  h.a.alpha = a_c.data_ptr<float>();
  h.a.beta = b_c.data_ptr<float>();
  at::Tensor lg = loss_grad.to(at::kFloat).contiguous();
  auto xg = packed_input ? at::zeros_like(h.x) : at::empty_like(h.x);
  transducer_loss_bwd(h.a, lg.data_ptr<float>(), xg.data_ptr(), fuse_softmax_backward, cur_stream());
  return xg;
}

// ---- NHWC max pool: x is a channels_last NCHW tensor (memory [N, H, W, C]) ----
PoolArgs pool_args(const at::Tensor& x, std::vector<int64_t> k, std::vector<int64_t> st, std::vector<int64_t> pad) {
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool_nhwc: channels_last 4-D input");
  PoolArgs a{};
  a.N = (int)x.size(0);
  a.C = (int)x.size(1);
  a.H = (int)x.size(2);
  a.W = (int)x.size(3);
  a.KH = (int)k[0];
  a.KW = (int)k[1];
  a.SH = (int)st[0];
  a.SW = (int)st[1];
  a.PH = (int)pad[0];
  a.PW = (int)pad[1];
  a.OH = (a.H + 2 * a.PH - a.KH) / a.SH + 1;
  a.OW = (a.W + 2 * a.PW - a.KW) / a.SW + 1;
  a.dtype = dtype_code(x.scalar_type());
  return a;
}

std::vector<at::Tensor> maxpool_fwd(at::Tensor x, std::vector<int64_t> k, std::vector<int64_t> st,
                                    std::vector<int64_t> pad) {
  const c10::hip::HIPGuard guard(x.get_device());
  PoolArgs a = pool_args(x, k, st, pad);
  auto opts = x.options().memory_format(at::MemoryFormat::ChannelsLast);
  auto y = at::empty({a.N, a.C, a.OH, a.OW}, opts);
  auto idx = at::empty({a.N, a.C, a.OH, a.OW}, opts.dtype(at::kByte));
  maxpool_nhwc_fwd(a, x.data_ptr(), y.data_ptr(), idx.data_ptr<uint8_t>(), device_cus(x.get_device()), cur_stream());
  return {y, idx};
}

at::Tensor maxpool_bwd(at::Tensor dy, at::Tensor idx, at::Tensor x_like, std::vector<int64_t> k,
                       std::vector<int64_t> st, std::vector<int64_t> pad) {
  const c10::hip::HIPGuard guard(dy.get_device());
  PoolArgs a = pool_args(x_like, k, st, pad);
  at::Tensor g = dy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(g.size(2) == a.OH && g.size(3) == a.OW && idx.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool_nhwc bwd: shape mismatch");
  auto dx = at::empty(x_like.sizes(), x_like.options().memory_format(at::MemoryFormat::ChannelsLast));
  maxpool_nhwc_bwd(a, g.data_ptr(), idx.data_ptr<uint8_t>(), dx.data_ptr(), device_cus(dy.get_device()),
                   cur_stream());
  return dx;
}

}  // namespace

void bind_contrib(pybind11::module_& root) {
  auto j = root.def_submodule("transducer_joint_cuda", "RNN-T joint (gfx950)");
  j.def("forward", &joint_forward);
  j.def("backward", &joint_backward);
  auto l = root.def_submodule("transducer_loss_cuda", "RNN-T loss (gfx950)");
  l.def("forward", &loss_forward);
  l.def("backward", &loss_backward);
  auto p = root.def_submodule("maxpool_nhwc", "channels_last max pooling with 1-byte indices (gfx950)");
  p.def("forward", &maxpool_fwd);
  p.def("backward", &maxpool_bwd);
  auto pm = root.def_submodule("peer_memory", "hipIpc peer-memory exchange for latency-bound collectives");
  pm.def("alloc", &pm_alloc);
  pm.def("free", &pm_free);
  pm.def("handle", &pm_handle);
  pm.def("open", &pm_open);
  pm.def("close", &pm_close);
  pm.def("max_group", &peer_max_group);
  pm.def("allgather", &pm_allgather);
  auto t = root.def_submodule("fused_transformer", "transformer block elementwise fusions (gfx950)");
  t.def("bias_dropout_add_forward", &bda_forward, pybind11::arg("x"), pybind11::arg("bias"), pybind11::arg("residual"),
        pybind11::arg("p"), pybind11::arg("seed"), pybind11::arg("offset"), pybind11::arg("rng_step") = c10::nullopt);
  t.def("bias_dropout_add_backward", &bda_backward, pybind11::arg("grad"), pybind11::arg("p"), pybind11::arg("seed"),
        pybind11::arg("offset"), pybind11::arg("rng_step") = c10::nullopt);
}

}  // namespace apex_amd
