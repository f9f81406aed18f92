// pybind surface of the gfx950 implicit-GEMM convolutions (csrc/conv/conv_igemm.hip):
// submodule ``_C.conv`` used by apex.ops.conv (ResNet 3x3 / strided convolutions, NHWC).
// Activations are dense NHWC [N, H, W, C] tensors (the python layer passes zero-copy views of
// torch channels_last tensors); weights are [K, taps, C] (k contiguous per tap).
#include "apex_amd/conv_ks.h"
#include "common.h"
#include "apex_amd/conv_api.h"
#include "apex_amd/layout_extra.h"
#include "apex_amd/conv_halo.h"

namespace apex_amd {
namespace {

void check_nhwc(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.is_contiguous(), "conv: ", what,
              " must be a contiguous NHWC [N, H, W, C] GPU tensor");
}

ConvTapArgs make_args(const at::Tensor& in, const at::Tensor& w, const at::Tensor& out, int64_t oh, int64_t ow,
                      int64_t ish, int64_t isw, int64_t osh, int64_t osw, int64_t oph, int64_t opw,
                      const std::vector<int64_t>& dh, const std::vector<int64_t>& dw) {
  check_nhwc(in, "input");
  check_nhwc(out, "output");
  TORCH_CHECK(w.is_cuda() && w.dim() == 3 && w.is_contiguous(), "conv: weight must be a contiguous [K, taps, C] tensor");
  TORCH_CHECK(in.scalar_type() == w.scalar_type() && in.scalar_type() == out.scalar_type(),
              "conv: input, weight and output must share a dtype");
  TORCH_CHECK(dh.size() == dw.size() && !dh.empty() && (int64_t)dh.size() <= kConvMaxTaps, "conv: 1..9 taps");
  TORCH_CHECK(w.size(1) == (int64_t)dh.size() && w.size(2) == in.size(3) && w.size(0) == out.size(3),
              "conv: weight [K, taps, C] does not match input / output");
  TORCH_CHECK(in.size(0) == out.size(0), "conv: batch mismatch");
  ConvTapArgs a{};
  a.in = in.data_ptr();
  a.wt = w.data_ptr();
  a.out = out.data_ptr();
  a.n = (int)in.size(0);
  a.ih = (int)in.size(1);
  a.iw = (int)in.size(2);
  a.c = (int)in.size(3);
  a.oh = (int)oh;
  a.ow = (int)ow;
  a.oht = (int)out.size(1);
  a.owt = (int)out.size(2);
  a.kout = (int)out.size(3);
  a.ish = (int)ish;
  a.isw = (int)isw;
  a.osh = (int)osh;
  a.osw = (int)osw;
  a.oph = (int)oph;
  a.opw = (int)opw;
  a.ntaps = (int)dh.size();
  for (size_t t = 0; t < dh.size(); ++t) {
    a.dh[t] = (int)dh[t];
    a.dw[t] = (int)dw[t];
  }
  a.dtype = dtype_code(in.scalar_type());
  TORCH_CHECK((oh - 1) * osh + oph < a.oht && (ow - 1) * osw + opw < a.owt, "conv: output grid exceeds the output");
  return a;
}

// out[n, oh*osh+oph, ow*osw+opw, k] = sum_t,c in[n, oh*ish+dh[t], ow*isw+dw[t], c] * w[k, t, c]
// Returns the BN-statistics partials [2, rows, K] (rows = the chosen tile configuration's M
// tiles) when ``stats_shift`` is given without a ``stats`` buffer, else None.
c10::optional<at::Tensor> tap_fprop(const at::Tensor& in, const at::Tensor& w, at::Tensor& out, int64_t oh, int64_t ow, int64_t ish,
               int64_t isw, int64_t osh, int64_t osw, int64_t oph, int64_t opw, std::vector<int64_t> dh,
               std::vector<int64_t> dw, const c10::optional<at::Tensor>& scale,
               const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& residual, bool relu,
               const c10::optional<at::Tensor>& mask, const c10::optional<at::Tensor>& stats,
               const c10::optional<at::Tensor>& stats_shift, const c10::optional<at::Tensor>& pcoef,
               const c10::optional<at::Tensor>& red_x, const c10::optional<at::Tensor>& red_coef,
               const c10::optional<at::Tensor>& red_mean) {
  ConvTapArgs a = make_args(in, w, out, oh, ow, ish, isw, osh, osw, oph, opw, dh, dw);
  auto per_channel = [&](const c10::optional<at::Tensor>& t, const char* what) -> const float* {
    if (!t.has_value()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == out.size(3),
                "conv tap_fprop: ", what, " must be a contiguous fp32 [K] tensor on the output's device");
    return t->data_ptr<float>();
  };
  a.scale = per_channel(scale, "scale");
  a.bias = per_channel(bias, "bias");
  if (residual.has_value()) {
    check_nhwc(*residual, "residual");
    TORCH_CHECK(residual->sizes() == out.sizes() && residual->strides() == out.strides() &&
                    residual->scalar_type() == out.scalar_type(),
                "conv tap_fprop: residual must match the output's shape, layout and dtype");
    a.residual = residual->data_ptr();
  }
  a.relu = relu ? 1 : 0;
  if (mask.has_value()) {
    check_nhwc(*mask, "mask");
    TORCH_CHECK(mask->sizes() == out.sizes() && mask->strides() == out.strides() &&
                    mask->scalar_type() == out.scalar_type(),
                "conv tap_fprop: mask must match the output's shape, layout and dtype");
    a.mask = mask->data_ptr();
  }
  if (red_x.has_value()) {
    // BN backward reduction of the stored gradient (returned as the [2, tiles, K] partials)
    check_nhwc(*red_x, "red_x");
    TORCH_CHECK(red_x->sizes() == out.sizes() && red_x->strides() == out.strides() &&
                    red_x->scalar_type() == out.scalar_type() && red_coef.has_value() && red_mean.has_value() &&
                    !stats_shift.has_value() && !mask.has_value() && !pcoef.has_value(),
                "conv tap_fprop: red_x must match the output (layout, dtype) and comes with red_coef / red_mean only");
    TORCH_CHECK(red_coef->is_cuda() && red_coef->scalar_type() == at::kFloat && red_coef->is_contiguous() &&
                    red_coef->numel() == 2 * out.size(3),
                "conv tap_fprop: red_coef must be a contiguous fp32 [2K] tensor");
    a.red_x = red_x->data_ptr();
    a.red_coef = red_coef->data_ptr<float>();
    a.red_mean = per_channel(red_mean, "red_mean");
  }
  const c10::hip::HIPGuard g(in.get_device());
  const int cus = device_cus(in.get_device());
  c10::optional<at::Tensor> made;
  if (stats.has_value() || stats_shift.has_value() || red_x.has_value()) {
    const int64_t rows = conv_tap_stats_tiles(a, cus);
    at::Tensor st = stats.has_value() ? *stats : at::empty({2, rows, out.size(3)}, out.options().dtype(at::kFloat));
    TORCH_CHECK(st.is_cuda() && st.scalar_type() == at::kFloat && st.is_contiguous() &&
                    st.numel() == 2 * rows * out.size(3),
                "conv tap_fprop: stats must be contiguous fp32 [2, stats_tiles, K]");
    a.stats = st.data_ptr<float>();
    a.stats_shift = per_channel(stats_shift, "stats_shift");
    if (!stats.has_value()) made = st;
  }
  TORCH_CHECK(conv_tap_supported(a), "conv tap_fprop: unsupported (C and K must be multiples of 64, bf16/fp16)");
  if (pcoef.has_value()) {
    // operand prologue relu(x * pcoef[c] + pcoef[C + c]) on the halo-tile kernel
    TORCH_CHECK(pcoef->is_cuda() && pcoef->scalar_type() == at::kFloat && pcoef->is_contiguous() &&
                    pcoef->numel() == 2 * in.size(3),
                "conv tap_fprop: pcoef must be a contiguous fp32 [2C] tensor");
    // the spatial-tile 64 -> 64 kernel where it is the route, else the halo-tile kernel
    if (conv_sp_default(a)) {
      conv_sp_fprop_pro(a, pcoef->data_ptr<float>(), cus, cur_stream());
      return made;
    }
    TORCH_CHECK(conv_hfp_supported(a), "conv tap_fprop: the BN prologue needs the spatial-tile (64 -> 64) or "
                "halo-tile kernel's shapes (3x3 stride 1, C % 64 == 0, K % 128 == 0, no fused epilogue)");
    conv_hfp(a, pcoef->data_ptr<float>(), cus, cur_stream());
    return made;
  }
  conv_tap_fprop(a, cus, cur_stream());
  return made;
}

// dw[k, t, c] (fp32-accumulated, written in dw's dtype) for the forward `in` -> dy geometry
void wgrad(const at::Tensor& in, const at::Tensor& dy, at::Tensor& dw_out, int64_t ish, int64_t isw,
           std::vector<int64_t> dh, std::vector<int64_t> dw, const c10::optional<at::Tensor>& xcoef) {
  check_nhwc(dy, "grad");
  TORCH_CHECK(dw_out.is_cuda() && dw_out.dim() == 3 && dw_out.is_contiguous(), "conv wgrad: dw must be [K, taps, C]");
  TORCH_CHECK(dw_out.size(0) == dy.size(3) && dw_out.size(1) == (int64_t)dh.size() && dw_out.size(2) == in.size(3),
              "conv wgrad: dw must be [K, taps, C]");
  TORCH_CHECK(dw_out.scalar_type() == in.scalar_type() || dw_out.scalar_type() == at::kFloat,
              "conv wgrad: dw must be fp32 or the activation dtype");
  ConvTapArgs a = make_args(in, dw_out.scalar_type() == in.scalar_type() ? dw_out : dw_out.to(in.scalar_type()), dy,
                            dy.size(1), dy.size(2), ish, isw, 1, 1, 0, 0, dh, dw);
  a.wt = nullptr;
  const c10::hip::HIPGuard g(in.get_device());
  TORCH_CHECK(conv_wgrad_supported(a), "conv wgrad: unsupported shape");
  const int cus = device_cus(in.get_device());
  if (xcoef.has_value()) {
    // input through the producing BN + ReLU: the halo-tile kernel only
    TORCH_CHECK(xcoef->is_cuda() && xcoef->scalar_type() == at::kFloat && xcoef->is_contiguous() &&
                    xcoef->numel() == 2 * in.size(3),
                "conv wgrad: xcoef must be a contiguous fp32 [2C] tensor");
    TORCH_CHECK(conv_hwgrad_supported(a), "conv wgrad: the BN prologue needs the halo-tile kernel's shapes");
    auto ws = at::empty({conv_hwgrad_workspace_floats(a, cus)}, in.options().dtype(at::kFloat));
    conv_hwgrad_pro(a, dy.data_ptr(), dw_out.data_ptr(), dtype_code(dw_out.scalar_type()), ws.data_ptr<float>(), cus,
                    cur_stream(), xcoef->data_ptr<float>());
    return;
  }
  auto ws = at::empty({conv_wgrad_workspace_floats(a, cus)}, in.options().dtype(at::kFloat));
  conv_wgrad(a, dy.data_ptr(), dw_out.data_ptr(), dtype_code(dw_out.scalar_type()), ws.data_ptr<float>(), cus,
             cur_stream());
}

// True when conv_wgrad takes the halo-tile kernel (csrc/conv/conv3x3_wgrad.hip) for a 3x3 pad-1
// stride-1 / stride-2 conv of an [n, h, w, c] input to kout channels (ops/conv.py tap_route)
bool halo_wgrad_supported(int64_t n, int64_t h, int64_t w, int64_t c, int64_t kout, int64_t stride) {
  ConvTapArgs a{};
  void* aligned = reinterpret_cast<void*>(static_cast<uintptr_t>(256));  // alignment checks only
  a.in = a.wt = aligned;
  a.out = aligned;
  a.n = (int)n;
  a.ih = (int)h;
  a.iw = (int)w;
  a.oh = a.oht = (int)((h - 1) / stride + 1);
  a.ow = a.owt = (int)((w - 1) / stride + 1);
  a.c = (int)c;
  a.kout = (int)kout;
  a.ish = a.isw = (int)stride;
  a.osh = a.osw = 1;
  a.oph = a.opw = 0;
  a.ntaps = 9;
  for (int t = 0; t < 9; ++t) {
    a.dh[t] = t / 3 - 1;
    a.dw[t] = t % 3 - 1;
  }
  a.dtype = kBF16;
  return conv_hwgrad_supported(a);
}

// y = pro(a) . W^T (+ BN statistics partials); see conv_api.h.  Returns (y, part or empty).
// rows of the residual: M, or those of its stride-2 subsample when res_h, res_w > 0 (M = N res_h res_w)
static int64_t res_rows(int64_t m, int64_t res_h, int64_t res_w) {
  if (res_h <= 0 || res_w <= 0) return m;
  TORCH_CHECK(m % (res_h * res_w) == 0, "subsampled residual: M is not a multiple of res_h * res_w");
  return m / (res_h * res_w) * ((res_h + 1) / 2) * ((res_w + 1) / 2);
}

std::vector<at::Tensor> bn1x1(const at::Tensor& a, const at::Tensor& w, bool w_kmajor_out,
                              const c10::optional<at::Tensor>& pcoef, const c10::optional<at::Tensor>& shift,
                              bool stats, const c10::optional<at::Tensor>& res,
                              const c10::optional<at::Tensor>& py, bool want_aout, int64_t res_h, int64_t res_w) {
  TORCH_CHECK(a.is_cuda() && a.dim() == 2 && a.is_contiguous(), "bn1x1: a must be a contiguous [M, K] GPU tensor");
  TORCH_CHECK(w.is_cuda() && w.dim() == 2 && w.is_contiguous() && w.scalar_type() == a.scalar_type(),
              "bn1x1: w must be a contiguous 2-D tensor of a's dtype");
  const int64_t m = a.size(0);
  const int k = (int)a.size(1);
  const int ncols = (int)(w_kmajor_out ? w.size(1) : w.size(0));
  TORCH_CHECK((w_kmajor_out ? w.size(0) : w.size(1)) == k, "bn1x1: weight does not match the reduction dim");
  // the deep reductions (k 1024 / 2048, ResNet stages 3-4) run on the K-streamed kernel
  const bool ks = !conv1x1_bn_supported(m, k, ncols) && conv1x1_ks_supported(m, k, ncols);
  TORCH_CHECK(ks || conv1x1_bn_supported(m, k, ncols), "bn1x1: unsupported shape (k % 64, ncols % 64)");
  auto f32 = [&](const c10::optional<at::Tensor>& t, int64_t n, const char* what) -> const float* {
    if (!t.has_value()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == n, "bn1x1: ",
                what, " must be a contiguous fp32 tensor of ", n, " elements");
    return t->data_ptr<float>();
  };
  const bool bnbwd = py.has_value();
  // BN-backward prologue: pcoef [3K] (a = the masked gradient) or [5K] (+ the forward scale | shift:
  // the ReLU mask recomputed from py, a = the unmasked gradient)
  const bool pmask = bnbwd && pcoef.has_value() && pcoef->numel() == 5 * (int64_t)k;
  const float* pc = f32(pcoef, (bnbwd ? (pmask ? 5 : 3) : 2) * (int64_t)k, "pcoef");
  TORCH_CHECK(!bnbwd || (pc && w_kmajor_out && py->is_cuda() && py->is_contiguous() &&
                         py->scalar_type() == a.scalar_type() && py->sizes() == a.sizes()),
              "bn1x1: py (BN-backward prologue) needs the dgrad form, pcoef [3K] / [5K] and a tensor shaped like a");
  TORCH_CHECK(!want_aout || bnbwd, "bn1x1: want_aout needs the BN-backward prologue");
  const float* sh = f32(shift, ncols, "shift");
  const c10::hip::HIPGuard g(a.get_device());
  const int cus = device_cus(a.get_device());
  auto y = at::empty({m, ncols}, a.options());
  at::Tensor part, aout;
  if (want_aout) aout = at::empty_like(a);
  if (ks) {
    TORCH_CHECK(!res.has_value() && res_h <= 0 && !pmask && (bnbwd || pc == nullptr),
                "bn1x1: the deep-reduction kernel takes no residual, recomputed-mask or BN-apply prologue");
    if (stats) part = at::empty({2, conv1x1_ks_partials(m, k, ncols, cus, bnbwd ? 2 : 0), ncols}, a.options().dtype(at::kFloat));
    conv1x1_ks(a.data_ptr(), w.data_ptr(), y.data_ptr(), m, k, ncols, w_kmajor_out, dtype_code(a.scalar_type()), pc,
               bnbwd ? 2 : 0, false, nullptr, sh, stats ? part.data_ptr<float>() : nullptr,
               bnbwd ? py->data_ptr() : nullptr, want_aout ? aout.data_ptr() : nullptr, nullptr, nullptr, nullptr,
               nullptr, cus, cur_stream());
    return {y, part, aout};
  }
  if (stats)
    part = at::empty({2, conv1x1_bn_partials(m, k, ncols, pc != nullptr, cus), ncols}, a.options().dtype(at::kFloat));
  if (res.has_value())
    TORCH_CHECK(res->is_cuda() && res->is_contiguous() && res->scalar_type() == a.scalar_type() &&
                    res->numel() == res_rows(m, res_h, res_w) * ncols,
                "bn1x1: res must be a contiguous [M, ncols] tensor of a's dtype (subsampled rows with res_hw)");
  TORCH_CHECK(res_h <= 0 || w_kmajor_out, "bn1x1: a subsampled residual is a dgrad-form option");
  conv1x1_bn(a.data_ptr(), w.data_ptr(), y.data_ptr(), m, k, ncols, w_kmajor_out, dtype_code(a.scalar_type()), pc, sh,
             stats ? part.data_ptr<float>() : nullptr, cus, cur_stream(), res.has_value() ? res->data_ptr() : nullptr,
             bnbwd ? py->data_ptr() : nullptr, want_aout ? aout.data_ptr() : nullptr, false, nullptr, (int)res_h,
             (int)res_w, false, nullptr, pmask);
  return {y, part, aout};
}

// Forward 1x1 conv whose operand is the block below's output computed on load:
// out = relu(fma(a, pcoef[0], pcoef[2]) + fma(res, pcoef[1], pcoef[3])) (a = that block's output-BN
// input y3, res = its shortcut: the identity input with pcoef[1] = 1, pcoef[3] = 0, or the
// downsample BN's input with that BN's scale / shift) — the same arithmetic as the standalone
// apply / dual-apply passes, so the deferred output is bitwise the one they would write.
// Returns (y = out . W^T, statistics partials about shift, out [M, K], ReLU bits [M K / 8]).
// [N * h * w, C] (NHWC rows) -> its stride-2 subsample [N * ceil(h/2) * ceil(w/2), C]
at::Tensor subsample2x(const at::Tensor& x, int64_t n, int64_t h, int64_t w) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.is_contiguous() && x.size(0) == n * h * w &&
                  (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "subsample2x: x must be a contiguous 16-bit [N * h * w, C] GPU tensor");
  const c10::hip::HIPGuard g(x.get_device());
  auto y = at::empty({n * ((h + 1) / 2) * ((w + 1) / 2), x.size(1)}, x.options());
  conv_subsample2x(x.data_ptr(), y.data_ptr(), (int)n, (int)h, (int)w, (int)x.size(1), dtype_code(x.scalar_type()),
                   device_cus(x.get_device()), cur_stream());
  return y;
}

// g [N, C] -> [N, C, h, w] channels_last with every pixel g * scale (global average pool backward)
at::Tensor spatial_broadcast_b(const at::Tensor& g, int64_t h, int64_t w, double scale) {
  TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous() &&
                  (g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kHalf) && g.size(1) % 8 == 0,
              "spatial_broadcast: g must be a contiguous 16-bit [N, C] GPU tensor, C % 8 == 0");
  const c10::hip::HIPGuard guard(g.get_device());
  auto y = at::empty({g.size(0), g.size(1), h, w}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  spatial_broadcast(g.data_ptr(), y.data_ptr(), (int)g.size(0), (int)(h * w), (int)g.size(1), (float)scale,
                    dtype_code(g.scalar_type()), device_cus(g.get_device()), cur_stream());
  return y;
}

// [K, C, R, S] channels_last 16-bit weight -> its data-gradient image [C, len(taps), K] (taps: r * S + s)
at::Tensor tap_weights(const at::Tensor& w, const std::vector<int64_t>& taps) {
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  (w.scalar_type() == at::kBFloat16 || w.scalar_type() == at::kHalf),
              "tap_weights: w must be a channels_last 16-bit [K, C, R, S] GPU tensor");
  const int k = (int)w.size(0), c = (int)w.size(1), rs = (int)(w.size(2) * w.size(3));
  TORCH_CHECK(!taps.empty() && taps.size() <= 9 && k % 8 == 0 && c % 8 == 0, "tap_weights: 1-9 taps, K, C % 8 == 0");
  std::vector<int> t(taps.begin(), taps.end());
  const c10::hip::HIPGuard g(w.get_device());
  auto dst = at::empty({c, (int64_t)t.size(), k}, w.options().memory_format(at::MemoryFormat::Contiguous));
  conv_tap_weights(w.data_ptr(), dst.data_ptr(), k, c, rs, t.data(), (int)t.size(), cur_stream());
  return dst;
}

// pcoef: [4K] (a scale | res scale | a shift | res shift), or with split the output BN's [2K]
// scale | shift and res_coef the residual BN's [2K] (none: the identity shortcut)
std::vector<at::Tensor> bn1x1_addrelu(const at::Tensor& a, const at::Tensor& res, const at::Tensor& pcoef,
                                      const at::Tensor& w, const c10::optional<at::Tensor>& shift,
                                      const c10::optional<at::Tensor>& out_opt, bool split,
                                      const c10::optional<at::Tensor>& res_coef) {
  TORCH_CHECK(a.is_cuda() && a.dim() == 2 && a.is_contiguous(), "bn1x1_addrelu: a must be a contiguous [M, K] GPU tensor");
  TORCH_CHECK(res.is_cuda() && res.is_contiguous() && res.sizes() == a.sizes() && res.scalar_type() == a.scalar_type(),
              "bn1x1_addrelu: res must be shaped like a");
  TORCH_CHECK(w.is_cuda() && w.dim() == 2 && w.is_contiguous() && w.scalar_type() == a.scalar_type() &&
                  w.size(1) == a.size(1),
              "bn1x1_addrelu: w must be [ncols, K] of a's dtype");
  const int64_t m = a.size(0);
  const int k = (int)a.size(1), ncols = (int)w.size(0);
  const bool ks = !conv1x1_bn_supported(m, k, ncols) && conv1x1_ks_supported(m, k, ncols);
  TORCH_CHECK((ks || conv1x1_bn_supported(m, k, ncols)) && (m * k) % 8 == 0, "bn1x1_addrelu: unsupported shape");
  TORCH_CHECK(pcoef.is_cuda() && pcoef.scalar_type() == at::kFloat && pcoef.is_contiguous() &&
                  pcoef.numel() == (split ? 2 : 4) * (int64_t)k,
              "bn1x1_addrelu: pcoef must be contiguous fp32 [4K] ([2K] with split)");
  TORCH_CHECK(!res_coef.has_value() || (split && res_coef->is_cuda() && res_coef->scalar_type() == at::kFloat &&
                                        res_coef->is_contiguous() && res_coef->numel() == 2 * (int64_t)k),
              "bn1x1_addrelu: res_coef (split form only) must be contiguous fp32 [2K]");
  if (shift.has_value())
    TORCH_CHECK(shift->is_cuda() && shift->scalar_type() == at::kFloat && shift->is_contiguous() && shift->numel() == ncols,
                "bn1x1_addrelu: shift must be contiguous fp32 [ncols]");
  const c10::hip::HIPGuard g(a.get_device());
  const int cus = device_cus(a.get_device());
  auto y = at::empty({m, ncols}, a.options());
  at::Tensor out;
  if (out_opt.has_value()) {
    TORCH_CHECK(out_opt->is_cuda() && out_opt->is_contiguous() && out_opt->sizes() == a.sizes() &&
                    out_opt->scalar_type() == a.scalar_type(),
                "bn1x1_addrelu: out must be a contiguous tensor shaped like a");
    out = *out_opt;
  } else {
    out = at::empty_like(a);
  }
  auto bits = at::empty({m * k / 8}, a.options().dtype(at::kByte));
  if (ks) {
    auto part = at::empty({2, conv1x1_ks_partials(m, k, ncols, cus, 3), ncols}, a.options().dtype(at::kFloat));
    conv1x1_ks(a.data_ptr(), w.data_ptr(), y.data_ptr(), m, k, ncols, false, dtype_code(a.scalar_type()),
               pcoef.data_ptr<float>(), 3, split, res_coef.has_value() ? res_coef->data_ptr<float>() : nullptr,
               shift.has_value() ? shift->data_ptr<float>() : nullptr, part.data_ptr<float>(), res.data_ptr(),
               out.data_ptr(), bits.data_ptr<uint8_t>(), nullptr, nullptr, nullptr, cus, cur_stream());
    return {y, part, out, bits};
  }
  auto part = at::empty({2, conv1x1_bn_partials(m, k, ncols, true, cus, true), ncols}, a.options().dtype(at::kFloat));
  conv1x1_bn(a.data_ptr(), w.data_ptr(), y.data_ptr(), m, k, ncols, false, dtype_code(a.scalar_type()),
             pcoef.data_ptr<float>(), shift.has_value() ? shift->data_ptr<float>() : nullptr, part.data_ptr<float>(), cus,
             cur_stream(), nullptr, res.data_ptr(), out.data_ptr(), true, bits.data_ptr<uint8_t>(), 0, 0, split,
             res_coef.has_value() ? res_coef->data_ptr<float>() : nullptr);
  return {y, part, out, bits};
}

// (save_mean, save_invstd, coef[2C]) from bn1x1 partials; running stats updated in place
std::vector<at::Tensor> bn_finalize(const at::Tensor& part, double count, const c10::optional<at::Tensor>& shift,
                                    const c10::optional<at::Tensor>& w, const c10::optional<at::Tensor>& b,
                                    const c10::optional<at::Tensor>& running_mean,
                                    const c10::optional<at::Tensor>& running_var, double eps, double momentum) {
  TORCH_CHECK(part.is_cuda() && part.dim() == 3 && part.size(0) == 2 && part.is_contiguous() &&
                  part.scalar_type() == at::kFloat,
              "bn_finalize: part must be the [2, G, C] fp32 partials");
  const int c = (int)part.size(2);
  auto f = [&](const c10::optional<at::Tensor>& t) -> float* {
    if (!t.has_value()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == c,
                "bn_finalize: per-channel tensors must be contiguous fp32 [C]");
    return t->data_ptr<float>();
  };
  const c10::hip::HIPGuard g(part.get_device());
  auto opt = part.options();
  auto sm = at::empty({c}, opt), si = at::empty({c}, opt), coef = at::empty({2 * c}, opt);
  conv1x1_bn_finalize(part.data_ptr<float>(), (int)part.size(1), c, (float)count, f(shift), f(w), f(b), (float)eps,
                      (float)momentum, f(running_mean), f(running_var), sm.data_ptr<float>(), si.data_ptr<float>(),
                      coef.data_ptr<float>(), cur_stream());
  return {sm, si, coef};
}

// bn_group > 1: this rank's Welford payload [mean | M2 | count] (2C + 1) from the partials
at::Tensor part_payload(const at::Tensor& part, double count, const c10::optional<at::Tensor>& shift) {
  TORCH_CHECK(part.is_cuda() && part.dim() == 3 && part.size(0) == 2 && part.is_contiguous() &&
                  part.scalar_type() == at::kFloat,
              "part_payload: part must be the [2, G, C] fp32 partials");
  const int c = (int)part.size(2);
  if (shift.has_value())
    TORCH_CHECK(shift->is_cuda() && shift->scalar_type() == at::kFloat && shift->is_contiguous() && shift->numel() == c,
                "part_payload: shift must be contiguous fp32 [C]");
  const c10::hip::HIPGuard g(part.get_device());
  auto payload = at::empty({2 * (int64_t)c + 1}, part.options());
  conv1x1_bn_part_payload(part.data_ptr<float>(), (int)part.size(1), c, (float)count,
                          shift.has_value() ? shift->data_ptr<float>() : nullptr, payload.data_ptr<float>(),
                          cur_stream());
  return payload;
}

// dW [N, K] = g^T . pro(x) (pro = relu(x * xcoef[:K] + xcoef[K:]) when given), out_dtype per `like`
at::Tensor wgrad1x1(const at::Tensor& g, const at::Tensor& x, const c10::optional<at::Tensor>& xcoef,
                    c10::optional<at::ScalarType> out_dtype) {
  TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous() && x.is_cuda() && x.dim() == 2 && x.is_contiguous() &&
                  g.size(0) == x.size(0) && g.scalar_type() == x.scalar_type(),
              "wgrad1x1: g [M, N] and x [M, K] must be contiguous GPU tensors of one dtype");
  const int64_t m = g.size(0);
  const int n = (int)g.size(1), k = (int)x.size(1);
  TORCH_CHECK(conv1x1_wgrad_supported(m, n, k), "wgrad1x1: unsupported shape (N, K multiples of 64)");
  const float* xc = nullptr;
  if (xcoef.has_value()) {
    TORCH_CHECK(xcoef->is_cuda() && xcoef->scalar_type() == at::kFloat && xcoef->is_contiguous() &&
                    xcoef->numel() == 2 * (int64_t)k,
                "wgrad1x1: xcoef must be contiguous fp32 [2K]");
    xc = xcoef->data_ptr<float>();
  }
  const c10::hip::HIPGuard guard(g.get_device());
  const int cus = device_cus(g.get_device());
  auto dw = at::empty({n, k}, g.options().dtype(out_dtype.value_or(g.scalar_type())));
  auto ws = at::empty({conv1x1_wgrad_workspace_floats(m, n, k, cus)}, g.options().dtype(at::kFloat));
  conv1x1_wgrad(g.data_ptr(), x.data_ptr(), dw.data_ptr(), dtype_code(dw.scalar_type()), m, n, k,
                dtype_code(g.scalar_type()), xc, ws.data_ptr<float>(), cus, cur_stream());
  return dw;
}

// conv dgrad (dgrad form W [k, ncols]) + residual, masked with the BN below's ReLU (its forward
// bit mask, or recomputed from x and its apply coefficients `coef`) and that BN's backward
// reduction partials.  Optional BN-backward prologue (py, pcoef [3k]) with the transformed
// operand written out (want_aout).  Returns (out, part, aout)
std::vector<at::Tensor> dgrad_bnred(const at::Tensor& g, const at::Tensor& w, const c10::optional<at::Tensor>& res,
                                    const c10::optional<at::Tensor>& bits, const at::Tensor& x, const at::Tensor& mean,
                                    const c10::optional<at::Tensor>& coef, const c10::optional<at::Tensor>& py,
                                    const c10::optional<at::Tensor>& pcoef, bool want_aout, int64_t res_h,
                                    int64_t res_w, const c10::optional<at::Tensor>& x2,
                                    const c10::optional<at::Tensor>& mean2) {
  TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous() && w.dim() == 2 && w.is_contiguous() &&
                  w.scalar_type() == g.scalar_type() && w.size(0) == g.size(1),
              "dgrad_bnred: g [M, k] and w [k, ncols] expected");
  const int64_t m = g.size(0);
  const int k = (int)g.size(1), ncols = (int)w.size(1);
  TORCH_CHECK(x.is_contiguous() && x.scalar_type() == g.scalar_type() && x.numel() == m * ncols,
              "dgrad_bnred: x must be the contiguous [M, ncols] BN input");
  TORCH_CHECK(bits.has_value() != coef.has_value(), "dgrad_bnred: exactly one of bits / coef");
  if (bits.has_value())
    TORCH_CHECK(bits->is_contiguous() && bits->scalar_type() == at::kByte && bits->numel() * 8 == m * ncols,
                "dgrad_bnred: bits must be the [M * ncols / 8] ReLU mask");
  if (coef.has_value())
    TORCH_CHECK(coef->is_contiguous() && coef->scalar_type() == at::kFloat && coef->numel() == 2 * (int64_t)ncols,
                "dgrad_bnred: coef must be fp32 [2 * ncols]");
  TORCH_CHECK(mean.is_contiguous() && mean.scalar_type() == at::kFloat && mean.numel() == ncols,
              "dgrad_bnred: mean must be fp32 [ncols]");
  if (res.has_value())
    TORCH_CHECK(res->is_contiguous() && res->scalar_type() == g.scalar_type() &&
                    res->numel() == res_rows(m, res_h, res_w) * ncols,
                "dgrad_bnred: res must be a contiguous [M, ncols] tensor (subsampled rows with res_hw)");
  const bool pro = py.has_value();
  TORCH_CHECK(pro == pcoef.has_value(), "dgrad_bnred: py and pcoef go together");
  const bool pmask = pro && pcoef->numel() == 5 * (int64_t)k;  // [5k]: the ReLU mask recomputed from py
  if (pro)
    TORCH_CHECK(py->is_contiguous() && py->sizes() == g.sizes() && py->scalar_type() == g.scalar_type() &&
                    pcoef->scalar_type() == at::kFloat && pcoef->is_contiguous() &&
                    (pcoef->numel() == 3 * (int64_t)k || pmask),
                "dgrad_bnred: py must match g, pcoef fp32 [3k] or [5k]");
  TORCH_CHECK(!want_aout || pro, "dgrad_bnred: want_aout needs the prologue");
  const bool ks = !conv1x1_bn_supported(m, k, ncols) && conv1x1_ks_supported(m, k, ncols);
  TORCH_CHECK(ks || conv1x1_bn_supported(m, k, ncols), "dgrad_bnred: unsupported shape");
  TORCH_CHECK(x2.has_value() == mean2.has_value(), "dgrad_bnred: x2 and mean2 go together");
  if (x2.has_value())
    TORCH_CHECK(x2->is_contiguous() && x2->scalar_type() == g.scalar_type() && x2->numel() == m * ncols &&
                    mean2->is_contiguous() && mean2->scalar_type() == at::kFloat && mean2->numel() == ncols,
                "dgrad_bnred: x2 must be the contiguous [M, ncols] input of the second BN, mean2 fp32 [ncols]");
  const c10::hip::HIPGuard guard(g.get_device());
  const int cus = device_cus(g.get_device());
  auto out = at::empty({m, ncols}, g.options());
  if (ks) {
    TORCH_CHECK(coef.has_value() && !res.has_value() && res_h <= 0 && !x2.has_value() && !pmask,
                "dgrad_bnred: the deep-reduction kernel takes the recomputed mask (coef) only: no bits, residual, "
                "second BN or masked prologue");
    auto part = at::empty({2, conv1x1_ks_partials(m, k, ncols, cus, pro ? 2 : 0), ncols}, g.options().dtype(at::kFloat));
    at::Tensor aout;
    if (want_aout) aout = at::empty_like(g);
    conv1x1_ks(g.data_ptr(), w.data_ptr(), out.data_ptr(), m, k, ncols, true, dtype_code(g.scalar_type()),
               pro ? pcoef->data_ptr<float>() : nullptr, pro ? 2 : 0, false, nullptr, nullptr, part.data_ptr<float>(),
               pro ? py->data_ptr() : nullptr, want_aout ? aout.data_ptr() : nullptr, nullptr,
               coef->data_ptr<float>(), x.data_ptr(), mean.data_ptr<float>(), cus, cur_stream());
    return {out, part, aout};
  }
  // [2][G][C], or [4][G][C] with the second BN: [sum g | sum g (x - mean) | sum g | sum g (x2 - mean2)]
  auto part = at::empty({x2.has_value() ? 4 : 2, conv1x1_dgrad_bnred_partials(m, k, ncols, cus, pro, pmask), ncols},
                        g.options().dtype(at::kFloat));
  at::Tensor aout;
  if (want_aout) aout = at::empty_like(g);
  conv1x1_dgrad_bnred(g.data_ptr(), w.data_ptr(), out.data_ptr(), m, k, ncols, dtype_code(g.scalar_type()),
                      res.has_value() ? res->data_ptr() : nullptr, bits.has_value() ? bits->data_ptr<uint8_t>() : nullptr,
                      x.data_ptr(), mean.data_ptr<float>(), part.data_ptr<float>(), cus, cur_stream(),
                      coef.has_value() ? coef->data_ptr<float>() : nullptr, pro ? py->data_ptr() : nullptr,
                      pro ? pcoef->data_ptr<float>() : nullptr, want_aout ? aout.data_ptr() : nullptr, (int)res_h,
                      (int)res_w, pmask, x2.has_value() ? x2->data_ptr() : nullptr,
                      mean2.has_value() ? mean2->data_ptr<float>() : nullptr);
  return {out, part, aout};
}

// (coef_bwd [3C], grad_w, grad_b) from dgrad_bnred partials
std::vector<at::Tensor> bnbwd_finalize(const at::Tensor& part, double count, const at::Tensor& mean,
                                       const at::Tensor& invstd, const c10::optional<at::Tensor>& w) {
  TORCH_CHECK(part.is_cuda() && part.dim() == 3 && part.size(0) == 2 && part.scalar_type() == at::kFloat,
              "bnbwd_finalize: part must be [2, G, C] fp32");
  const int c = (int)part.size(2);
  const c10::hip::HIPGuard guard(part.get_device());
  auto opt = part.options();
  auto coef = at::empty({3 * c}, opt), gw = at::empty({c}, opt), gb = at::empty({c}, opt);
  conv1x1_bnbwd_finalize(part.data_ptr<float>(), (int)part.size(1), c, (float)(1.0 / count), mean.data_ptr<float>(),
                         invstd.data_ptr<float>(), w.has_value() ? w->data_ptr<float>() : nullptr,
                         gw.data_ptr<float>(), gb.data_ptr<float>(), coef.data_ptr<float>(), cur_stream());
  return {coef, gw, gb};
}

// dW [K, 3, 3, C] (channels_last memory [K][3][3][C]) of a pad-1 3x3 conv: dy [N, OH, OW, K]
// (NHWC), x [N, H, W, C] (NHWC), optional BN-apply+ReLU prologue on x (xcoef [2C])
at::Tensor wgrad3x3(const at::Tensor& dy, const at::Tensor& x, int64_t stride, const c10::optional<at::Tensor>& xcoef,
                    c10::optional<at::ScalarType> out_dtype) {
  check_nhwc(dy, "dy");
  check_nhwc(x, "x");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && dy.size(0) == x.size(0), "wgrad3x3: dtype / batch mismatch");
  const int nimg = (int)x.size(0), h = (int)x.size(1), w = (int)x.size(2), c = (int)x.size(3);
  const int oh = (int)dy.size(1), ow = (int)dy.size(2), kout = (int)dy.size(3);
  TORCH_CHECK(oh == (h + 2 - 3) / stride + 1 && ow == (w + 2 - 3) / stride + 1, "wgrad3x3: geometry mismatch");
  TORCH_CHECK(conv3x3_wgrad_supported(c, kout), "wgrad3x3: C and K must be multiples of 64");
  const float* xc = nullptr;
  if (xcoef.has_value()) {
    TORCH_CHECK(xcoef->is_cuda() && xcoef->scalar_type() == at::kFloat && xcoef->is_contiguous() &&
                    xcoef->numel() == 2 * (int64_t)c,
                "wgrad3x3: xcoef must be contiguous fp32 [2C]");
    xc = xcoef->data_ptr<float>();
  }
  const c10::hip::HIPGuard guard(dy.get_device());
  const int cus = device_cus(dy.get_device());
  const int64_t m = (int64_t)nimg * oh * ow;
  auto dw = at::empty({kout, 3, 3, c}, dy.options().dtype(out_dtype.value_or(dy.scalar_type())));
  auto ws = at::empty({conv3x3_wgrad_workspace_floats(m, kout, c, cus)}, dy.options().dtype(at::kFloat));
  conv3x3_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), dtype_code(dw.scalar_type()), nimg, h, w, c, oh, ow,
                (int)stride, kout, dtype_code(dy.scalar_type()), xc, ws.data_ptr<float>(), cus, cur_stream());
  return dw.permute({0, 3, 1, 2});  // [K, C, 3, 3] in channels_last memory
}

// ---- ResNet stem (csrc/conv/stem.hip): activations are torch channels_last tensors ----
void check_cl(const at::Tensor& t, int64_t c, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.size(1) == c && t.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem: ", what, " must be a channels_last [N, ", c, ", H, W] GPU tensor");
}

// x [N, cin <= 4, H, W] image (any strides, fp32 / fp16 / bf16), w [64, cin, 7, 7] (compute dtype),
// shift [64] fp32 (statistics shift, the running mean) -> (y [N, 64, OH, OW] channels_last,
// statistics partials [2, G, 64], the halo'd NHWC4 image for the weight gradient)
std::vector<at::Tensor> stem_fprop_b(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& shift) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.size(1) >= 1 && x.size(1) <= 4, "stem: x must be [N, 1-4, H, W] on the GPU");
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.size(0) == 64 && w.size(1) == x.size(1) && w.size(2) == 7 && w.size(3) == 7,
              "stem: w must be [64, cin, 7, 7]");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 || w.scalar_type() == at::kHalf, "stem: bf16 / fp16 weights");
  if (shift.has_value())
    TORCH_CHECK(shift->is_cuda() && shift->scalar_type() == at::kFloat && shift->is_contiguous() && shift->numel() == 64,
                "stem: shift must be contiguous fp32 [64]");
  const c10::hip::HIPGuard guard(x.get_device());
  const int n = (int)x.size(0), cin = (int)x.size(1), h = (int)x.size(2), wd = (int)x.size(3);
  int oh, ow, hp, wp, ph, pw;
  stem_geometry(n, h, wd, &oh, &ow, &hp, &wp, &ph, &pw);
  const int cus = device_cus(x.get_device());
  const int t = dtype_code(w.scalar_type());
  auto opt = w.options();
  auto xp = at::empty({n, hp, wp, 4}, opt);
  auto wpk = at::empty({64, 224}, opt);
  auto y = at::empty({n, 64, oh, ow}, opt.memory_format(at::MemoryFormat::ChannelsLast));
  auto part = at::empty({2, stem_fprop_rows(cus), 64}, opt.dtype(at::kFloat));
  const int64_t xs[4] = {x.stride(0), x.stride(1), x.stride(2), x.stride(3)};
  const int64_t wsd[4] = {w.stride(0), w.stride(1), w.stride(2), w.stride(3)};
  stem_pad(x.data_ptr(), dtype_code(x.scalar_type()), n, cin, h, wd, xs, xp.data_ptr(), t, cus, cur_stream());
  stem_wpack(w.data_ptr(), t, cin, wsd, wpk.data_ptr(), t, cur_stream());
  stem_fprop(xp.data_ptr(), wpk.data_ptr(), shift.has_value() ? shift->data_ptr<float>() : nullptr, y.data_ptr(),
             part.data_ptr<float>(), n, h, wd, t, cus, cur_stream());
  return {y, part, xp};
}

void check_coef(const at::Tensor& c, int64_t n, const char* what) {
  TORCH_CHECK(c.is_cuda() && c.scalar_type() == at::kFloat && c.is_contiguous() && c.numel() == n, "stem: ", what,
              " must be contiguous fp32 [", n, "]");
}

// y [N, 64, OH, OW] channels_last, coef [128] scale | shift -> (pooled [N, 64, PH, PW] channels_last,
// window indices [N, PH, PW, 64] uint8)
std::vector<at::Tensor> stem_pool_b(const at::Tensor& y, const at::Tensor& coef) {
  check_cl(y, 64, "y");
  check_coef(coef, 128, "coef");
  const c10::hip::HIPGuard guard(y.get_device());
  const int n = (int)y.size(0), oh = (int)y.size(2), ow = (int)y.size(3);
  const int ph = (oh - 1) / 2 + 1, pw = (ow - 1) / 2 + 1;
  auto p = at::empty({n, 64, ph, pw}, y.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({n, ph, pw, 64}, y.options().dtype(at::kByte));
  stem_pool_fwd(y.data_ptr(), coef.data_ptr<float>(), p.data_ptr(), idx.data_ptr<uint8_t>(), n, 2 * oh, 2 * ow,
                dtype_code(y.scalar_type()), device_cus(y.get_device()), cur_stream());
  return {p, idx};
}

void check_bwd(const at::Tensor& dp, const at::Tensor& idx, const at::Tensor& y) {
  check_cl(y, 64, "y");
  check_cl(dp, 64, "dp");
  const int64_t oh = y.size(2), ow = y.size(3);
  TORCH_CHECK(dp.scalar_type() == y.scalar_type() && dp.size(0) == y.size(0) && dp.size(2) == (oh - 1) / 2 + 1 &&
                  dp.size(3) == (ow - 1) / 2 + 1,
              "stem: pooled gradient does not match y");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte && idx.is_contiguous() && idx.dim() == 4 &&
                  idx.size(0) == dp.size(0) && idx.size(1) == dp.size(2) && idx.size(2) == dp.size(3) && idx.size(3) == 64,
              "stem: idx must be the forward's [N, PH, PW, 64] uint8 indices");
}

// [2, G, 64] partials of sum(g), sum(g * (y - mean)); g = ReLU-masked pool backward of dp
at::Tensor stem_reduce_b(const at::Tensor& dp, const at::Tensor& idx, const at::Tensor& y, const at::Tensor& coef,
                         const at::Tensor& mean) {
  check_bwd(dp, idx, y);
  check_coef(coef, 128, "coef");
  check_coef(mean, 64, "mean");
  const c10::hip::HIPGuard guard(y.get_device());
  const int cus = device_cus(y.get_device());
  auto part = at::empty({2, stem_reduce_rows(cus), 64}, y.options().dtype(at::kFloat));
  stem_bwd_reduce(dp.data_ptr(), idx.data_ptr<uint8_t>(), y.data_ptr(), coef.data_ptr<float>(), mean.data_ptr<float>(),
                  part.data_ptr<float>(), (int)y.size(0), 2 * (int)y.size(2), 2 * (int)y.size(3),
                  dtype_code(y.scalar_type()), cus, cur_stream());
  return part;
}

// weight gradient [64, cin, 7, 7] (w's strides and dtype); cb [192] = the BN backward's A | B | K
at::Tensor stem_wgrad_b(const at::Tensor& dp, const at::Tensor& idx, const at::Tensor& y, const at::Tensor& coef,
                        const at::Tensor& cb, const at::Tensor& xp, const at::Tensor& w) {
  check_bwd(dp, idx, y);
  check_coef(coef, 128, "coef");
  check_coef(cb, 192, "cb");
  const int n = (int)y.size(0), oh = (int)y.size(2), ow = (int)y.size(3);
  TORCH_CHECK(xp.is_cuda() && xp.is_contiguous() && xp.dim() == 4 && xp.size(0) == n && xp.size(1) == 2 * (oh - 1) + 7 &&
                  xp.size(2) == 2 * (ow - 1) + 8 && xp.size(3) == 4 && xp.scalar_type() == y.scalar_type(),
              "stem: xp must be the forward's halo'd image");
  TORCH_CHECK(w.dim() == 4 && w.size(0) == 64 && w.size(1) >= 1 && w.size(1) <= 4 && w.size(2) == 7 && w.size(3) == 7,
              "stem: w must be [64, cin, 7, 7]");
  const c10::hip::HIPGuard guard(y.get_device());
  const int cus = device_cus(y.get_device());
  auto dw = at::empty_like(w);
  auto ws = at::empty({(int64_t)stem_wgrad_parts(cus) * 64 * 224}, y.options().dtype(at::kFloat));
  const int64_t st[4] = {dw.stride(0), dw.stride(1), dw.stride(2), dw.stride(3)};
  stem_wgrad(dp.data_ptr(), idx.data_ptr<uint8_t>(), y.data_ptr(), coef.data_ptr<float>(), cb.data_ptr<float>(),
             xp.data_ptr(), ws.data_ptr<float>(), dw.data_ptr(), dtype_code(dw.scalar_type()), (int)w.size(1), st, n,
             2 * oh, 2 * ow, dtype_code(y.scalar_type()), cus, cur_stream());
  return dw;
}

// bottleneck conv3 backward, both BNs fused: dm / y3 [M, C4], y2 [M, W] (dense NHWC views), w3
// [C4, W] (any 2-D view of the [C4, W, 1, 1] weight, contiguous), cb3 [3 C4], c2 [2 W], mean2 [W]
// -> (dz2 [M, W], bn2 partials [2, G, W], dW3 [C4, W] in w3's dtype)
std::vector<at::Tensor> conv3_bwd_b(const at::Tensor& dm, const at::Tensor& y3, const at::Tensor& y2,
                                    const at::Tensor& w3, const at::Tensor& cb3, const at::Tensor& c2,
                                    const at::Tensor& mean2) {
  auto chk2 = [](const at::Tensor& t, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.is_contiguous(), "conv3_bwd: ", what, " must be a contiguous 2-D GPU tensor");
  };
  chk2(dm, "dm");
  chk2(y3, "y3");
  chk2(y2, "y2");
  chk2(w3, "w3");
  const int64_t m = dm.size(0), c4 = dm.size(1), w = y2.size(1);
  TORCH_CHECK(y3.sizes() == dm.sizes() && y2.size(0) == m && w3.size(0) == c4 && w3.size(1) == w,
              "conv3_bwd: shape mismatch");
  TORCH_CHECK(dm.scalar_type() == y3.scalar_type() && dm.scalar_type() == y2.scalar_type() &&
                  dm.scalar_type() == w3.scalar_type(),
              "conv3_bwd: one dtype");
  TORCH_CHECK(conv3_bwd_fused_supported((int)c4, (int)w), "conv3_bwd: unsupported channel counts");
  auto f32 = [](const at::Tensor& t, int64_t n, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n, "conv3_bwd: ",
                what, " must be contiguous fp32 [", n, "]");
  };
  f32(cb3, 3 * c4, "cb3");
  f32(c2, 2 * w, "c2");
  f32(mean2, w, "mean2");
  const c10::hip::HIPGuard guard(dm.get_device());
  const int cus = device_cus(dm.get_device());
  const int g = conv3_bwd_fused_parts(cus);
  auto dz2 = at::empty({m, w}, y2.options());
  auto part2 = at::empty({2, g, w}, y2.options().dtype(at::kFloat));
  auto ws = at::empty({(int64_t)g * c4 * w}, y2.options().dtype(at::kFloat));
  auto dw3 = at::empty({c4, w}, w3.options());
  conv3_bwd_fused(dm.data_ptr(), y3.data_ptr(), y2.data_ptr(), w3.data_ptr(), cb3.data_ptr<float>(), c2.data_ptr<float>(),
                  mean2.data_ptr<float>(), dz2.data_ptr(), part2.data_ptr<float>(), ws.data_ptr<float>(), dw3.data_ptr(),
                  dtype_code(dw3.scalar_type()), m, (int)c4, (int)w, dtype_code(dm.scalar_type()), cus, cur_stream());
  return {dz2, part2, dw3};
}

}  // namespace

void bind_conv(pybind11::module_& root) {
  auto m = root.def_submodule("conv", "gfx950 implicit-GEMM NHWC convolutions");
  m.def("tap_fprop", &tap_fprop, pybind11::arg("input"), pybind11::arg("weight"), pybind11::arg("out"),
        pybind11::arg("oh"), pybind11::arg("ow"), pybind11::arg("ish"), pybind11::arg("isw"), pybind11::arg("osh"),
        pybind11::arg("osw"), pybind11::arg("oph"), pybind11::arg("opw"), pybind11::arg("dh"), pybind11::arg("dw"),
        pybind11::arg("scale") = pybind11::none(), pybind11::arg("bias") = pybind11::none(),
        pybind11::arg("residual") = pybind11::none(), pybind11::arg("relu") = false,
        pybind11::arg("mask") = pybind11::none(), pybind11::arg("stats") = pybind11::none(),
        pybind11::arg("stats_shift") = pybind11::none(), pybind11::arg("pcoef") = pybind11::none(),
        pybind11::arg("red_x") = pybind11::none(), pybind11::arg("red_coef") = pybind11::none(),
        pybind11::arg("red_mean") = pybind11::none());
  m.def("hfp_supported", [](int64_t n, int64_t h, int64_t w, int64_t c, int64_t kout) {
    ConvTapArgs a{};
    void* aligned = reinterpret_cast<void*>(static_cast<uintptr_t>(256));  // alignment checks only
    a.in = a.wt = aligned;
    a.out = aligned;
    a.n = (int)n;
    a.ih = a.oh = a.oht = (int)h;
    a.iw = a.ow = a.owt = (int)w;
    a.c = (int)c;
    a.kout = (int)kout;
    a.ish = a.isw = a.osh = a.osw = 1;
    a.ntaps = 9;
    for (int t = 0; t < 9; ++t) {
      a.dh[t] = t / 3 - 1;
      a.dw[t] = t % 3 - 1;
    }
    a.dtype = kBF16;
    return conv_hfp_supported(a);
  });
  m.def("wgrad", &wgrad, pybind11::arg("x"), pybind11::arg("dy"), pybind11::arg("dw"), pybind11::arg("ish"),
        pybind11::arg("isw"), pybind11::arg("dh"), pybind11::arg("dw_taps"),
        pybind11::arg("xcoef") = pybind11::none());
  m.def("force_fprop_cfg", &conv_force_fprop_cfg);
  m.def("force_wgrad_variant", &conv_force_wgrad_variant);
  m.def("halo_wgrad_supported", &halo_wgrad_supported, pybind11::arg("n"), pybind11::arg("h"), pybind11::arg("w"),
        pybind11::arg("c"), pybind11::arg("kout"), pybind11::arg("stride") = 1);
  m.attr("WGRAD_HALO") = kWgradHalo;
  m.def("bn1x1", &bn1x1, pybind11::arg("a"), pybind11::arg("w"), pybind11::arg("w_kmajor_out") = false,
        pybind11::arg("pcoef") = pybind11::none(), pybind11::arg("shift") = pybind11::none(),
        pybind11::arg("stats") = false, pybind11::arg("res") = pybind11::none(),
        pybind11::arg("py") = pybind11::none(), pybind11::arg("want_aout") = false, pybind11::arg("res_h") = 0,
        pybind11::arg("res_w") = 0);
  m.def("bn_finalize", &bn_finalize);
  m.def("hfp_set_mode", &conv_hfp_set_mode, pybind11::arg("mode"));
  m.def("subsample2x", &subsample2x, pybind11::arg("x"), pybind11::arg("n"), pybind11::arg("h"), pybind11::arg("w"));
  m.def("tap_weights", &tap_weights, pybind11::arg("w"), pybind11::arg("taps"));
  m.def("spatial_broadcast", &spatial_broadcast_b, pybind11::arg("g"), pybind11::arg("h"), pybind11::arg("w"),
        pybind11::arg("scale"));
  m.def("bn1x1_addrelu", &bn1x1_addrelu, pybind11::arg("a"), pybind11::arg("res"), pybind11::arg("pcoef"),
        pybind11::arg("w"), pybind11::arg("shift") = pybind11::none(), pybind11::arg("out") = pybind11::none(),
        pybind11::arg("split") = false, pybind11::arg("res_coef") = pybind11::none());
  m.def("wgrad3x3", &wgrad3x3, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("stride"),
        pybind11::arg("xcoef") = pybind11::none(), pybind11::arg("out_dtype") = pybind11::none());
  m.def("dgrad_bnred", &dgrad_bnred, pybind11::arg("g"), pybind11::arg("w"), pybind11::arg("res"),
        pybind11::arg("bits"), pybind11::arg("x"), pybind11::arg("mean"), pybind11::arg("coef") = pybind11::none(),
        pybind11::arg("py") = pybind11::none(), pybind11::arg("pcoef") = pybind11::none(),
        pybind11::arg("want_aout") = false, pybind11::arg("res_h") = 0, pybind11::arg("res_w") = 0,
        pybind11::arg("x2") = pybind11::none(), pybind11::arg("mean2") = pybind11::none());
  m.def("bnbwd_finalize", &bnbwd_finalize);
  m.def("ks1x1_supported", [](int64_t m, int64_t k, int64_t ncols) { return conv1x1_ks_supported(m, (int)k, (int)ncols); });
  m.def("part_payload", &part_payload, pybind11::arg("part"), pybind11::arg("count"),
        pybind11::arg("shift") = pybind11::none());
  m.def("conv3_bwd", &conv3_bwd_b);
  m.def("supports_conv3_bwd", &conv3_bwd_fused_supported);
  m.def("stem_fprop", &stem_fprop_b, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("shift") = pybind11::none());
  m.def("stem_pool", &stem_pool_b);
  m.def("stem_reduce", &stem_reduce_b);
  m.def("stem_wgrad", &stem_wgrad_b);
  m.def("wgrad1x1", &wgrad1x1, pybind11::arg("g"), pybind11::arg("x"), pybind11::arg("xcoef") = pybind11::none(),
        pybind11::arg("out_dtype") = pybind11::none());
}

}  // namespace apex_amd
