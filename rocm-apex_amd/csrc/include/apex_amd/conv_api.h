// Torch-free launchers for the gfx950 implicit-GEMM convolutions (csrc/conv/conv_igemm.hip) on
// NHWC (torch channels_last) bf16/fp16 activations.  They replace MIOpen for the ResNet 3x3 /
// strided convolutions, where MIOpen runs at 20-30 % of the MFMA roofline on MI355X
// (profiles/conv_shapes_miopen_r02.jsonl).  Reference capability: the fused convolutions of
// apex/contrib/bottleneck (cudnn-frontend graphs, apex/contrib/csrc/bottleneck/bottleneck.cpp).
//
// ONE "tap" formulation covers forward and data-gradient:
//   out[n, oh*osh + oph, ow*osw + opw, k] = sum_{t < ntaps, c} in[n, oh*ish + dh[t], ow*isw + dw[t], c]
//                                                             * w[k][t][c]
// with zero padding outside `in`.  Forward: taps (r - pad, s - pad), ish = stride.  Data gradient
// of a stride-1 conv: the forward over dY with the flipped, transposed weight w'[c][t][k].  Data
// gradient of a stride-2 conv: one launch per output phase (oph, opw), each with the 1-4 taps
// that reach that phase (osh = osw = 2).  Weight gradient: its own kernel (split over pixels).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

constexpr int kConvMaxTaps = 9;

struct ConvTapArgs {
  const void* in;   // [n][h][w][c]
  const void* wt;   // [kout][ntaps][c]
  void* out;        // [n][oht][owt][kout]
  int n, ih, iw, c;  // input tensor
  int oh, ow;       // output grid computed (per image)
  int oht, owt;     // output tensor spatial dims
  int kout;
  int ish, isw;     // input step per output step
  int osh, osw, oph, opw;  // output placement
  int ntaps;
  int dh[kConvMaxTaps], dw[kConvMaxTaps];
  int dtype;        // kBF16 / kF16
  // optional fprop epilogue, applied to the fp32 accumulator before the store (null = off):
  //   y = act(acc * scale[k] + bias[k] + residual[pix, k]),  act = ReLU when relu != 0
  // scale / bias are fp32 [kout]; residual has the output tensor's layout and dtype
  const float* scale = nullptr;
  const float* bias = nullptr;
  const void* residual = nullptr;
  int relu = 0;
  // optional gradient mask (data-gradient launches of a ReLU chain): y *= (mask[pix, k] > 0), with
  // `mask` the producing layer's ReLU output in the output tensor's layout and dtype — the dReLU
  // of the previous stage applied in this dconv's epilogue
  const void* mask = nullptr;
  // optional BN statistics of the fprop output (the consuming training-mode batch norm):
  // per-M-tile partial sums of (y - shift) and (y - shift)^2, [2][conv_tap_stats_tiles][kout]
  // (rows = the chosen tile configuration's M tiles)
  // fp32, finalized by conv1x1_bn_finalize (no separate statistics pass over y)
  float* stats = nullptr;
  const float* stats_shift = nullptr;
  // optional BN backward reduction instead (data-gradient launches whose output is the gradient of
  // a BN + ReLU's output; red_x = that BN's input in the output's layout and dtype): the stored
  // value is masked by red_x * red_coef[k] + red_coef[K + k] > 0 (the forward ReLU recomputed) and
  // `stats` gets the per-M-tile sums of it and of it * (red_x - red_mean[k]) — the BN's backward
  // reduction, finalized by conv1x1_bnbwd_finalize (no reduction pass over the gradient)
  const void* red_x = nullptr;
  const float* red_coef = nullptr;
  const float* red_mean = nullptr;
};

// shape constraints: c % 64 == 0, kout % 64 == 0, 16-byte aligned pointers
bool conv_tap_supported(const ConvTapArgs& a);
// A/B hook: force one fprop tile configuration (-1 = per-shape choice); see conv_igemm.hip
void conv_force_fprop_cfg(int cfg);
void conv_tap_fprop(const ConvTapArgs& a, int cus, hipStream_t s);
// number of M tiles of a tap fprop launch (the stats partial rows)
int conv_tap_stats_tiles(const ConvTapArgs& a, int cus);
// spatial-tile 3x3 kernel (csrc/conv/conv3x3_sp.hip): 64 -> 64 channels, stride 1, identity
// placement, no fused epilogue but the BN statistics; conv_tap_fprop routes supported launches to
// it by default (APEX_AMD_CONV_SP=0 disables; forced tile configuration 21 selects it)
bool conv_sp_supported(const ConvTapArgs& a);
bool conv_sp_default(const ConvTapArgs& a);
int conv_sp_grid(const ConvTapArgs& a, int cus);
void conv_sp_fprop(const ConvTapArgs& a, int cus, hipStream_t s);

// weight gradient: dw[k][t][c] = sum_{n,oh,ow} dy[n,oh,ow,k] * x[n, oh*ish + dh[t], ow*isw + dw[t], c]
// (dy = `out` geometry with osh = osw = 1, oph = opw = 0; x = `in`).  fp32 result [kout][ntaps][c]
// through split-K partials in `ws` (conv_wgrad_workspace_floats), summed in a fixed order.
bool conv_wgrad_supported(const ConvTapArgs& a);
// A/B hook: force one weight-gradient variant (launch_plan.h conv_wgrad; -1 = per-shape default;
// kWgradHalo = the halo-tile kernel below)
void conv_force_wgrad_variant(int v);
constexpr int kWgradHalo = 5;
// halo-tile 3x3 stride-1 weight gradient (csrc/conv/conv3x3_wgrad.hip): one workgroup per
// (output-channel block x all 9 taps x 64 input channels) over a range of pixel tiles, the input
// halo staged once per tile; the default engine of conv_wgrad wherever it applies
bool conv_hwgrad_supported(const ConvTapArgs& a);
int64_t conv_hwgrad_workspace_floats(const ConvTapArgs& a, int cus);
void conv_hwgrad(const ConvTapArgs& a, const void* dy, void* dw_out, int out_dtype, float* ws, int cus,
                 hipStream_t s);
int64_t conv_wgrad_workspace_floats(const ConvTapArgs& a, int cus);
void conv_wgrad(const ConvTapArgs& a, const void* dy, void* dw_out, int out_dtype, float* ws, int cus,
                hipStream_t s);

// ---- memory-bound 1x1 convolutions with the batch norm fused in (csrc/conv/conv1x1_bn.hip) ----
// y[M][ncols] = pro(a[M][k]) . W^T with W [ncols][k] (forward) or, w_kmajor_out, W [k][ncols]
// (data gradient dX = dY . W of a [k-out][ncols-in] conv weight).  pcoef (nullable, [2][k]
// scale | shift): pro(a) = relu(a * scale + shift), the producing batch norm applied on load.
// part (nullable, [2][G][ncols] with G = conv1x1_bn_partials(...)): per-workgroup sums of
// (y - shift) and (y - shift)^2 for the consuming batch norm, finalized by conv1x1_bn_finalize.
// Shapes: k in {64, 128, 256, 512}, ncols % 64 == 0, bf16 / fp16, 16-byte aligned rows.
bool conv1x1_bn_supported(int64_t m, int k, int ncols);
// y [N][ceil(h/2)][ceil(w/2)][c] = x [N][h][w][c] at even (y, x): a stride-2 1x1 conv's operand
// (csrc/conv/layout.hip; 16-bit, c % 8 == 0, 16-byte aligned)
void conv_subsample2x(const void* x, void* y, int n, int h, int w, int c, int dtype, int cus, hipStream_t s);
// dst[c][j][k] = w[k][taps[j]][c]: the data-gradient weight image [C][ntaps][K] of a channels_last
// [K][rs][C] 16-bit weight (rs = R * S), for an ordered tap subset (1..9 taps)
void conv_tap_weights(const void* w, void* dst, int k, int c, int rs, const int* taps, int ntaps, hipStream_t s);
int conv1x1_bn_partials(int64_t m, int k, int ncols, bool pro, int cus, bool pro_addrelu = false);
void conv1x1_bn(const void* a, const void* w, void* y, int64_t m, int k, int ncols, bool w_kmajor_out, int dtype,
                const float* pcoef, const float* shift, float* part, int cus, hipStream_t s,
                const void* res = nullptr,    // nullable [M][ncols]: y += res (same dtype)
                const void* py = nullptr,     // dgrad form: BN-backward prologue a' = c0 a + c1 py + c2,
                void* aout = nullptr,         //   pcoef [3][k]; aout (nullable) receives a' [M][k]
                bool pro_relu = false,        // forward form with py: a' = relu(c0 a + c1 py + c2) (the
                uint8_t* bout = nullptr,      //   block output: BN + residual + ReLU), bits to bout
                int res_h = 0, int res_w = 0,  // > 0: res is [N][ceil(res_h/2)][ceil(res_w/2)][ncols], the
                                               //   stride-2 subsample's gradient, added at even (y, x) only
                bool pc_split = false,         // add + ReLU form: pcoef = the output BN's [2][k] and pc_res
                const float* pc_res = nullptr,   //   the residual BN's [2][k] (null: identity) instead of [4][k]
                bool pro_mask = false);          // BN-backward prologue with the ReLU mask recomputed from py:
                                                 //   pcoef [5][k] = A | B | K | fwd scale | fwd shift,
                                                 //   a' = A (py * scale + shift > 0 ? a : 0) + B py + K
// batch statistics from the partials: save_mean / save_invstd, running-stat EMA (nullable),
// coef = [scale | shift] of the apply (w, b nullable = affine-free)
void conv1x1_bn_finalize(const float* part, int g, int c, float n, const float* shift, const float* w, const float* b,
                         float eps, float momentum, float* rmean, float* rvar, float* save_mean, float* save_invstd,
                         float* coef, hipStream_t s);

// bn_group > 1: this rank's Welford payload [mean(C) | M2(C) | n] from the partials (the group
// exchange + csrc/groupbn stats merge replace conv1x1_bn_finalize)
void conv1x1_bn_part_payload(const float* part, int g, int c, float n, const float* shift, float* payload,
                             hipStream_t s);

// dW [n][k] (out_dtype) = sum_m g[m][n] . pro(x[m][k]), pro = relu(x * xcoef[k] + xcoef[K + k]) when
// xcoef is non-null; fp32 split partials in ws (conv1x1_wgrad_workspace_floats), fixed-order sum
bool conv1x1_wgrad_supported(int64_t m, int n, int k);
int64_t conv1x1_wgrad_workspace_floats(int64_t m, int n, int k, int cus);
void conv1x1_wgrad(const void* g, const void* x, void* dw, int out_dtype, int64_t m, int n, int k, int dtype,
                   const float* xcoef, float* ws, int cus, hipStream_t s);

// dgrad form with the BN-backward reduction of the block below in the epilogue:
// out = mask(g . W + res) (mask = bits, that BN's forward ReLU bit mask) and per-column partial
// sums [2][G][ncols] of out and out * (x - mean); G = conv1x1_dgrad_bnred_partials(...).
// conv1x1_bnbwd_finalize turns them into grad_w, grad_b and coef_bwd [3][C].
int conv1x1_dgrad_bnred_partials(int64_t m, int k, int ncols, int cus, bool pro = false, bool pro_mask = false);
// bits null: mask = x * rcoef[c] + rcoef[ncols + c] > 0 (a plain BN + ReLU, recomputed);
// py / pcoef (optional): the BN-backward operand prologue a' = pcoef0 g + pcoef1 py + pcoef2 of
// the BN below this conv, with a' written to aout (nullable) for the weight gradient
void conv1x1_dgrad_bnred(const void* g, const void* w, void* out, int64_t m, int k, int ncols, int dtype,
                         const void* res, const uint8_t* bits, const void* x, const float* mean, float* part, int cus,
                         hipStream_t s, const float* rcoef = nullptr, const void* py = nullptr,
                         const float* pcoef = nullptr, void* aout = nullptr, int res_h = 0, int res_w = 0,
                         bool pro_mask = false,  // pcoef [5][k] with the recomputed ReLU mask (see conv1x1_bn)
                         // a second BN fed by the same masked gradient (the downsample BN): part is
                         // then [4][G][ncols] = [sum g | sum g (x - mean) | sum g | sum g (x2 - mean2)]
                         const void* x2 = nullptr, const float* mean2 = nullptr);
void conv1x1_bnbwd_finalize(const float* part, int g, int c, float inv_n, const float* mean, const float* istd,
                            const float* w, float* gw, float* gb, float* coef, hipStream_t s);

// 3x3 (pad 1, stride 1 / 2) weight gradient on the split-M kernel with the input gathered per
// tap: dw [kout][9][c] = sum over output pixels dy[p][k] * pro(x[tap-shifted p][c]), zero padding;
// pro = relu(x * xcoef[c] + xcoef[C + c]) when xcoef (the producing BN + ReLU), padding stays 0
bool conv3x3_wgrad_supported(int c, int kout);
int64_t conv3x3_wgrad_workspace_floats(int64_t m, int kout, int c, int cus);
void conv3x3_wgrad(const void* g, const void* x, void* dw, int out_dtype, int nimg, int h, int w, int c, int oh,
                   int ow, int stride, int kout, int dtype, const float* xcoef, float* ws, int cus, hipStream_t s);

// ---- ResNet stem (csrc/conv/stem.hip): 7x7/2 conv (1-4 -> 64 channels, pad 3) + BN + ReLU +
// 3x3/2 max pool (pad 1).  Compute dtype t = bf16 / fp16; activations NHWC.
// image -> halo'd NHWC4 xp [n][hp][wp][4]; strides of the [n, cin, h, w] image in elements
void stem_geometry(int n, int h, int w, int* oh, int* ow, int* hp, int* wp, int* ph, int* pw);
int stem_fprop_rows(int cus);   // partial rows G of stem_fprop's statistics [2][G][64]
int stem_reduce_rows(int cus);  // partial rows G of stem_bwd_reduce's sums [2][G][64]
int stem_wgrad_parts(int cus);  // fp32 partial slabs [G][64][224] of stem_wgrad's workspace
void stem_pad(const void* x, int x_t, int n, int cin, int h, int w, const int64_t* strides, void* xp, int t,
              int cus, hipStream_t s);
// weight [64, cin, 7, 7] (strided, dtype w_t) -> packed [64][224], k = r * 32 + s * 4 + c
void stem_wpack(const void* w, int w_t, int cin, const int64_t* strides, void* wp, int t, hipStream_t s);
// y [n*oh*ow][64] = conv(xp, wp) + statistics partials of (y - shift)
void stem_fprop(const void* xp, const void* wp, const float* shift, void* y, float* part, int n, int h, int w,
                int t, int cus, hipStream_t s);
// p / idx [n][ph][pw][64] = maxpool(relu(y * coef[c] + coef[64 + c])), idx = window position
void stem_pool_fwd(const void* y, const float* coef, void* p, uint8_t* idx, int n, int h, int w, int t, int cus,
                   hipStream_t s);
// [2][G][64] partials of sum(g) and sum(g * (y - mean)), g = ReLU-masked pool-backward of dp
void stem_bwd_reduce(const void* dp, const uint8_t* idx, const void* y, const float* coef, const float* mean,
                     float* part, int n, int h, int w, int t, int cus, hipStream_t s);
// dw (strided [64, cin, 7, 7], dtype dw_t) = sum_p dx[p] (x) im2col(xp)[p], dx = cb0 g + cb1 y + cb2
void stem_wgrad(const void* dp, const uint8_t* idx, const void* y, const float* coef, const float* cb,
                const void* xp, float* ws, void* dw, int dw_t, int cin, const int64_t* dw_strides, int n, int h, int w,
                int t, int cus, hipStream_t s);

// ---- bottleneck conv3 backward with both batch norms fused (csrc/conv/conv3_bwd.hip) ----
// dx3 = cb3[0] dm + cb3[1] y3 + cb3[2] (bn3's dx, never stored); dz2 = relu2-mask(dx3 . W3) written
// with bn2's backward partial sums part2 [2][G][W] (sum g, sum g (y2 - mean2)); dW3 [C4][W] (dtype
// dw_t) = dx3^T relu(y2 c2[0] + c2[1]) through fp32 slabs ws [G][C4][W]; G = conv3_bwd_fused_parts
bool conv3_bwd_fused_supported(int c4, int w);
int conv3_bwd_fused_parts(int cus);
void conv3_bwd_fused(const void* dm, const void* y3, const void* y2, const void* w3, const float* cb3, const float* c2,
                     const float* mean2, void* dz2, float* part2, float* ws, void* dw3, int dw_t, int64_t m, int c4,
                     int w, int t, int cus, hipStream_t s);

}  // namespace apex_amd
