// Host-side launch planners of the native kernels: tensor shapes -> grid / split counts /
// workspace sizes.  Host-only and dependency-free (no HIP runtime), so tools/host_checks.cpp can
// sweep them under AddressSanitizer + UBSan on the CPU (tools/host_sanitize.sh): a wrong value
// here becomes an out-of-bounds access on the GPU.
#pragma once

#include <cstdint>

#include "apex_amd/conv_api.h"
#include "apex_amd/gemm_api.h"

namespace apex_amd {
namespace plan {

// ---- implicit-GEMM convolutions (csrc/conv/conv_igemm.hip) ----
constexpr int kWgradBK = 64;   // wgrad pixels per K-step

struct WgPlan {
  int bm, bn, tiles, splits, chunk;
};

// wgrad: (kout x ntaps*c) output tiles x pixel splits (fp32 partial per split, fixed-order reduce).
// variant 0: wgrad_kernel, 128 x 128 tiles when kout and c allow, else 64 x 64; variants 1-4:
// wgrad2_kernel (buffer-load staging) with (bm, bn) = (64, 64), (128, 128), (128, 64), (64, 128)
constexpr int kWgradVariants = 5;
inline bool conv_wgrad_variant_ok(const ConvTapArgs& a, int v) {
  static const int bm[kWgradVariants] = {64, 64, 128, 128, 64}, bn[kWgradVariants] = {64, 64, 128, 64, 128};
  if (v < 0 || v >= kWgradVariants) return false;
  if (v == 0) return true;
  const int64_t xb = (int64_t)a.n * a.ih * a.iw * a.c * 2, db = (int64_t)a.n * a.oh * a.ow * a.kout * 2;
  return a.kout % bm[v] == 0 && (a.ntaps * a.c) % bn[v] == 0 && a.c % bn[v] == 0 && xb < (1ll << 31) &&
         db < (1ll << 31);
}
inline WgPlan conv_wgrad(const ConvTapArgs& a, int cus, int variant = 0) {
  WgPlan p;
  static const int vbm[kWgradVariants] = {0, 64, 128, 128, 64}, vbn[kWgradVariants] = {0, 64, 128, 64, 128};
  if (!conv_wgrad_variant_ok(a, variant)) variant = 0;
  const bool big = a.kout % 128 == 0 && a.c % 128 == 0;
  p.bm = variant ? vbm[variant] : (big ? 128 : 64);
  p.bn = variant ? vbn[variant] : (big ? 128 : 64);
  p.tiles = (a.kout / p.bm) * (a.ntaps * a.c / p.bn);
  const int64_t m = (int64_t)a.n * a.oh * a.ow;
  // resident workgroups per CU (LDS ring: 3 stages x 64 pixels x (bm + bn) x 2 B) x two rounds
  const int per_cu = variant ? (int)(160 * 1024 / (3 * 64 * (p.bm + p.bn) * 2)) : (big ? 1 : 2);
  const int target = cus * 2 * (per_cu < 1 ? 1 : per_cu);
  int64_t s = (target + p.tiles - 1) / p.tiles;
  const int64_t max_s = (m + 16 * kWgradBK - 1) / (16 * kWgradBK);  // >= 16 K-steps per workgroup
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  int64_t chunk = (m + s - 1) / s;
  chunk = (chunk + kWgradBK - 1) / kWgradBK * kWgradBK;
  p.chunk = (int)chunk;
  p.splits = (int)((m + chunk - 1) / chunk);
  return p;
}

// fprop tile configurations (conv_igemm.hip): 0-6 = fprop_kernel (BM 256; the < 2 GiB-or-larger
// fallback), 7-13 = fprop2_kernel (buffer-load staging, 64 x 64+ per wave), 14-20 = fprop3_kernel
// (persistent, transposed accumulators, register epilogue).  (BM, BN) per index:
constexpr int kConvCfgs = 21;
inline int conv_fprop_bm(int cfg) {
  static const int bm[kConvCfgs] = {256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 128,
                                    128, 256, 128, 256, 128, 128, 128, 256, 128, 256};
  return cfg >= 0 && cfg < kConvCfgs ? bm[cfg] : 256;
}
inline int conv_fprop_bn(int cfg) {
  static const int bn[kConvCfgs] = {128, 64, 128, 64, 128, 64, 256, 64, 64, 128, 128,
                                    128, 256, 256, 64, 64, 128, 128, 128, 256, 64};
  return cfg >= 0 && cfg < kConvCfgs ? bn[cfg] : 64;
}
// fprop2 needs the input / weight byte ranges to fit a buffer descriptor (< 2 GiB)
inline bool conv_fprop2_ok(const ConvTapArgs& a) {
  const int64_t xb = (int64_t)a.n * a.ih * a.iw * a.c * 2, wb = (int64_t)a.kout * a.ntaps * a.c * 2;
  return xb < (1ll << 31) && wb < (1ll << 31);
}
// forced >= 0 overrides when legal.  Defaults from the r04 sweeps of every ResNet-50 3x3 / strided
// 1x1 shape, forward and data gradient, bs 256 (profiles/conv_cfg_sweep_r04{,b}.jsonl):
//  * <= 128 output channels: fprop2 8 waves x (32 px x 64 ch), 2 stages (cfg 7, two workgroups /
//    16 waves per CU: 109 us at 56x56x64 vs 111 for fprop_kernel's cfg 5, 88.7 vs 90.8 at
//    28x28x128);
//  * wider: fprop2 256 x 256 (cfg 12) while it still gives >= 3/4 of a wave of workgroups, else
//    128 x 128 (cfg 11) — 5-20 % faster than the fprop_kernel choices at stages 2-4.
// The persistent fprop3 tiles (cfg 14-20) measured within +-5 % of these (no fill / drain to
// win at 16 waves per CU) and stay opt-in.  > 2 GiB operands: fprop_kernel (r02 choices).
inline int conv_fprop_cfg(const ConvTapArgs& a, int cus, int forced) {
  auto ok = [&](int cfg) {
    return a.kout % conv_fprop_bn(cfg) == 0 && (cfg < 7 || conv_fprop2_ok(a));
  };
  if (forced >= 0 && forced < kConvCfgs && ok(forced)) return forced;
  const int64_t m = (int64_t)a.n * a.oh * a.ow;
  auto tiles = [&](int cfg) {
    return (m + conv_fprop_bm(cfg) - 1) / conv_fprop_bm(cfg) * (a.kout / conv_fprop_bn(cfg));
  };
  if (conv_fprop2_ok(a)) {
    if (a.kout <= 128) return 7;
    if (a.kout % 256 == 0 && 4 * tiles(12) >= 3 * (int64_t)cus) return 12;
    if (a.kout % 128 == 0) return 11;
    return 7;
  }
  const int64_t tiles_m = (m + 255) / 256;
  if (a.kout <= 128) return 5;
  if (a.kout % 256 == 0 && tiles_m * (a.kout / 256) >= cus / 2) return 6;
  return a.kout % 128 == 0 ? 4 : 5;
}

// ---- GEMM (csrc/gemm/gemm_mfma.hip, 256 x 256 x 64 tiles) ----
constexpr int kGemmBM = 256, kGemmBN = 256, kGemmBK = 64;

// number of K chunks for a split-K launch of g (1 = no split); chunk length in *kchunk
inline int gemm_splitk_parts(const GemmArgs& g, int cus, int* kchunk) {
  *kchunk = g.k;
  if (g.epilogue != kEpiNone || g.k % kGemmBK || g.n % 8) return 1;
  const int64_t tiles = (int64_t)((g.m + kGemmBM - 1) / kGemmBM) * ((g.n + kGemmBN - 1) / kGemmBN);
  if (tiles >= cus || g.k < 2048) return 1;
  int64_t sp = (cus + tiles - 1) / tiles;
  if (sp > g.k / 1024) sp = g.k / 1024;
  if (sp < 2) return 1;
  const int chunk = (int)(((g.k + sp - 1) / sp + kGemmBK - 1) / kGemmBK * kGemmBK);
  *kchunk = chunk;
  return (g.k + chunk - 1) / chunk;
}

// row partitions of the column-sum (bias-gradient) partial pass
inline int colsum_parts(int64_t m, int n, int cus) {
  const int gx = (n / 8 + 31) / 32;
  int64_t p = ((int64_t)cus * 4 + gx - 1) / gx;
  const int64_t cap = (m + 7) / 8;
  if (p > cap) p = cap;
  if (p > 512) p = 512;
  return (int)(p < 1 ? 1 : p);
}

// ---- LayerNorm backward (csrc/norm/layer_norm_bwd.hip) ----
// persistent grid: enough resident blocks to saturate HBM, few enough that the gamma/beta
// partial slab stays small
inline int ln_bwd_grid(int64_t ngroups, int cus) {
  const int64_t cap = (int64_t)cus * 2;
  return (int)(ngroups < cap ? (ngroups > 0 ? ngroups : 1) : cap);
}

}  // namespace plan
}  // namespace apex_amd
