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
constexpr int kConvBM = 256;   // fprop output-pixel tile
constexpr int kWgradBK = 64;   // wgrad pixels per K-step

struct WgPlan {
  int bm, bn, tiles, splits, chunk;
};

// wgrad: (kout x ntaps*c) output tiles x pixel splits (fp32 partial per split, fixed-order reduce)
inline WgPlan conv_wgrad(const ConvTapArgs& a, int cus) {
  WgPlan p;
  const bool big = a.kout % 128 == 0 && a.c % 128 == 0;
  p.bm = big ? 128 : 64;
  p.bn = big ? 128 : 64;
  p.tiles = (a.kout / p.bm) * (a.ntaps * a.c / p.bn);
  const int64_t m = (int64_t)a.n * a.oh * a.ow;
  const int target = cus * (big ? 2 : 4);  // resident workgroups per CU (LDS ring) x two rounds
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

// fprop tile configuration index (conv_igemm.hip FC0..FC6); forced >= 0 overrides when legal.
// Measured on MI355X (profiles/conv_cfg_sweep_r02.jsonl, ResNet-50 3x3 shapes, bs 256): the
// 2-stage rings win; BN 256 where it still gives >= half a wave of tiles, BN 64 for <= 128
// output channels (two workgroups per CU), BN 128 otherwise
inline int conv_fprop_bn(int cfg) { return cfg == 6 ? 256 : (cfg % 2 == 0 ? 128 : 64); }
inline int conv_fprop_cfg(const ConvTapArgs& a, int cus, int forced) {
  const int64_t tiles_m = ((int64_t)a.n * a.oh * a.ow + kConvBM - 1) / kConvBM;
  auto ok = [&](int bn) { return a.kout % bn == 0; };
  if (forced >= 0 && forced <= 6 && ok(conv_fprop_bn(forced))) return forced;
  if (a.kout <= 128) return 5;
  if (ok(256) && tiles_m * (a.kout / 256) >= cus / 2) return 6;
  return ok(128) ? 4 : 5;
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
