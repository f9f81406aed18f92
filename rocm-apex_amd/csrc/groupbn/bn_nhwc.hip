// Fused NHWC batch norm (+ residual add + ReLU) for gfx950: the engine behind
// apex.contrib.groupbn.BatchNorm2d_NHWC and the fused ResNet blocks.
//
// Reference: apex/contrib/csrc/groupbn/nhwc_batch_norm_kernel.h (persistent-CTA NHWC BN with
// an in-kernel grid sync and a bitmask for the fused ReLU), batch_norm.cu :44/:143/:226,
// batch_norm_add_relu.cu.
//
// MI355X design (no grid-wide sync, no persistent CTAs, deterministic):
//  forward   1. stats_partial : every lane owns 8 channels (one 16-byte load per row), keeps
//               4 rows in flight, accumulates sums of (x - shift), (x - shift)^2 with a common
//               per-channel shift (row 0); summed across the block's row-groups in LDS
//            2. stats_finalize: sums the partials in a fixed order, writes mean / inv_std, the
//               running-stat EMA and the epilogue constants scale/shift (one launch per layer)
//            3. apply         : y = relu(x*scale + shift + z) — one FMA per element, 16-byte I/O
//  backward  1. bwd_partial   : sum(dy'), sum(dy'*(x-mean)) with dy' = dy masked by the ReLU
//               output recomputed in registers (never stored unless the residual branch needs
//               it as grad_z, then written here in the same pass)
//            2. bwd_finalize  : grad_w, grad_b and dx = A*dy' + B*x + K constants
//            3. bwd_apply     : dx in one FMA pair per element
// Passes over the activation per layer: fwd 3 (x, x, y) [+z], bwd 5 (dy, x, dy, x, dx) — vs
// 5 / 8 for MIOpen BN + separate ReLU / threshold-backward kernels.  Residual add+ReLU layers
// also write the ReLU mask as 1 bit per element in the apply pass (1/16 of a bf16 pass); their
// backward reduction masks dy with those bits, so z is neither re-read nor kept alive.
#include "apex_amd/bn_nhwc_api.h"
#include "apex_amd/colsum.h"
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"

#include <cstdlib>
#include <type_traits>

namespace apex_amd {
namespace bnh {

constexpr int kU = 4;   // rows in flight per lane (backward: two tensors per row)
constexpr int kUS = 8;  // rows in flight per lane in the one-tensor statistics pass

struct Geo {
  int tx, ty, gx, gy;
};

// workgroups per CU of the partial passes: the read-only statistics pass keeps twice as many
// bytes in flight (4 per CU) as the two-tensor gradient pass (2 per CU), which otherwise reads at
// ~3 TB/s (profiles/resnet50_steady_r02b.md)
// (APEX_BN_STATS_BPC / APEX_BN_BWD_BPC override them for A/B sweeps, tools/bn_bench.py)
inline int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  const int v = e ? std::atoi(e) : 0;
  return v > 0 ? v : dflt;
}
static const int kStatsBlocksPerCu = env_int("APEX_BN_STATS_BPC", 4);
static const int kBwdBlocksPerCu = env_int("APEX_BN_BWD_BPC", 2);

inline Geo geo(int64_t m, int c, int cus, int blocks_per_cu = kBwdBlocksPerCu) {
  Geo g;
  const int cv = c / 8;
  g.tx = cv < 64 ? cv : 64;
  g.ty = 256 / g.tx;
  if (g.ty > 32) g.ty = 32;
  g.gx = (cv + g.tx - 1) / g.tx;
  const int64_t rows_per_iter = (int64_t)g.ty * kU;
  int64_t gy = ((int64_t)cus * blocks_per_cu + g.gx - 1) / g.gx;
  const int64_t cap = (m + rows_per_iter - 1) / rows_per_iter;
  if (gy > cap) gy = cap;
  if (gy > 1024) gy = 1024;
  g.gy = (int)(gy < 1 ? 1 : gy);
  return g;
}

__device__ __forceinline__ void load8f(float (&v)[8], const float* p) { Vec8<float>::load(v, p); }

// ------------------------------------------------------------------------------------------
// Statistics use a COMMON per-channel shift (the channel's value in row 0): every block
// accumulates plain sums S1 = sum(x - shift), S2 = sum((x - shift)^2), so the cross-block merge
// is a plain (fixed-order, deterministic) sum and mean/var follow from S1/n and S2/n - (S1/n)^2.
// A real sample of the channel as the shift keeps the cancellation in S2 benign.
template <typename T>
__global__ void __launch_bounds__(256) stats_partial(const T* __restrict__ x, int64_t m, int c,
                                                     float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int TX = blockDim.x, TY = blockDim.y, tx = threadIdx.x, ty = threadIdx.y;
  const int c0 = (blockIdx.x * TX + tx) * 8;
  const bool active = c0 < c;
  float sh[8], s[8], ss[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sh[k] = s[k] = ss[k] = 0.f;
  if (active) Vec8<T>::load(sh, x + c0);
  const int64_t R = (int64_t)TY * kUS;
  for (int64_t base = (int64_t)blockIdx.y * R; base < m; base += R * gridDim.y) {
    float v[kUS][8];
    bool ok[kUS];
#pragma unroll
    for (int u = 0; u < kUS; ++u) {
      const int64_t r = base + ty + (int64_t)u * TY;
      ok[u] = active && r < m;
      if (ok[u]) Vec8<T>::load(v[u], x + r * c + c0);
    }
#pragma unroll
    for (int u = 0; u < kUS; ++u) {
      if (!ok[u]) continue;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[u][k] - sh[k];
        s[k] += d;
        ss[k] = fmaf(d, d, ss[k]);
      }
    }
  }
  ColSum<8>::stash(smem, 0, s, tx, ty, TX, TY);
  ColSum<8>::stash(smem, 1, ss, tx, ty, TX, TY);
  __syncthreads();
  ColSum<8>::reduce_store(smem, 2, TX, TY, c, blockIdx.x * TX * 8, part, (int64_t)gridDim.y * c, blockIdx.y);
}

// Sum the gy partial rows of two [gy][C] slabs for kFinC channels per block: thread (ch, g) sums
// rows g, g + kFinG, ... (4 independent accumulators keep loads in flight), then a fixed-order
// LDS reduce over the kFinG row groups (deterministic).  8 channels x 32 row groups per block:
// the finalize is latency-bound (a few KB per block), so it spreads the rows over many lanes.
constexpr int kFinC = 8, kFinG = 256 / kFinC;

__device__ __forceinline__ void sum_partials(const float* __restrict__ part, int gy, int c, int ch, int g,
                                             float (&red)[2][kFinG][kFinC + 1], float& a, float& b) {
  float a4[4] = {0.f, 0.f, 0.f, 0.f}, b4[4] = {0.f, 0.f, 0.f, 0.f};
  if (ch < c) {
    int j = g;
    for (; j + 3 * kFinG < gy; j += 4 * kFinG) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a4[u] += part[(int64_t)(j + kFinG * u) * c + ch];
        b4[u] += part[(int64_t)(gy + j + kFinG * u) * c + ch];
      }
    }
    for (; j < gy; j += kFinG) {
      a4[0] += part[(int64_t)j * c + ch];
      b4[0] += part[(int64_t)(gy + j) * c + ch];
    }
  }
  const int lc = threadIdx.x % kFinC;
  red[0][g][lc] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
  red[1][g][lc] = (b4[0] + b4[1]) + (b4[2] + b4[3]);
  __syncthreads();
  a = 0.f;
  b = 0.f;
  if (g == 0) {
#pragma unroll 8
    for (int i = 0; i < kFinG; ++i) {
      a += red[0][i][lc];
      b += red[1][i][lc];
    }
  }
}

#define BN_FIN_INDEX                               \
  __shared__ float red[2][kFinG][kFinC + 1];       \
  const int g = threadIdx.x / kFinC;               \
  const int ch = blockIdx.x * kFinC + (threadIdx.x % kFinC)

template <typename T>
__global__ void __launch_bounds__(256) stats_finalize(const float* __restrict__ part, int gy, int c, float n,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      float eps, float momentum, float* __restrict__ rmean,
                                                      float* __restrict__ rvar, float* __restrict__ save_mean,
                                                      float* __restrict__ save_invstd, float* __restrict__ coef,
                                                      const T* __restrict__ x) {
  BN_FIN_INDEX;
  float s1, s2;
  sum_partials(part, gy, c, ch, g, red, s1, s2);
  if (g != 0 || ch >= c) return;
  const float shift = to_f(x[ch]);  // the stats kernel's shift: row 0
  const float dm = s1 / n;
  const float var_b = fmaxf(s2 / n - dm * dm, 0.f);
  const float mm = shift + dm;
  const float istd = rsqrtf(var_b + eps);
  save_mean[ch] = mm;
  save_invstd[ch] = istd;
  const float sc = istd * (w ? w[ch] : 1.f);
  coef[ch] = sc;
  coef[c + ch] = (b ? b[ch] : 0.f) - mm * sc;
  if (rmean) rmean[ch] = (1.f - momentum) * rmean[ch] + momentum * mm;
  if (rvar) rvar[ch] = (1.f - momentum) * rvar[ch] + momentum * (n > 1.f ? var_b * n / (n - 1.f) : var_b);
}

// ------------------------------------------------------------------------------------------
// Group (cross-rank) statistics, bn_group > 1.  Each rank reduces its own partials to a payload
// [mean(C) | M2(C) | count] (M2 = sum of squared deviations from the local mean), the payloads
// of the group are exchanged (xGMI peer memory or RCCL all-gather), and every rank merges the
// SAME gathered block in the same fixed order (Chan et al. pairwise update), so all members end
// with bit-identical mean / inv_std / running statistics.
template <typename T>
__global__ void __launch_bounds__(256) stats_local(const float* __restrict__ part, int gy, int c, float n,
                                                   const T* __restrict__ x, float* __restrict__ payload) {
  BN_FIN_INDEX;
  float s1, s2;
  sum_partials(part, gy, c, ch, g, red, s1, s2);
  if (g != 0 || ch >= c) return;
  const float shift = to_f(x[ch]);
  const float dm = s1 / n;
  payload[ch] = shift + dm;
  payload[c + ch] = fmaxf(s2 - s1 * dm, 0.f);
  if (ch == 0) payload[2 * c] = n;
}

__global__ void __launch_bounds__(256) stats_merge(const float* __restrict__ gathered, int world, int c,
                                                   const float* __restrict__ w, const float* __restrict__ b,
                                                   float eps, float momentum, float* __restrict__ rmean,
                                                   float* __restrict__ rvar, float* __restrict__ save_mean,
                                                   float* __restrict__ save_invstd, float* __restrict__ coef,
                                                   float* __restrict__ inv_count) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const int64_t row = 2 * (int64_t)c + 1;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int r = 0; r < world; ++r) {
    const float* p = gathered + r * row;
    const double nr = (double)p[2 * c];
    if (nr <= 0.0) continue;
    const double mr = (double)p[ch];
    const double nt = n + nr;
    const double d = mr - mean;
    mean += d * (nr / nt);
    m2 += (double)p[c + ch] + d * d * (n * nr / nt);
    n = nt;
  }
  const float var_b = (float)(n > 0.0 ? m2 / n : 0.0);
  const float mm = (float)mean;
  const float istd = rsqrtf(var_b + eps);
  save_mean[ch] = mm;
  save_invstd[ch] = istd;
  const float sc = istd * (w ? w[ch] : 1.f);
  coef[ch] = sc;
  coef[c + ch] = (b ? b[ch] : 0.f) - mm * sc;
  // a timed-out peer exchange hands back NaN payloads (csrc/comm/peer.hip): the step's outputs are
  // poisoned so the loss scaler skips it, but the running statistics must survive unchanged
  const bool finite = isfinite(mm) && isfinite(var_b);
  if (rmean && finite) rmean[ch] = (1.f - momentum) * rmean[ch] + momentum * mm;
  if (rvar && finite) rvar[ch] = (1.f - momentum) * rvar[ch] + momentum * (float)(n > 1.0 ? m2 / (n - 1.0) : var_b);
  if (ch == 0) inv_count[0] = (float)(n > 0.0 ? 1.0 / n : 0.0);
}

__global__ void coef_from_stats(const float* __restrict__ mean, const float* __restrict__ v, int is_var,
                                const float* __restrict__ w, const float* __restrict__ b, float eps, int c,
                                float* __restrict__ coef) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const float istd = is_var ? rsqrtf(v[ch] + eps) : v[ch];
  const float sc = istd * (w ? w[ch] : 1.f);
  coef[ch] = sc;
  coef[c + ch] = (b ? b[ch] : 0.f) - mean[ch] * sc;
}

// ------------------------------------------------------------------------------------------
// MASKOUT: also write the ReLU mask as one bit per element (bit k of byte i = element 8i+k), so
// the backward of a residual add+ReLU needs neither z nor a recompute (1/16 of a bf16 tensor)
template <typename T, bool HAS_Z, bool RELU, bool MASKOUT>
__device__ __forceinline__ void apply_vec(const T* __restrict__ x, const T* __restrict__ z, T* __restrict__ y,
                                          uint8_t* __restrict__ mask, int64_t i, float (&v)[8], const float (&zz)[8],
                                          const float (&sc)[8], const float (&sh)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float o = fmaf(v[k], sc[k], sh[k]);
    if constexpr (HAS_Z) o += zz[k];
    if constexpr (RELU) o = fmaxf(o, 0.f);
    v[k] = o;
  }
  Vec8<T>::store(y + i * 8, v);
  if constexpr (MASKOUT) {
    unsigned b = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) b |= (v[k] > 0.f ? 1u : 0u) << k;
    mask[i] = (uint8_t)b;
  }
}

// Elementwise passes: when the grid stride is a multiple of C (every power-of-two C up to the
// stride: all ResNet widths), a lane keeps ONE 8-channel group for the whole pass, so its
// per-channel coefficients are loaded once into registers instead of once per vector (they were
// 2-5 extra 32-byte loads per 16-byte data load), and kEwU vectors are in flight per lane.
constexpr int kEwU = 4;

template <typename T, bool HAS_Z, bool RELU, bool MASKOUT>
__global__ void __launch_bounds__(256) apply_kernel(const T* __restrict__ x, const T* __restrict__ z,
                                                    const float* __restrict__ coef, T* __restrict__ y, int64_t nvec,
                                                    int c, uint8_t* __restrict__ mask) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int cstep = (int)((stride * 8) % c);
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (cstep == 0) {
    const int c0 = (int)((i * 8) % c);
    float sc[8], sh[8];
    load8f(sc, coef + c0);
    load8f(sh, coef + c + c0);
    for (; i + (kEwU - 1) * stride < nvec; i += kEwU * stride) {
      float v[kEwU][8], zz[kEwU][8];
#pragma unroll
      for (int u = 0; u < kEwU; ++u) {
        Vec8<T>::load(v[u], x + (i + u * stride) * 8);
        if constexpr (HAS_Z) Vec8<T>::load(zz[u], z + (i + u * stride) * 8);
      }
#pragma unroll
      for (int u = 0; u < kEwU; ++u) apply_vec<T, HAS_Z, RELU, MASKOUT>(x, z, y, mask, i + u * stride, v[u], zz[u], sc, sh);
    }
    for (; i < nvec; i += stride) {
      float v[8], zz[8];
      Vec8<T>::load(v, x + i * 8);
      if constexpr (HAS_Z) Vec8<T>::load(zz, z + i * 8);
      apply_vec<T, HAS_Z, RELU, MASKOUT>(x, z, y, mask, i, v, zz, sc, sh);
    }
    return;
  }
  // general C: the channel offset advances by a fixed step per grid stride (no 64-bit modulo)
  for (int c0 = (int)((i * 8) % c); i < nvec; i += stride, c0 = c0 + cstep >= c ? c0 + cstep - c : c0 + cstep) {
    float v[8], sc[8], sh[8], zz[8];
    Vec8<T>::load(v, x + i * 8);
    load8f(sc, coef + c0);
    load8f(sh, coef + c + c0);
    if constexpr (HAS_Z) Vec8<T>::load(zz, z + i * 8);
    apply_vec<T, HAS_Z, RELU, MASKOUT>(x, z, y, mask, i, v, zz, sc, sh);
  }
}

// ------------------------------------------------------------------------------------------
// Two batch norms summed under one ReLU (a downsampling residual block's output:
// y = relu(bn_main(x) + bn_short(z))): both normalizations in the single output pass, so the
// shortcut branch's normalized tensor is never written or re-read.
template <typename T, bool MASKOUT>
__device__ __forceinline__ void apply_dual_vec(T* __restrict__ y, uint8_t* __restrict__ mask, int64_t i,
                                               float (&v)[8], const float (&w)[8], const float (&sx)[8],
                                               const float (&hx)[8], const float (&sz)[8], const float (&hz)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = fmaxf(fmaf(v[k], sx[k], hx[k]) + fmaf(w[k], sz[k], hz[k]), 0.f);
  Vec8<T>::store(y + i * 8, v);
  if constexpr (MASKOUT) {
    unsigned b = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) b |= (v[k] > 0.f ? 1u : 0u) << k;
    mask[i] = (uint8_t)b;
  }
}

template <typename T, bool MASKOUT>
__global__ void __launch_bounds__(256) apply_dual_kernel(const T* __restrict__ x, const T* __restrict__ z,
                                                         const float* __restrict__ cx, const float* __restrict__ cz,
                                                         T* __restrict__ y, int64_t nvec, int c,
                                                         uint8_t* __restrict__ mask) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int cstep = (int)((stride * 8) % c);
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (cstep == 0) {  // fixed channel group per lane (see apply_kernel)
    const int c0 = (int)((i * 8) % c);
    float sx[8], hx[8], sz[8], hz[8];
    load8f(sx, cx + c0);
    load8f(hx, cx + c + c0);
    load8f(sz, cz + c0);
    load8f(hz, cz + c + c0);
    for (; i + (kEwU - 1) * stride < nvec; i += kEwU * stride) {
      float v[kEwU][8], w[kEwU][8];
#pragma unroll
      for (int u = 0; u < kEwU; ++u) {
        Vec8<T>::load(v[u], x + (i + u * stride) * 8);
        Vec8<T>::load(w[u], z + (i + u * stride) * 8);
      }
#pragma unroll
      for (int u = 0; u < kEwU; ++u) apply_dual_vec<T, MASKOUT>(y, mask, i + u * stride, v[u], w[u], sx, hx, sz, hz);
    }
    for (; i < nvec; i += stride) {
      float v[8], w[8];
      Vec8<T>::load(v, x + i * 8);
      Vec8<T>::load(w, z + i * 8);
      apply_dual_vec<T, MASKOUT>(y, mask, i, v, w, sx, hx, sz, hz);
    }
    return;
  }
  for (int c0 = (int)((i * 8) % c); i < nvec; i += stride, c0 = c0 + cstep >= c ? c0 + cstep - c : c0 + cstep) {
    float v[8], w[8], sx[8], hx[8], sz[8], hz[8];
    Vec8<T>::load(v, x + i * 8);
    Vec8<T>::load(w, z + i * 8);
    load8f(sx, cx + c0);
    load8f(hx, cx + c + c0);
    load8f(sz, cz + c0);
    load8f(hz, cz + c + c0);
    apply_dual_vec<T, MASKOUT>(y, mask, i, v, w, sx, hx, sz, hz);
  }
}

// ------------------------------------------------------------------------------------------
// BN apply + ReLU + max pool in one pass (the ResNet stem: conv -> BN -> ReLU -> 3x3/2 max pool):
// every window element is normalized in registers as it is loaded, so the full-resolution
// normalized tensor is never written nor re-read by the pool.  One lane per (n, oh, ow, 8
// channels); 16-byte loads; 1-byte window indices as in the standalone NHWC pool
// (csrc/pool/maxpool_nhwc.hip), so the pool backward and the BN backward are unchanged.
struct PoolGeo {
  int n, h, w, c, oh, ow, kh, kw, sh, sw, ph, pw;
};

template <typename T>
__global__ void __launch_bounds__(256) apply_relu_maxpool_kernel(const T* __restrict__ x,
                                                                 const float* __restrict__ coef, PoolGeo g,
                                                                 T* __restrict__ y, uint8_t* __restrict__ idx) {
  const uint32_t cv = (uint32_t)(g.c / 8);
  const uint32_t total = (uint32_t)g.n * g.oh * g.ow * cv;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const int c8 = (int)(i % cv) * 8;
    uint32_t r = i / cv;
    const int ow = (int)(r % (uint32_t)g.ow);
    r /= (uint32_t)g.ow;
    const int oh = (int)(r % (uint32_t)g.oh);
    const int n = (int)(r / (uint32_t)g.oh);
    float sc[8], sh[8], best[8];
    uint8_t bi[8];
    load8f(sc, coef + c8);
    load8f(sh, coef + g.c + c8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      bi[e] = 0;
    }
    const int h0 = oh * g.sh - g.ph, w0 = ow * g.sw - g.pw;
    for (int a = 0; a < g.kh; ++a) {
      const int ih = h0 + a;
      if (ih < 0 || ih >= g.h) continue;
      for (int b = 0; b < g.kw; ++b) {
        const int iw = w0 + b;
        if (iw < 0 || iw >= g.w) continue;
        float v[8];
        Vec8<T>::load(v, x + (((int64_t)n * g.h + ih) * g.w + iw) * g.c + c8);
        const uint8_t k = (uint8_t)(a * g.kw + b);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // normalized + ReLU value, rounded to the storage type exactly as the unfused apply
          // pass would store it, so argmax ties resolve identically
          const float o = to_f(from_f<T>(fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f)));
          if (o > best[e] || (o != o && best[e] == best[e])) {
            best[e] = o;
            bi[e] = k;
          }
        }
      }
    }
    const int64_t o = (((int64_t)n * g.oh + oh) * g.ow + ow) * g.c + c8;
    Vec8<T>::store(y + o, best);
    uint2 w;
    w.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    w.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = w;
  }
}

// ------------------------------------------------------------------------------------------
// DY2: the output fed two consumers (a residual block's main and shortcut branches) and its
// gradient arrives as two tensors, summed here in registers instead of by a separate add pass
// BITS: the ReLU mask comes from the forward's bit mask instead of a recompute from x (and z)
template <typename T, bool HAS_Z, bool RELU, bool WRITE_MASKED, bool DY2, bool BITS>
__global__ void __launch_bounds__(256) bwd_partial(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                   const T* __restrict__ x,
                                                   const T* __restrict__ z, const float* __restrict__ coef,
                                                   const float* __restrict__ mean, T* __restrict__ dym, int64_t m,
                                                   int c, float* __restrict__ part,
                                                   const uint8_t* __restrict__ bits) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int TX = blockDim.x, TY = blockDim.y, tx = threadIdx.x, ty = threadIdx.y;
  const int c0 = (blockIdx.x * TX + tx) * 8;
  const bool active = c0 < c;
  float a1[8], a2[8], mu[8], sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a1[k] = a2[k] = 0.f;
  if (active) {
    load8f(mu, mean + c0);
    if constexpr (RELU && !BITS) {
      load8f(sc, coef + c0);
      load8f(sh, coef + c + c0);
    }
  }
  const int64_t R = (int64_t)TY * kU;
  for (int64_t base = (int64_t)blockIdx.y * R; base < m; base += R * gridDim.y) {
    float g[kU][8], v[kU][8];
    unsigned mb[kU];
    bool ok[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t r = base + ty + (int64_t)u * TY;
      ok[u] = active && r < m;
      if (ok[u]) {
        Vec8<T>::load(g[u], dy + r * c + c0);
        Vec8<T>::load(v[u], x + r * c + c0);
        if constexpr (BITS) mb[u] = bits[(r * c + c0) >> 3];
        if constexpr (DY2) {
          float h[8];
          Vec8<T>::load(h, dy2 + r * c + c0);
#pragma unroll
          for (int k = 0; k < 8; ++k) g[u][k] += h[k];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (!ok[u]) continue;
      const int64_t e = (base + ty + (int64_t)u * TY) * c + c0;
      if constexpr (RELU && BITS) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (!((mb[u] >> k) & 1u)) g[u][k] = 0.f;
        if constexpr (WRITE_MASKED) Vec8<T>::store(dym + e, g[u]);
      } else if constexpr (RELU) {
        float zz[8];
        if constexpr (HAS_Z) Vec8<T>::load(zz, z + e);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float o = fmaf(v[u][k], sc[k], sh[k]);
          if constexpr (HAS_Z) o += zz[k];
          if (!(o > 0.f)) g[u][k] = 0.f;
        }
        if constexpr (WRITE_MASKED) Vec8<T>::store(dym + e, g[u]);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a1[k] += g[u][k];
        a2[k] = fmaf(g[u][k], v[u][k] - mu[k], a2[k]);
      }
    }
  }
  ColSum<8>::stash(smem, 0, a1, tx, ty, TX, TY);
  ColSum<8>::stash(smem, 1, a2, tx, ty, TX, TY);
  __syncthreads();
  ColSum<8>::reduce_store(smem, 2, TX, TY, c, blockIdx.x * TX * 8, part, (int64_t)gridDim.y * c, blockIdx.y);
}

__global__ void __launch_bounds__(256) bwd_finalize(const float* __restrict__ part, int gy, int c, float inv_n,
                                                    const float* __restrict__ mean, const float* __restrict__ istd,
                                                    const float* __restrict__ w, float* __restrict__ gw,
                                                    float* __restrict__ gb, float* __restrict__ coef) {
  BN_FIN_INDEX;
  float sdy, sdyx;
  sum_partials(part, gy, c, ch, g, red, sdy, sdyx);
  if (g != 0 || ch >= c) return;
  const float is = istd[ch];
  if (gw) gw[ch] = sdyx * is;
  if (gb) gb[ch] = sdy;
  const float A = is * (w ? w[ch] : 1.f);
  const float B = -A * is * is * (sdyx * inv_n);
  coef[ch] = A;
  coef[c + ch] = B;
  coef[2 * c + ch] = -A * (sdy * inv_n) - B * mean[ch];
}

// group backward, step 1: this rank's sums as the exchange payload [sum_dy(C) | sum_dy_xmu(C)]
// plus the LOCAL weight / bias gradients (data-parallel averages those like any other grad)
__global__ void __launch_bounds__(256) bwd_local(const float* __restrict__ part, int gy, int c,
                                                 const float* __restrict__ istd, float* __restrict__ gw,
                                                 float* __restrict__ gb, float* __restrict__ payload) {
  BN_FIN_INDEX;
  float sdy, sdyx;
  sum_partials(part, gy, c, ch, g, red, sdy, sdyx);
  if (g != 0 || ch >= c) return;
  if (gw) gw[ch] = sdyx * istd[ch];
  if (gb) gb[ch] = sdy;
  payload[ch] = sdy;
  payload[c + ch] = sdyx;
}

// group backward, step 2: dx coefficients from the group's sums; `rows` payload rows (one per
// rank after a peer all-gather, summed here in rank order; 1 after an RCCL all-reduce)
__global__ void __launch_bounds__(256) bwd_coef_group(const float* __restrict__ sums, int rows, int c,
                                                      const float* __restrict__ inv_count,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ istd, const float* __restrict__ w,
                                                      float* __restrict__ coef) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  float sdy = 0.f, sdyx = 0.f;
  for (int r = 0; r < rows; ++r) {
    sdy += sums[(int64_t)r * 2 * c + ch];
    sdyx += sums[(int64_t)r * 2 * c + c + ch];
  }
  const float inv_n = inv_count[0];
  const float is = istd[ch];
  const float A = is * (w ? w[ch] : 1.f);
  const float B = -A * is * is * (sdyx * inv_n);
  coef[ch] = A;
  coef[c + ch] = B;
  coef[2 * c + ch] = -A * (sdy * inv_n) - B * mean[ch];
}

template <typename T, bool HAS_Z, bool MASK>
__device__ __forceinline__ void bwd_apply_vec(T* __restrict__ dx, int64_t i, float (&g)[8], float (&v)[8],
                                              const float (&zz)[8], const float (&A)[8], const float (&B)[8],
                                              const float (&K)[8], const float (&sc)[8], const float (&sh)[8]) {
  if constexpr (MASK) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float o = fmaf(v[k], sc[k], sh[k]);
      if constexpr (HAS_Z) o += zz[k];
      if (!(o > 0.f)) g[k] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = fmaf(A[k], g[k], fmaf(B[k], v[k], K[k]));
  Vec8<T>::store(dx + i * 8, v);
}

template <typename T, bool HAS_Z, bool MASK>
__global__ void __launch_bounds__(256) bwd_apply(const T* __restrict__ dy, const T* __restrict__ x,
                                                 const T* __restrict__ z, const float* __restrict__ cf,
                                                 const float* __restrict__ cb, T* __restrict__ dx, int64_t nvec,
                                                 int c) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int cstep = (int)((stride * 8) % c);
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float sc[8], sh[8], zz[8];
  if (cstep == 0) {  // fixed channel group per lane (see apply_kernel)
    const int c0 = (int)((i * 8) % c);
    float A[8], B[8], K[8];
    load8f(A, cb + c0);
    load8f(B, cb + c + c0);
    load8f(K, cb + 2 * c + c0);
    if constexpr (MASK) {
      load8f(sc, cf + c0);
      load8f(sh, cf + c + c0);
    }
    for (; i + (kEwU - 1) * stride < nvec; i += kEwU * stride) {
      float g[kEwU][8], v[kEwU][8], zu[kEwU][8];
#pragma unroll
      for (int u = 0; u < kEwU; ++u) {
        Vec8<T>::load(g[u], dy + (i + u * stride) * 8);
        Vec8<T>::load(v[u], x + (i + u * stride) * 8);
        if constexpr (MASK && HAS_Z) Vec8<T>::load(zu[u], z + (i + u * stride) * 8);
      }
#pragma unroll
      for (int u = 0; u < kEwU; ++u)
        bwd_apply_vec<T, HAS_Z, MASK>(dx, i + u * stride, g[u], v[u], zu[u], A, B, K, sc, sh);
    }
    for (; i < nvec; i += stride) {
      float g[8], v[8];
      Vec8<T>::load(g, dy + i * 8);
      Vec8<T>::load(v, x + i * 8);
      if constexpr (MASK && HAS_Z) Vec8<T>::load(zz, z + i * 8);
      bwd_apply_vec<T, HAS_Z, MASK>(dx, i, g, v, zz, A, B, K, sc, sh);
    }
    return;
  }
  for (int c0 = (int)((i * 8) % c); i < nvec; i += stride, c0 = c0 + cstep >= c ? c0 + cstep - c : c0 + cstep) {
    float g[8], v[8], A[8], B[8], K[8];
    Vec8<T>::load(g, dy + i * 8);
    Vec8<T>::load(v, x + i * 8);
    load8f(A, cb + c0);
    load8f(B, cb + c + c0);
    load8f(K, cb + 2 * c + c0);
    if constexpr (MASK) {
      load8f(sc, cf + c0);
      load8f(sh, cf + c + c0);
      if constexpr (HAS_Z) Vec8<T>::load(zz, z + i * 8);
    }
    bwd_apply_vec<T, HAS_Z, MASK>(dx, i, g, v, zz, A, B, K, sc, sh);
  }
}

inline unsigned ew_grid(int64_t nvec, int cus) {
  int64_t g = (nvec + 255) / 256;
  const int64_t cap = (int64_t)cus * 8;
  if (g > cap) g = cap;
  return (unsigned)(g < 1 ? 1 : g);
}

inline void check_shape(int64_t m, int c) {
  if (c % 8 != 0 || c <= 0 || m <= 0) throw std::runtime_error("bn_nhwc: C must be a positive multiple of 8");
}

}  // namespace bnh

int bn_nhwc_plan(int64_t m, int c, int cus, int64_t* ws_floats) {
  const bnh::Geo g = bnh::geo(m, c, cus);
  const bnh::Geo gs = bnh::geo(m, c, cus, bnh::kStatsBlocksPerCu);
  if (ws_floats) *ws_floats = 2 * (int64_t)(g.gy > gs.gy ? g.gy : gs.gy) * c;
  return g.gy;
}

void bn_nhwc_stats(const void* x, int x_t, int64_t m, int c, const float* w, const float* b, float eps, float momentum,
                   float* running_mean, float* running_var, float* save_mean, float* save_invstd, float* coef_fwd,
                   float* ws, int gy, int cus, hipStream_t s) {
  bnh::check_shape(m, c);
  (void)gy;  // the statistics pass has its own (deeper) geometry; ws is sized for it by bn_nhwc_plan
  const bnh::Geo g = bnh::geo(m, c, cus, bnh::kStatsBlocksPerCu);
  const size_t lds = ColSum<8>::lds_floats(g.tx, g.ty, 2) * sizeof(float);
  dispatch_float(x_t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    hipLaunchKernelGGL((bnh::stats_partial<T>), dim3(g.gx, g.gy), dim3(g.tx, g.ty), lds, s, (const T*)x, m, c, ws);
    hipLaunchKernelGGL((bnh::stats_finalize<T>), dim3((c + bnh::kFinC - 1) / bnh::kFinC), dim3(256), 0, s, ws, g.gy, c, (float)m, w, b,
                       eps, momentum, running_mean, running_var, save_mean, save_invstd, coef_fwd, (const T*)x);
  }, "bn_nhwc stats");
  check_launch("bn_nhwc_stats");
}

void bn_nhwc_stats_local(const void* x, int x_t, int64_t m, int c, float* payload, float* ws, int gy, int cus,
                         hipStream_t s) {
  bnh::check_shape(m, c);
  (void)gy;
  const bnh::Geo g = bnh::geo(m, c, cus, bnh::kStatsBlocksPerCu);
  const size_t lds = ColSum<8>::lds_floats(g.tx, g.ty, 2) * sizeof(float);
  dispatch_float(x_t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    hipLaunchKernelGGL((bnh::stats_partial<T>), dim3(g.gx, g.gy), dim3(g.tx, g.ty), lds, s, (const T*)x, m, c, ws);
    hipLaunchKernelGGL((bnh::stats_local<T>), dim3((c + bnh::kFinC - 1) / bnh::kFinC), dim3(256), 0, s, ws, g.gy, c, (float)m, (const T*)x,
                       payload);
  }, "bn_nhwc stats local");
  check_launch("bn_nhwc_stats_local");
}

void bn_nhwc_stats_merge(const float* gathered, int world, int c, const float* w, const float* b, float eps,
                         float momentum, float* running_mean, float* running_var, float* save_mean, float* save_invstd,
                         float* coef_fwd, float* inv_count, hipStream_t s) {
  if (world < 1 || c <= 0) throw std::runtime_error("bn_nhwc stats merge: bad group / channels");
  hipLaunchKernelGGL(bnh::stats_merge, dim3((c + 255) / 256), dim3(256), 0, s, gathered, world, c, w, b, eps, momentum,
                     running_mean, running_var, save_mean, save_invstd, coef_fwd, inv_count);
  check_launch("bn_nhwc_stats_merge");
}

void bn_nhwc_bwd_coef_group(const float* sums, int rows, int c, const float* inv_count, const float* save_mean,
                            const float* save_invstd, const float* w, float* coef_bwd, hipStream_t s) {
  if (rows < 1 || c <= 0) throw std::runtime_error("bn_nhwc bwd coef: bad rows / channels");
  hipLaunchKernelGGL(bnh::bwd_coef_group, dim3((c + 255) / 256), dim3(256), 0, s, sums, rows, c, inv_count, save_mean,
                     save_invstd, w, coef_bwd);
  check_launch("bn_nhwc_bwd_coef_group");
}

void bn_nhwc_bwd_local(const float* part, int gy, int c, const float* save_invstd, float* grad_w, float* grad_b,
                       float* payload, hipStream_t s) {
  if (gy < 1 || c <= 0) throw std::runtime_error("bn_nhwc bwd local: bad partial rows / channels");
  hipLaunchKernelGGL(bnh::bwd_local, dim3((c + bnh::kFinC - 1) / bnh::kFinC), dim3(256), 0, s, part, gy, c, save_invstd,
                     grad_w, grad_b, payload);
  check_launch("bn_nhwc_bwd_local");
}

void bn_nhwc_coef_from_stats(const float* mean, const float* v, bool is_var, const float* w, const float* b, float eps,
                             int c, float* coef_fwd, hipStream_t s) {
  hipLaunchKernelGGL(bnh::coef_from_stats, dim3((c + 255) / 256), dim3(256), 0, s, mean, v, is_var ? 1 : 0, w, b, eps,
                     c, coef_fwd);
  check_launch("bn_nhwc_coef_from_stats");
}

void bn_nhwc_apply(const void* x, int x_t, const void* z, const float* coef_fwd, bool relu, void* y, int64_t m, int c,
                   int cus, hipStream_t s, uint8_t* mask_out) {
  if (mask_out && !relu) throw std::runtime_error("bn_nhwc apply: a ReLU bit mask needs the fused ReLU");
  bnh::check_shape(m, c);
  const int64_t nvec = m * c / 8;
  const unsigned grid = bnh::ew_grid(nvec, cus);
  dispatch_float(x_t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    auto go = [&](auto hz, auto rl) {
      hipLaunchKernelGGL((bnh::apply_kernel<T, decltype(hz)::value, decltype(rl)::value, false>), dim3(grid), dim3(256),
                         0, s, (const T*)x, (const T*)z, coef_fwd, (T*)y, nvec, c, nullptr);
    };
    if (mask_out) {
      if (z)
        hipLaunchKernelGGL((bnh::apply_kernel<T, true, true, true>), dim3(grid), dim3(256), 0, s, (const T*)x,
                           (const T*)z, coef_fwd, (T*)y, nvec, c, mask_out);
      else
        hipLaunchKernelGGL((bnh::apply_kernel<T, false, true, true>), dim3(grid), dim3(256), 0, s, (const T*)x,
                           (const T*)z, coef_fwd, (T*)y, nvec, c, mask_out);
    } else if (z) {
      if (relu) go(std::true_type{}, std::true_type{});
      else go(std::true_type{}, std::false_type{});
    } else {
      if (relu) go(std::false_type{}, std::true_type{});
      else go(std::false_type{}, std::false_type{});
    }
  }, "bn_nhwc apply");
  check_launch("bn_nhwc_apply");
}

void bn_nhwc_apply_relu_maxpool(const void* x, int x_t, const float* coef_fwd, int n, int h, int w, int c, int kh,
                                int kw, int sh, int sw, int ph, int pw, int oh, int ow, void* y, uint8_t* idx, int cus,
                                hipStream_t s) {
  if (c % 8 || c <= 0) throw std::runtime_error("bn_nhwc apply+pool: C must be a positive multiple of 8");
  if (kh * kw > 255 || kh <= 0 || kw <= 0) throw std::runtime_error("bn_nhwc apply+pool: bad window");
  const int64_t total = (int64_t)n * oh * ow * (c / 8);
  int64_t grid = (total + 255) / 256;
  if (grid > (int64_t)cus * 16) grid = (int64_t)cus * 16;
  if (grid < 1) grid = 1;
  if (total + grid * 256 >= (int64_t)UINT32_MAX) throw std::runtime_error("bn_nhwc apply+pool: tensor too large");
  const bnh::PoolGeo g{n, h, w, c, oh, ow, kh, kw, sh, sw, ph, pw};
  dispatch_float(x_t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    hipLaunchKernelGGL((bnh::apply_relu_maxpool_kernel<T>), dim3((unsigned)grid), dim3(256), 0, s, (const T*)x,
                       coef_fwd, g, (T*)y, idx);
  }, "bn_nhwc apply+pool");
  check_launch("bn_nhwc_apply_relu_maxpool");
}

void bn_nhwc_apply_dual(const void* x, const void* z, int x_t, const float* coef_x, const float* coef_z, void* y,
                        int64_t m, int c, int cus, hipStream_t s, uint8_t* mask_out) {
  bnh::check_shape(m, c);
  const int64_t nvec = m * c / 8;
  const unsigned grid = bnh::ew_grid(nvec, cus);
  dispatch_float(x_t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (mask_out)
      hipLaunchKernelGGL((bnh::apply_dual_kernel<T, true>), dim3(grid), dim3(256), 0, s, (const T*)x, (const T*)z,
                         coef_x, coef_z, (T*)y, nvec, c, mask_out);
    else
      hipLaunchKernelGGL((bnh::apply_dual_kernel<T, false>), dim3(grid), dim3(256), 0, s, (const T*)x, (const T*)z,
                         coef_x, coef_z, (T*)y, nvec, c, nullptr);
  }, "bn_nhwc apply dual");
  check_launch("bn_nhwc_apply_dual");
}

void bn_nhwc_bwd_reduce(const void* dy, const void* x, int x_t, const void* z, const float* coef_fwd, bool relu,
                        const float* save_mean, const float* save_invstd, const float* w, float* grad_w, float* grad_b,
                        float* coef_bwd, void* dy_masked_out, int64_t m, int c, float* ws, int gy, int cus,
                        hipStream_t s, const void* dy2, const uint8_t* mask_in, float* group_payload) {
  if (mask_in && !(relu && dy_masked_out))
    throw std::runtime_error("bn_nhwc bwd: the ReLU bit mask path writes the masked gradient");
  if (dy2 && !(relu && dy_masked_out))
    throw std::runtime_error("bn_nhwc bwd: a second gradient needs the fused-ReLU masked-gradient path");
  bnh::check_shape(m, c);
  bnh::Geo g = bnh::geo(m, c, cus);
  g.gy = gy;
  const size_t lds = ColSum<8>::lds_floats(g.tx, g.ty, 2) * sizeof(float);
  dispatch_float(x_t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    auto go = [&](auto hz, auto rl, auto wm, auto d2) {
      hipLaunchKernelGGL((bnh::bwd_partial<T, decltype(hz)::value, decltype(rl)::value, decltype(wm)::value,
                                           decltype(d2)::value, false>),
                         dim3(g.gx, g.gy), dim3(g.tx, g.ty), lds, s, (const T*)dy, (const T*)dy2, (const T*)x,
                         (const T*)z, coef_fwd, save_mean, (T*)dy_masked_out, m, c, ws, nullptr);
    };
    auto go_bits = [&](auto d2) {
      hipLaunchKernelGGL((bnh::bwd_partial<T, false, true, true, decltype(d2)::value, true>), dim3(g.gx, g.gy),
                         dim3(g.tx, g.ty), lds, s, (const T*)dy, (const T*)dy2, (const T*)x, nullptr, coef_fwd,
                         save_mean, (T*)dy_masked_out, m, c, ws, mask_in);
    };
    using F = std::false_type;
    using Tr = std::true_type;
    if (mask_in) {
      if (dy2) go_bits(Tr{});
      else go_bits(F{});
    } else if (!relu) go(F{}, F{}, F{}, F{});
    else if (z && dy_masked_out) {
      if (dy2) go(Tr{}, Tr{}, Tr{}, Tr{});
      else go(Tr{}, Tr{}, Tr{}, F{});
    } else if (z) go(Tr{}, Tr{}, F{}, F{});
    else if (dy_masked_out) {
      if (dy2) go(F{}, Tr{}, Tr{}, Tr{});
      else go(F{}, Tr{}, Tr{}, F{});
    } else go(F{}, Tr{}, F{}, F{});
  }, "bn_nhwc bwd reduce");
  if (group_payload)  // bn_group > 1: local sums for the exchange, coefficients after it
    hipLaunchKernelGGL(bnh::bwd_local, dim3((c + bnh::kFinC - 1) / bnh::kFinC), dim3(256), 0, s, ws, g.gy, c, save_invstd, grad_w, grad_b,
                       group_payload);
  else
    hipLaunchKernelGGL(bnh::bwd_finalize, dim3((c + bnh::kFinC - 1) / bnh::kFinC), dim3(256), 0, s, ws, g.gy, c, 1.f / (float)m, save_mean,
                       save_invstd, w, grad_w, grad_b, coef_bwd);
  check_launch("bn_nhwc_bwd_reduce");
}

void bn_nhwc_bwd_apply(const void* dy, bool dy_is_masked, const void* x, int x_t, const void* z, const float* coef_fwd,
                       bool relu, const float* coef_bwd, void* dx, int64_t m, int c, int cus, hipStream_t s) {
  bnh::check_shape(m, c);
  const int64_t nvec = m * c / 8;
  const unsigned grid = bnh::ew_grid(nvec, cus);
  const bool mask = relu && !dy_is_masked;
  dispatch_float(x_t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    auto go = [&](auto hz, auto mk) {
      hipLaunchKernelGGL((bnh::bwd_apply<T, decltype(hz)::value, decltype(mk)::value>), dim3(grid), dim3(256), 0, s,
                         (const T*)dy, (const T*)x, (const T*)z, coef_fwd, coef_bwd, (T*)dx, nvec, c);
    };
    if (!mask) go(std::false_type{}, std::false_type{});
    else if (z) go(std::true_type{}, std::true_type{});
    else go(std::false_type{}, std::true_type{});
  }, "bn_nhwc bwd apply");
  check_launch("bn_nhwc_bwd_apply");
}

}  // namespace apex_amd
