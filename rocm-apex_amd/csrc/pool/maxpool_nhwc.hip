// Channels-last max pooling for gfx950 (the ResNet stem's 3x3/2 pool runs on a [N, 112, 112, 64]
// activation: PyTorch's NHWC kernels spent 0.85 ms/step there in our ResNet-50 profile,
// profiles/resnet50_o2_fusedbn_steady_r01.md, largely because they save int64 indices).
//  * forward: one lane per (n, oh, ow, 8 channels): 16-byte loads of the window rows, max with
//    NaN propagation, 16-byte output store + 8 one-byte window indices (1/8 of int64 traffic);
//  * backward as a GATHER: one lane per (n, ih, iw, 8 channels) visits the <= ceil(K/S)^2
//    windows that contain the pixel and sums the gradients whose index points at it — every dx
//    element written exactly once, no atomics and no zero-fill pass.
// Index decomposition runs in 32-bit unsigned math whenever the lane count allows (IDX =
// uint32_t): 64-bit div/mod expands to a long VALU sequence and was the pool kernels' bottleneck.
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/pool_api.h"

namespace apex_amd {
namespace pool {

template <typename T, typename IDX>
__global__ void __launch_bounds__(256) fwd_kernel(const PoolArgs a, const T* __restrict__ x, T* __restrict__ y,
                                                  uint8_t* __restrict__ idx) {
  const IDX cv = (IDX)(a.C / 8);
  const IDX total = (IDX)a.N * a.OH * a.OW * cv;
  for (IDX i = blockIdx.x * (IDX)blockDim.x + threadIdx.x; i < total; i += (IDX)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cv) * 8;
    IDX r = i / cv;
    const int ow = (int)(r % (IDX)a.OW);
    r /= (IDX)a.OW;
    const int oh = (int)(r % (IDX)a.OH);
    const int n = (int)(r / (IDX)a.OH);
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      bi[e] = 0;
    }
    const int h0 = oh * a.SH - a.PH, w0 = ow * a.SW - a.PW;
    for (int kh = 0; kh < a.KH; ++kh) {
      const int ih = h0 + kh;
      if (ih < 0 || ih >= a.H) continue;
      for (int kw = 0; kw < a.KW; ++kw) {
        const int iw = w0 + kw;
        if (iw < 0 || iw >= a.W) continue;
        float v[8];
        Vec8<T>::load(v, x + (((int64_t)n * a.H + ih) * a.W + iw) * a.C + c8);
        const uint8_t k = (uint8_t)(kh * a.KW + kw);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (v[e] > best[e] || (v[e] != v[e] && best[e] == best[e])) {
            best[e] = v[e];
            bi[e] = k;
          }
        }
      }
    }
    const int64_t o = (((int64_t)n * a.OH + oh) * a.OW + ow) * a.C + c8;
    Vec8<T>::store(y + o, best);
    uint2 w;
    w.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    w.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = w;
  }
}

template <typename T, typename IDX>
__global__ void __launch_bounds__(256) bwd_kernel(const PoolArgs a, const T* __restrict__ dy,
                                                  const uint8_t* __restrict__ idx, T* __restrict__ dx) {
  const IDX cv = (IDX)(a.C / 8);
  const IDX total = (IDX)a.N * a.H * a.W * cv;
  for (IDX i = blockIdx.x * (IDX)blockDim.x + threadIdx.x; i < total; i += (IDX)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cv) * 8;
    IDX r = i / cv;
    const int iw = (int)(r % (IDX)a.W);
    r /= (IDX)a.W;
    const int ih = (int)(r % (IDX)a.H);
    const int n = (int)(r / (IDX)a.H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // windows oh with oh*SH - PH <= ih <= oh*SH - PH + KH - 1
    const int hh = ih + a.PH, ww = iw + a.PW;
    const int oh_lo = hh >= a.KH ? (hh - a.KH) / a.SH + 1 : 0;
    const int oh_hi = min(a.OH - 1, hh / a.SH);
    const int ow_lo = ww >= a.KW ? (ww - a.KW) / a.SW + 1 : 0;
    const int ow_hi = min(a.OW - 1, ww / a.SW);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int kh = hh - oh * a.SH;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int kw = ww - ow * a.SW;
        const uint8_t k = (uint8_t)(kh * a.KW + kw);
        const int64_t o = (((int64_t)n * a.OH + oh) * a.OW + ow) * a.C + c8;
        const uint2 w = *reinterpret_cast<const uint2*>(idx + o);
        const uint32_t ws[2] = {w.x, w.y};
        bool any = false;
        uint8_t hit[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          hit[e] = ((ws[e >> 2] >> (8 * (e & 3))) & 0xffu) == k;
          any |= hit[e];
        }
        if (!any) continue;
        float g[8];
        Vec8<T>::load(g, dy + o);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += hit[e] ? g[e] : 0.f;
      }
    }
    Vec8<T>::store(dx + (((int64_t)n * a.H + ih) * a.W + iw) * a.C + c8, acc);
  }
}

inline int grid_for(int64_t total, int cus) {
  int64_t g = (total + 255) / 256;
  const int64_t cap = (int64_t)cus * 16;
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

// the grid-stride loop's last increment must not wrap a 32-bit counter
inline bool fits32(int64_t total, unsigned grid) { return total + (int64_t)grid * 256 < (int64_t)UINT32_MAX; }

}  // namespace pool

void maxpool_nhwc_fwd(const PoolArgs& a, const void* x, void* y, uint8_t* idx, int cus, hipStream_t s) {
  if (a.C % 8) throw std::runtime_error("maxpool_nhwc: C must be a multiple of 8");
  if (a.KH * a.KW > 255) throw std::runtime_error("maxpool_nhwc: window too large for 1-byte indices");
  dispatch_float(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    const int64_t total = (int64_t)a.N * a.OH * a.OW * (a.C / 8);
    const dim3 grid(pool::grid_for(total, cus));
    if (pool::fits32(total, grid.x))
      hipLaunchKernelGGL((pool::fwd_kernel<T, uint32_t>), grid, dim3(256), 0, s, a, (const T*)x, (T*)y, idx);
    else
      hipLaunchKernelGGL((pool::fwd_kernel<T, int64_t>), grid, dim3(256), 0, s, a, (const T*)x, (T*)y, idx);
  }, "maxpool_nhwc_fwd");
  check_launch("maxpool_nhwc_fwd");
}

void maxpool_nhwc_bwd(const PoolArgs& a, const void* dy, const uint8_t* idx, void* dx, int cus, hipStream_t s) {
  dispatch_float(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    const int64_t total = (int64_t)a.N * a.H * a.W * (a.C / 8);
    const dim3 grid(pool::grid_for(total, cus));
    if (pool::fits32(total, grid.x))
      hipLaunchKernelGGL((pool::bwd_kernel<T, uint32_t>), grid, dim3(256), 0, s, a, (const T*)dy, idx, (T*)dx);
    else
      hipLaunchKernelGGL((pool::bwd_kernel<T, int64_t>), grid, dim3(256), 0, s, a, (const T*)dy, idx, (T*)dx);
  }, "maxpool_nhwc_bwd");
  check_launch("maxpool_nhwc_bwd");
}

}  // namespace apex_amd
