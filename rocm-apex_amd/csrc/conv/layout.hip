// Layout passes of the convolution routes (NHWC, 16-bit).
//
// conv_subsample2x: y[n][i][j][:] = x[n][2 i][2 j][:] — the operand of a stride-2 1x1 convolution
// (the ResNet downsample) as a dense [N * ceil(H/2) * ceil(W/2)][C] matrix, so the native 1x1 GEMMs
// (conv1x1_bn.hip, its BN-statistics epilogue and split-M weight gradient) run it.  One 16-byte
// vector per lane, grid-stride; a pixel's C channels are contiguous in both tensors, so each wave
// reads and writes whole 128-byte runs (torch's generic strided copy took 36 us per ResNet call).
// conv_tap_weights: the data-gradient weight image (below).
#include "apex_amd/conv_api.h"
#include "apex_amd/device.h"
#include "apex_amd/layout_extra.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/fastdiv.h"

#include <stdexcept>

namespace apex_amd {
namespace layout {

__global__ void __launch_bounds__(256) subsample2x_kernel(const uint4* __restrict__ x, uint4* __restrict__ y,
                                                          uint32_t total, FastDiv cv, FastDiv w2, FastDiv hw2, int h,
                                                          int w) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t pix = fdiv(i, cv), v = i - pix * cv.d;
    const uint32_t nn = fdiv(pix, hw2), rem = pix - nn * hw2.d;
    const uint32_t oy = fdiv(rem, w2), ox = rem - oy * w2.d;
    const size_t src = (((size_t)nn * h + 2 * oy) * w + 2 * ox) * cv.d + v;
    y[i] = x[src];
  }
}

// tap_weights: dst[c][j][k] = w[k][tap[j]][c] — the [C][taps][K] operand image the tap kernels
// take for a data gradient (conv_tap_dgrad), from the channels_last [K][R S][C] weight, with an
// optional tap subset (the stride-2 phases).  A 64 (k) x 64 (c) tile per workgroup through LDS:
// 16-byte reads along c, 16-byte writes along k (torch's permute-copy ran a 2-byte strided
// kernel: ~13 us per ResNet-50 3x3 layer and step).
struct TapList {
  int n;
  int t[9];
};

template <int PAD>
__global__ void __launch_bounds__(256) tap_weights_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ dst,
                                                          int k, int c, int rs, TapList taps) {
  __shared__ uint16_t tile[64][64 + PAD];
  const int c0 = blockIdx.x * 64, k0 = blockIdx.y * 64, j = blockIdx.z;
  const int tap = taps.t[j];
  const int tid = threadIdx.x;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = tid / 8 + 32 * h, c8 = (tid % 8) * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (k0 + r < k && c0 + c8 < c)
      v = *reinterpret_cast<const uint4*>(w + ((size_t)(k0 + r) * rs + tap) * c + c0 + c8);
    const uint32_t q[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tile[r][c8 + 2 * e] = (uint16_t)(q[e] & 0xffffu);
      tile[r][c8 + 2 * e + 1] = (uint16_t)(q[e] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int cc = tid / 8 + 32 * h, k8 = (tid % 8) * 8;
    if (c0 + cc >= c || k0 + k8 >= k) continue;
    uint32_t q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      q[e] = (uint32_t)tile[k8 + 2 * e][cc] | ((uint32_t)tile[k8 + 2 * e + 1][cc] << 16);
    *reinterpret_cast<uint4*>(dst + ((size_t)(c0 + cc) * taps.n + j) * k + k0 + k8) = make_uint4(q[0], q[1], q[2], q[3]);
  }
}

// spatial_broadcast: y[n][p][c] = g[n][c] * scale for p < hw — the input gradient of a global
// average pool written straight into channels_last memory (16-byte stores, grid-stride)
template <typename T>
__global__ void __launch_bounds__(256) spatial_broadcast_kernel(const T* __restrict__ g, T* __restrict__ y,
                                                                uint32_t total, FastDiv cv, FastDiv hwd, float scale) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t pix = fdiv(i, cv), v = i - pix * cv.d;
    const uint32_t nn = fdiv(pix, hwd);
    float a[8];
    Vec8<T>::load(a, g + ((size_t)nn * cv.d + v) * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] *= scale;
    Vec8<T>::store(y + (size_t)i * 8, a);
  }
}

}  // namespace layout

void spatial_broadcast(const void* g, void* y, int n, int hw, int c, float scale, int dtype, int cus, hipStream_t s) {
  if ((dtype != kBF16 && dtype != kF16) || c % 8 || n <= 0 || hw <= 0)
    throw std::runtime_error("spatial_broadcast: 16-bit, C % 8 == 0");
  if (((uintptr_t)g & 15) || ((uintptr_t)y & 15)) throw std::runtime_error("spatial_broadcast: 16-byte alignment");
  const int64_t total = (int64_t)n * hw * (c / 8);
  if (total >= (1ll << 32)) throw std::runtime_error("spatial_broadcast: output past 2^32 vectors");
  int64_t grid = (total + 255) / 256;
  if (grid > (int64_t)cus * 8) grid = (int64_t)cus * 8;
  dispatch_16(dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    hipLaunchKernelGGL((layout::spatial_broadcast_kernel<T>), dim3((unsigned)grid), dim3(256), 0, s, (const T*)g, (T*)y,
                       (uint32_t)total, make_fastdiv((uint32_t)(c / 8)), make_fastdiv((uint32_t)hw), scale);
  }, "spatial_broadcast");
  check_launch("spatial_broadcast");
}

void conv_tap_weights(const void* w, void* dst, int k, int c, int rs, const int* taps, int ntaps, hipStream_t s) {
  if (k % 8 || c % 8 || k <= 0 || c <= 0 || ntaps < 1 || ntaps > 9 || rs < 1 || rs > 9)
    throw std::runtime_error("conv_tap_weights: K, C multiples of 8, 1-9 taps");
  if (((uintptr_t)w & 15) || ((uintptr_t)dst & 15)) throw std::runtime_error("conv_tap_weights: 16-byte alignment");
  layout::TapList tl{};
  tl.n = ntaps;
  for (int j = 0; j < ntaps; ++j) {
    if (taps[j] < 0 || taps[j] >= rs) throw std::runtime_error("conv_tap_weights: tap index out of range");
    tl.t[j] = taps[j];
  }
  hipLaunchKernelGGL(layout::tap_weights_kernel<2>, dim3((unsigned)((c + 63) / 64), (unsigned)((k + 63) / 64), ntaps),
                     dim3(256), 0, s, (const uint16_t*)w, (uint16_t*)dst, k, c, rs, tl);
  check_launch("conv_tap_weights");
}

void conv_subsample2x(const void* x, void* y, int n, int h, int w, int c, int dtype, int cus, hipStream_t s) {
  if ((dtype != kBF16 && dtype != kF16) || c % 8 || n <= 0 || h <= 0 || w <= 0)
    throw std::runtime_error("conv_subsample2x: 16-bit NHWC with C % 8 == 0");
  if (((uintptr_t)x & 15) || ((uintptr_t)y & 15)) throw std::runtime_error("conv_subsample2x: 16-byte alignment");
  const int h2 = (h + 1) / 2, w2 = (w + 1) / 2;
  const int64_t total = (int64_t)n * h2 * w2 * (c / 8);
  if (total >= (1ll << 32)) throw std::runtime_error("conv_subsample2x: output past 2^32 vectors");
  int64_t grid = (total + 255) / 256;
  if (grid > (int64_t)cus * 8) grid = (int64_t)cus * 8;
  hipLaunchKernelGGL(layout::subsample2x_kernel, dim3((unsigned)grid), dim3(256), 0, s, (const uint4*)x, (uint4*)y,
                     (uint32_t)total, make_fastdiv((uint32_t)(c / 8)), make_fastdiv((uint32_t)w2),
                     make_fastdiv((uint32_t)(h2 * w2)), h, w);
  check_launch("conv_subsample2x");
}

}  // namespace apex_amd
