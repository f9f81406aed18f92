// Layout passes of the convolution routes (NHWC, 16-bit).
//
// conv_subsample2x: y[n][i][j][:] = x[n][2 i][2 j][:] — the operand of a stride-2 1x1 convolution
// (the ResNet downsample) as a dense [N * ceil(H/2) * ceil(W/2)][C] matrix, so the native 1x1 GEMMs
// (conv1x1_bn.hip, its BN-statistics epilogue and split-M weight gradient) run it.  One 16-byte
// vector per lane, grid-stride; a pixel's C channels are contiguous in both tensors, so each wave
// reads and writes whole 128-byte runs (torch's generic strided copy took 36 us per ResNet call).
#include "apex_amd/conv_api.h"
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

}  // namespace layout

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
