// Deterministic column sums of an fp32 partial-sum slab [parts][n] — the second stage of every
// two-stage reduction here (GEMM bias gradients, LayerNorm dgamma / dbeta).
//
// One 256-thread block owns 16 columns: thread (col = tid & 15, grp = tid >> 4) sums rows grp,
// grp + 16, ... with four independent accumulators (four loads in flight per lane), then the 16
// group sums are added in a fixed order through LDS.  ceil(n / 16) blocks keep the whole chip
// busy even for n = 1024, where a column-per-thread loop over 256-512 partial rows is a serial
// chain of dependent-latency loads on a handful of CUs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

// Returns the sum of column `blockIdx.x * 16 + (threadIdx.x & 15)` in the threads with
// (threadIdx.x >> 4) == 0; other threads return 0.  All 256 threads must call it.
__device__ __forceinline__ float colreduce16(const float* __restrict__ part, int parts, int n,
                                             float (&red)[16][17]) {
  const int cl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < n) {
    int j = grp;
    for (; j + 48 < parts; j += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += part[(int64_t)(j + 16 * u) * n + c];
    }
    for (; j < parts; j += 16) a[0] += part[(int64_t)j * n + c];
  }
  red[grp][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  float s = 0.f;
  if (grp == 0) {
#pragma unroll
    for (int g = 0; g < 16; ++g) s += red[g][cl];
  }
  return s;
}

}  // namespace apex_amd
