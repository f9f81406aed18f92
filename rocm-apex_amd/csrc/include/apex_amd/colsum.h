// Block-level column reduction of the channel-tiled statistics kernels (BN / SyncBN partials).
//
// A block is TX channel-vectors x TY rows; every lane holds NQ accumulators of VEC channels.  The
// per-ty values are staged in LDS component-major, smem[(q*VEC + k) * KS + ty*TX + tx] with
// KS = TX*TY + 8: for one component k a wave's stores are lane-contiguous (conflict-free), and
// the reduction lanes o = (q, tx, k) -- k fastest, so the global partial rows are written
// coalesced -- read word offsets 8k + tx + const, distinct banks for the 8 x 8 lanes of a
// 64-lane group.  (The previous [ty][tx*8 + k] image put the 8 components of a lane 8 words
// apart: 84% of the LDS cycles of the BN partial kernels were bank conflicts, profiles/
// pmc_kernels_r02.md, and only the TX lanes of ty == 0 reduced, TY loads in series each.)
// Every output is summed over ty in a fixed order (deterministic).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace apex_amd {

template <int VEC>
struct ColSum {
  // row pitch TX*TY + 4 words: the reduction's 32-lane groups read components k = 0..7 of lane
  // columns txo = 0..3 at banks 4k + txo (TX*TY is a multiple of 32), all distinct; with + 8 the
  // components k and k + 4 shared a bank (2-way: the 33 % conflict cycles of the BN partial
  // kernels in profiles/pmc_resnet_kernels_r04al.md)
  static __host__ __device__ __forceinline__ int ks(int tx, int ty) { return tx * ty + 4; }
  static __host__ __device__ __forceinline__ size_t lds_floats(int tx, int ty, int nq) {
    return (size_t)nq * VEC * ks(tx, ty);
  }

  static __device__ __forceinline__ void stash(float* smem, int q, const float (&a)[VEC], int tx, int ty, int TX,
                                               int TY) {
    const int base = ty * TX + tx, K = ks(TX, TY);
#pragma unroll
    for (int k = 0; k < VEC; ++k) smem[(q * VEC + k) * K + base] = a[k];
  }

  // column q*VEC + k of lane-column txo, summed over the TY rows (4 independent chains)
  static __device__ __forceinline__ float column(const float* smem, int q, int k, int txo, int TX, int TY) {
    const float* p = smem + (q * VEC + k) * ks(TX, TY) + txo;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int j = 0;
    for (; j + 3 < TY; j += 4) {
      s0 += p[j * TX];
      s1 += p[(j + 1) * TX];
      s2 += p[(j + 2) * TX];
      s3 += p[(j + 3) * TX];
    }
    for (; j < TY; ++j) s0 += p[j * TX];
    return (s0 + s1) + (s2 + s3);
  }

  // after a barrier: part[q * q_stride + row * c + ch] = column sums of the block's channels
  static __device__ __forceinline__ void reduce_store(const float* smem, int nq, int TX, int TY, int c,
                                                      int cbase, float* __restrict__ part, int64_t q_stride,
                                                      int64_t row) {
    const int nthreads = TX * TY, tid = threadIdx.y * TX + threadIdx.x;
    for (int o = tid; o < nq * VEC * TX; o += nthreads) {
      const int q = o / (VEC * TX), r = o - q * VEC * TX;
      const int txo = r / VEC, k = r - txo * VEC;
      const int ch = cbase + txo * VEC + k;
      if (ch >= c) continue;
      part[q * q_stride + row * c + ch] = column(smem, q, k, txo, TX, TY);
    }
  }
};

}  // namespace apex_amd
