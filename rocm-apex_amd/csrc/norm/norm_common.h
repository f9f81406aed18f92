// Shared pieces of the LayerNorm / RMSNorm kernels (fwd in layer_norm_fwd.hip, bwd in
// layer_norm_bwd.hip).
//
// Geometry (MI355X, wave64): a row of n2 elements is owned by W waves (W = 1, 4 or 8); each
// lane holds VPT vectors of 8 elements in registers (one 16-byte load per vector for 16-bit
// types), so a row is read from HBM exactly once per pass and all statistics are two-pass
// (mean, then sum of squared deviations) on register-resident data — no Welford merge chain,
// no re-read.  Vector j of lane li covers columns [(j*W*64 + li)*8, +8).  Fast-path widths:
// n2 % 8 == 0 and n2 <= 65536 (above 16384: one 1024-thread workgroup of 16 waves per row with
// gamma / beta read per row from L2 instead of held in registers, the "wide" kernels); anything
// else takes the generic block-per-row kernels.
#pragma once
#include "apex_amd/colreduce.h"
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/norm_api.h"

namespace apex_amd {
namespace norm {

struct Cfg {
  int W;    // waves per row
  int VPT;  // 8-element vectors per lane
};

// smallest register-resident geometry that covers n2 (0 => generic path)
inline Cfg pick_cfg(int n2) {
  if (n2 <= 512) return {1, 1};
  if (n2 <= 1024) return {1, 2};
  if (n2 <= 2048) return {1, 4};
  if (n2 <= 4096) return {4, 2};
  if (n2 <= 8192) return {4, 4};
  if (n2 <= 16384) return {8, 4};
  if (n2 <= 32768) return {16, 4};
  if (n2 <= 65536) return {16, 8};
  return {0, 0};
}

template <int W>
constexpr int block_threads() { return W == 16 ? 1024 : W == 8 ? 512 : 256; }

// Sum over the W waves of one row; `red` is LDS of [rows_per_block * W] floats.  Every thread
// of the block must call it (it contains barriers).
template <int W>
__device__ __forceinline__ float row_sum(float v, float* red, int row_in_block, int wave_in_row) {
  v = wave_sum(v);
  if constexpr (W == 1) {
    return v;
  } else {
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[row_in_block * W + wave_in_row] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < W; ++i) s += red[row_in_block * W + i];
    return s;
  }
}

template <int W>
__device__ __forceinline__ void row_sum2(float& a, float& b, float* red, int row_in_block, int wave_in_row) {
  a = wave_sum(a);
  b = wave_sum(b);
  if constexpr (W > 1) {
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
      red[2 * (row_in_block * W + wave_in_row)] = a;
      red[2 * (row_in_block * W + wave_in_row) + 1] = b;
    }
    __syncthreads();
    a = 0.f;
    b = 0.f;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      a += red[2 * (row_in_block * W + i)];
      b += red[2 * (row_in_block * W + i) + 1];
    }
  }
}

// 8 raw elements held in registers between a prefetch and their use (16-bit types: one 16-byte
// load; fp32: two).  Keeping the NEXT row's data raw lets its loads stay in flight while the
// current row is reduced (the software pipeline of the persistent kernels).
template <typename T>
struct Raw8 {
  static constexpr int kWords = (int)sizeof(T) * 2;  // 32-bit words for 8 elements
  uint32_t w[kWords];
  __device__ __forceinline__ void load(const T* p) {
#pragma unroll
    for (int i = 0; i < kWords / 4; ++i) {
      const uint4 u = reinterpret_cast<const uint4*>(p)[i];
      w[4 * i] = u.x;
      w[4 * i + 1] = u.y;
      w[4 * i + 2] = u.z;
      w[4 * i + 3] = u.w;
    }
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < kWords; ++i) w[i] = 0u;
  }
  __device__ __forceinline__ void unpack(float (&r)[8]) const {
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] = __uint_as_float(w[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        r[2 * i] = to_f(T{(uint16_t)(w[i] & 0xffffu)});
        r[2 * i + 1] = to_f(T{(uint16_t)(w[i] >> 16)});
      }
    }
  }
};

// typed dispatch over the (input, weight, output) triples the python layer can produce
template <typename F>
inline void dispatch_norm_types(int in_t, int w_t, int out_t, F&& f) {
  dispatch_float(in_t, [&](auto ti) {
    dispatch_float(w_t, [&](auto tw) {
      using TI = typename decltype(ti)::type;
      using TW = typename decltype(tw)::type;
      if (out_t == in_t) {
        f(ti, tw, Tag<TI>{});
      } else if (out_t == w_t) {
        f(ti, tw, Tag<TW>{});
      } else {
        throw std::runtime_error("norm: output dtype must equal the input or the weight dtype");
      }
    }, "norm weight");
  }, "norm input");
}

}  // namespace norm
}  // namespace apex_amd
