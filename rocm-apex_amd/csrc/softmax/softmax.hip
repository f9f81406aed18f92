// Fused scale + mask + softmax (forward) and softmax backward for gfx950.
//
// Reference: csrc/megatron/scaled_masked_softmax.h:99 (fwd), :219 (bwd), dispatch :315-418;
// csrc/megatron/scaled_upper_triang_masked_softmax.h:114 / :233.  The reference maps one
// 32-lane "warp" per row with WARP_BATCH rows in registers and caps sk at 2048.
//
// gfx950 design: a row is owned by W wave64s (W = 1 for sk <= 2048, 4 or 8 beyond), each lane
// holds VPT vectors of 8 elements loaded with 16-byte loads (8-byte uint8 mask loads), so each
// element is read once and written once — the HBM minimum for this op.  Max/sum reductions are
// 6 xor-shuffle steps (+ an LDS step across waves).  Causal rows skip loading the masked upper
// triangle entirely (roughly half the input bytes).  Masking follows Megatron exactly:
// padding-masked scores become -10000 before the max, causal-masked entries are exactly 0.
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/softmax_api.h"

namespace apex_amd {
namespace smx {

template <int W>
constexpr int block_threads() { return W == 8 ? 512 : 256; }

struct Cfg {
  int W, VPT;
};
inline Cfg pick_cfg(int sk) {
  if (sk <= 512) return {1, 1};
  if (sk <= 1024) return {1, 2};
  if (sk <= 2048) return {1, 4};
  if (sk <= 4096) return {4, 2};
  if (sk <= 8192) return {4, 4};
  if (sk <= 16384) return {8, 4};
  return {0, 0};
}

template <int W, bool MAX>
__device__ __forceinline__ float row_reduce(float v, float* red, int row_in_block, int wave_in_row) {
  v = MAX ? wave_max(v) : wave_sum(v);
  if constexpr (W == 1) {
    return v;
  } else {
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[row_in_block * W + wave_in_row] = v;
    __syncthreads();
    float r = MAX ? -INFINITY : 0.f;
#pragma unroll
    for (int i = 0; i < W; ++i) r = MAX ? fmaxf(r, red[row_in_block * W + i]) : r + red[row_in_block * W + i];
    return r;
  }
}

__device__ __forceinline__ void load_mask8(uint8_t (&m)[8], const uint8_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    m[k] = (uint8_t)(u.x >> (8 * k));
    m[4 + k] = (uint8_t)(u.y >> (8 * k));
  }
}

template <typename T, int W, int VPT, int MODE>
__global__ void __launch_bounds__(block_threads<W>())
softmax_fwd_kernel(const T* __restrict__ x, const uint8_t* __restrict__ mask, T* __restrict__ y, int64_t rows,
                   int sq, int sk, int heads, int pad_batches, float scale) {
  constexpr int NT = block_threads<W>();
  constexpr int RPB = NT / 64 / W;
  __shared__ float red[2 * RPB * W];
  const int wave = threadIdx.x >> 6;
  const int row_in_block = wave / W;
  const int wave_in_row = wave % W;
  const int li = wave_in_row * 64 + (threadIdx.x & 63);
  const int64_t row = (int64_t)blockIdx.x * RPB + row_in_block;
  const bool valid = row < rows;
  const int64_t rr = valid ? row : 0;
  const int nv = sk >> 3;
  const int q = (int)(rr % sq);
  int limit = sk;  // columns < limit are live
  if constexpr (MODE == kMaskCausal) limit = q + 1 < sk ? q + 1 : sk;
  const uint8_t* mrow = nullptr;
  if constexpr (MODE == kMaskPad) {
    const int64_t bi = pad_batches == 1 ? 0 : rr / ((int64_t)heads * sq);
    mrow = mask + (bi * sq + q) * (int64_t)sk;
  }
  const T* xr = x + rr * sk;
  float r[VPT][8];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int v = j * W * 64 + li;
    const int c0 = v * 8;
    if (valid && v < nv && c0 < limit) {
      Vec8<T>::load(r[j], xr + c0);
      uint8_t m[8];
      if constexpr (MODE == kMaskPad) load_mask8(m, mrow + c0);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float e = r[j][k] * scale;
        if constexpr (MODE == kMaskPad) e = (m[k] == 1) ? -10000.f : e;
        if constexpr (MODE == kMaskCausal) e = (c0 + k < limit) ? e : -INFINITY;
        r[j][k] = e;
        mx = fmaxf(mx, e);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) r[j][k] = -INFINITY;
    }
  }
  mx = row_reduce<W, true>(mx, red, row_in_block, wave_in_row);
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float e = (r[j][k] == -INFINITY) ? 0.f : __expf(r[j][k] - mx);
      r[j][k] = e;
      sum += e;
    }
  sum = row_reduce<W, false>(sum, red + RPB * W, row_in_block, wave_in_row);
  const float inv = 1.f / sum;
  if (!valid) return;
  T* yr = y + rr * sk;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int v = j * W * 64 + li;
    if (v < nv) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = r[j][k] * inv;
      Vec8<T>::store(yr + v * 8, o);
    }
  }
}

template <typename T, int W, int VPT>
__global__ void __launch_bounds__(block_threads<W>())
softmax_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y, T* dx, int64_t rows, int sk, float scale) {
  constexpr int NT = block_threads<W>();
  constexpr int RPB = NT / 64 / W;
  __shared__ float red[RPB * W];
  const int wave = threadIdx.x >> 6;
  const int row_in_block = wave / W;
  const int wave_in_row = wave % W;
  const int li = wave_in_row * 64 + (threadIdx.x & 63);
  const int64_t row = (int64_t)blockIdx.x * RPB + row_in_block;
  const bool valid = row < rows;
  const int64_t rr = valid ? row : 0;
  const int nv = sk >> 3;
  float g[VPT][8], p[VPT][8];
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int v = j * W * 64 + li;
    if (valid && v < nv) {
      Vec8<T>::load(g[j], dy + rr * sk + v * 8);
      Vec8<T>::load(p[j], y + rr * sk + v * 8);
#pragma unroll
      for (int k = 0; k < 8; ++k) dot += g[j][k] * p[j][k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g[j][k] = 0.f;
        p[j][k] = 0.f;
      }
    }
  }
  dot = row_reduce<W, false>(dot, red, row_in_block, wave_in_row);
  if (!valid) return;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int v = j * W * 64 + li;
    if (v < nv) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = scale * p[j][k] * (g[j][k] - dot);
      Vec8<T>::store(dx + rr * sk + v * 8, o);
    }
  }
}

// ---- generic (any sk / alignment): block per row, three passes over L2-resident data ----
template <typename T, int MODE>
__global__ void __launch_bounds__(256)
softmax_fwd_generic_kernel(const T* __restrict__ x, const uint8_t* __restrict__ mask, T* __restrict__ y,
                           int64_t rows, int sq, int sk, int heads, int pad_batches, float scale) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  const int q = (int)(row % sq);
  const int limit = MODE == kMaskCausal ? (q + 1 < sk ? q + 1 : sk) : sk;
  const uint8_t* mrow = nullptr;
  if (MODE == kMaskPad) {
    const int64_t bi = pad_batches == 1 ? 0 : row / ((int64_t)heads * sq);
    mrow = mask + (bi * sq + q) * (int64_t)sk;
  }
  const T* xr = x + row * sk;
  auto score = [&](int c) {
    float e = to_f(xr[c]) * scale;
    if (MODE == kMaskPad && mrow[c] == 1) e = -10000.f;
    return e;
  };
  float mx = -INFINITY;
  for (int c = threadIdx.x; c < limit; c += 256) mx = fmaxf(mx, score(c));
  mx = block_max(mx, red);
  float sum = 0.f;
  for (int c = threadIdx.x; c < limit; c += 256) sum += __expf(score(c) - mx);
  sum = block_sum(sum, red + 4);
  const float inv = 1.f / sum;
  T* yr = y + row * sk;
  for (int c = threadIdx.x; c < sk; c += 256) yr[c] = from_f<T>(c < limit ? __expf(score(c) - mx) * inv : 0.f);
}

template <typename T>
__global__ void __launch_bounds__(256)
softmax_bwd_generic_kernel(const T* __restrict__ dy, const T* __restrict__ y, T* dx, int64_t rows, int sk,
                           float scale) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  float dot = 0.f;
  for (int c = threadIdx.x; c < sk; c += 256) dot += to_f(dy[row * sk + c]) * to_f(y[row * sk + c]);
  dot = block_sum(dot, red);
  for (int c = threadIdx.x; c < sk; c += 256) {
    const float p = to_f(y[row * sk + c]);
    dx[row * sk + c] = from_f<T>(scale * p * (to_f(dy[row * sk + c]) - dot));
  }
}

static bool al16(const void* p) { return p == nullptr || ((uintptr_t)p & 15u) == 0; }
static bool al8(const void* p) { return p == nullptr || ((uintptr_t)p & 7u) == 0; }

template <typename T, int W, int VPT, int MODE>
static void launch_fwd(const SoftmaxFwdArgs& a, hipStream_t s) {
  constexpr int RPB = block_threads<W>() / 64 / W;
  const int64_t grid = (a.rows + RPB - 1) / RPB;
  hipLaunchKernelGGL((softmax_fwd_kernel<T, W, VPT, MODE>), dim3((unsigned)grid), dim3(block_threads<W>()), 0, s,
                     (const T*)a.x, a.mask, (T*)a.y, a.rows, a.sq, a.sk, a.heads, a.pad_batches, a.scale);
}

template <typename T, int MODE>
static void fwd_mode(const SoftmaxFwdArgs& a, hipStream_t s) {
  const Cfg c = pick_cfg(a.sk);
  const bool fast = c.W > 0 && a.sk % 8 == 0 && al16(a.x) && al16(a.y) && al8(a.mask);
  if (!fast) {
    hipLaunchKernelGGL((softmax_fwd_generic_kernel<T, MODE>), dim3((unsigned)a.rows), dim3(256), 0, s,
                       (const T*)a.x, a.mask, (T*)a.y, a.rows, a.sq, a.sk, a.heads, a.pad_batches, a.scale);
    return;
  }
  if (c.W == 1 && c.VPT == 1) launch_fwd<T, 1, 1, MODE>(a, s);
  else if (c.W == 1 && c.VPT == 2) launch_fwd<T, 1, 2, MODE>(a, s);
  else if (c.W == 1 && c.VPT == 4) launch_fwd<T, 1, 4, MODE>(a, s);
  else if (c.W == 4 && c.VPT == 2) launch_fwd<T, 4, 2, MODE>(a, s);
  else if (c.W == 4 && c.VPT == 4) launch_fwd<T, 4, 4, MODE>(a, s);
  else launch_fwd<T, 8, 4, MODE>(a, s);
}

template <typename T, int W, int VPT>
static void launch_bwd(const SoftmaxBwdArgs& a, hipStream_t s) {
  constexpr int RPB = block_threads<W>() / 64 / W;
  const int64_t grid = (a.rows + RPB - 1) / RPB;
  hipLaunchKernelGGL((softmax_bwd_kernel<T, W, VPT>), dim3((unsigned)grid), dim3(block_threads<W>()), 0, s,
                     (const T*)a.dy, (const T*)a.y, (T*)a.dx, a.rows, a.sk, a.scale);
}

}  // namespace smx

void softmax_fwd(const SoftmaxFwdArgs& a, hipStream_t s) {
  if (a.rows <= 0 || a.sk <= 0) return;
  dispatch_float(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (a.mode == kMaskPad) smx::fwd_mode<T, kMaskPad>(a, s);
    else if (a.mode == kMaskCausal) smx::fwd_mode<T, kMaskCausal>(a, s);
    else smx::fwd_mode<T, kMaskNone>(a, s);
  }, "softmax forward");
  check_launch("softmax forward");
}

void softmax_bwd(const SoftmaxBwdArgs& a, hipStream_t s) {
  if (a.rows <= 0 || a.sk <= 0) return;
  dispatch_float(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    const smx::Cfg c = smx::pick_cfg(a.sk);
    const bool fast = c.W > 0 && a.sk % 8 == 0 && smx::al16(a.dy) && smx::al16(a.y) && smx::al16(a.dx);
    if (!fast) {
      hipLaunchKernelGGL((smx::softmax_bwd_generic_kernel<T>), dim3((unsigned)a.rows), dim3(256), 0, s,
                         (const T*)a.dy, (const T*)a.y, (T*)a.dx, a.rows, a.sk, a.scale);
    } else if (c.W == 1 && c.VPT == 1) smx::launch_bwd<T, 1, 1>(a, s);
    else if (c.W == 1 && c.VPT == 2) smx::launch_bwd<T, 1, 2>(a, s);
    else if (c.W == 1 && c.VPT == 4) smx::launch_bwd<T, 1, 4>(a, s);
    else if (c.W == 4 && c.VPT == 2) smx::launch_bwd<T, 4, 2>(a, s);
    else if (c.W == 4 && c.VPT == 4) smx::launch_bwd<T, 4, 4>(a, s);
    else smx::launch_bwd<T, 8, 4>(a, s);
  }, "softmax backward");
  check_launch("softmax backward");
}

}  // namespace apex_amd
