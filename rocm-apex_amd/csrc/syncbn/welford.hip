// Batch-norm statistics and apply kernels for gfx950 (SyncBatchNorm, fused BN+ReLU).
//
// Reference: csrc/welford.cu — welford_kernel :272 (NCHW), welford_kernel_c_last :454 (NHWC with
// grid semaphores), welford_kernel_parallel :597, batchnorm_forward(_c_last) :314/:633,
// relu_backward_c_last :686, reduce_bn(_c_last) :344/:739, batchnorm_backward(_c_last) :411/:895.
//
// gfx950 design:
//  * c_last ([M, C], the ResNet/channels_last case): a lane owns 8 consecutive channels and
//    moves them with one 16-byte load; a 256-thread block is TX channel-vectors x TY rows, so a
//    wave reads whole contiguous row segments.  Statistics are per-lane Welford (mean, M2, n),
//    merged across TY in LDS with Chan's formula, then across the gy row-partitions by a tiny
//    finalize kernel in a fixed order (deterministic; no float atomics, no semaphores).
//  * reductions for backward (sum_dy, sum_dy*(x-mean)) use the same tiling with plain sums.
//  * fused ReLU: forward writes relu(bn(x)+z); backward kernels recompute that value in
//    registers to mask dy instead of materialising the masked gradient.
//  * elementwise kernels are grid-stride over 8-element vectors, grid sized to the 256 CUs.
#include "apex_amd/colsum.h"
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/syncbn_api.h"

namespace apex_amd {
namespace bn {

struct Tiling {
  int tx, ty, gx, gy, vec;
};

inline Tiling clast_tiling(int64_t m, int c, bool vec8, int cus) {
  Tiling t;
  t.vec = vec8 ? 8 : 1;
  const int cv = (c + t.vec - 1) / t.vec;
  t.tx = cv < 64 ? cv : 64;
  t.ty = 256 / t.tx;
  if (t.ty > 64) t.ty = 64;
  t.gx = (cv + t.tx - 1) / t.tx;
  int64_t gy = ((int64_t)cus * 4 + t.gx - 1) / t.gx;
  const int64_t rows_cap = (m + t.ty - 1) / t.ty;
  if (gy > rows_cap) gy = rows_cap;
  if (gy > 256) gy = 256;
  t.gy = (int)(gy < 1 ? 1 : gy);
  return t;
}

inline int nchw_parts(int64_t n, int64_t s, int c, int cus) {
  int64_t p = ((int64_t)cus * 4 + c - 1) / c;
  const int64_t cap = (n * s + 255) / 256;
  if (p > cap) p = cap;
  if (p > 256) p = 256;
  return (int)(p < 1 ? 1 : p);
}

template <typename T, int VEC>
__device__ __forceinline__ void load_vec(float (&v)[VEC], const T* p) {
  if constexpr (VEC == 8) Vec8<T>::load(v, p);
  else v[0] = to_f(p[0]);
}
template <typename T, int VEC>
__device__ __forceinline__ void store_vec(T* p, const float (&v)[VEC]) {
  if constexpr (VEC == 8) Vec8<T>::store(p, v);
  else p[0] = from_f<T>(v[0]);
}

__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float mb, float m2b) {
  if (nb == 0.f) return;
  const float nn = n + nb;
  const float d = mb - mean;
  const float f = nb / nn;
  mean += d * f;
  m2 += m2b + d * d * n * f;
  n = nn;
}

// ---------------------------------------------------------------------------------------------
// statistics
// ---------------------------------------------------------------------------------------------
template <typename T, int VEC>
__global__ void __launch_bounds__(256) welford_clast_kernel(const T* __restrict__ x, int64_t m, int c,
                                                            float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int TX = blockDim.x, TY = blockDim.y, tx = threadIdx.x, ty = threadIdx.y;
  const int c0 = (blockIdx.x * TX + tx) * VEC;
  const bool active = c0 < c;
  float mean[VEC], m2[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) mean[k] = m2[k] = 0.f;
  float n = 0.f;
  for (int64_t r = (int64_t)blockIdx.y * TY + ty; r < m; r += (int64_t)TY * gridDim.y) {
    n += 1.f;
    if (active) {
      float v[VEC];
      load_vec<T, VEC>(v, x + r * c + c0);
      const float inv = 1.f / n;
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const float d = v[k] - mean[k];
        mean[k] += d * inv;
        m2[k] += d * (v[k] - mean[k]);
      }
    }
  }
  // (mean, M2) staged component-major (apex_amd/colsum.h layout), merged over ty with Chan's
  // formula in a fixed order by lanes o = (tx, k), k fastest
  using CS = ColSum<VEC>;
  const int KS = CS::ks(TX, TY);
  float* sn = smem + CS::lds_floats(TX, TY, 2);
  CS::stash(smem, 0, mean, tx, ty, TX, TY);
  CS::stash(smem, 1, m2, tx, ty, TX, TY);
  if (tx == 0) sn[ty] = n;
  __syncthreads();
  const int gy = gridDim.y, tid = ty * TX + tx;
  for (int o = tid; o < VEC * TX; o += TX * TY) {
    const int txo = o / VEC, k = o - txo * VEC;
    const int ch = (blockIdx.x * TX + txo) * VEC + k;
    if (ch >= c) continue;
    const float* pm = smem + k * KS + txo;
    const float* p2 = smem + (VEC + k) * KS + txo;
    float nn = sn[0], mm = pm[0], MM = p2[0];
    for (int j = 1; j < TY; ++j) chan_merge(nn, mm, MM, sn[j], pm[j * TX], p2[j * TX]);
    ws[(int64_t)blockIdx.y * c + ch] = mm;
    ws[(int64_t)gy * c + (int64_t)blockIdx.y * c + ch] = MM;
  }
  if (blockIdx.x == 0 && tid == 0) {
    float nn = 0.f;
    for (int j = 0; j < TY; ++j) nn += sn[j];
    ws[2 * (int64_t)gy * c + blockIdx.y] = nn;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) welford_nchw_kernel(const T* __restrict__ x, int64_t n, int c, int64_t s,
                                                           float* __restrict__ ws) {
  __shared__ float sm[256], s2[256], sn[256];
  const int ch = blockIdx.x;
  const int64_t total = n * s;
  float mean = 0.f, m2 = 0.f, cnt = 0.f;
  for (int64_t j = (int64_t)blockIdx.y * 256 + threadIdx.x; j < total; j += (int64_t)256 * gridDim.y) {
    const int64_t ni = j / s, si = j - ni * s;
    const float v = to_f(x[(ni * c + ch) * s + si]);
    cnt += 1.f;
    const float d = v - mean;
    mean += d / cnt;
    m2 += d * (v - mean);
  }
  sm[threadIdx.x] = mean;
  s2[threadIdx.x] = m2;
  sn[threadIdx.x] = cnt;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      float nn = sn[threadIdx.x], mm = sm[threadIdx.x], MM = s2[threadIdx.x];
      chan_merge(nn, mm, MM, sn[threadIdx.x + off], sm[threadIdx.x + off], s2[threadIdx.x + off]);
      sn[threadIdx.x] = nn;
      sm[threadIdx.x] = mm;
      s2[threadIdx.x] = MM;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int gy = gridDim.y;
    ws[(int64_t)blockIdx.y * c + ch] = sm[0];
    ws[(int64_t)gy * c + (int64_t)blockIdx.y * c + ch] = s2[0];
    ws[2 * (int64_t)gy * c + (int64_t)gy * ch + blockIdx.y] = sn[0];  // per (channel, part) count
  }
}

// merge gy partial (mean, M2, n) rows per channel in fixed order; cnt_stride: 0 => counts[gy]
// shared by all channels (c_last), gy => counts[c][gy] (nchw)
__global__ void welford_finalize_kernel(const float* __restrict__ ws, int gy, int c, int per_channel_counts,
                                        float* __restrict__ mean, float* __restrict__ var_biased) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const float* cnts = ws + 2 * (int64_t)gy * c + (per_channel_counts ? (int64_t)gy * ch : 0);
  float n = 0.f, mm = 0.f, MM = 0.f;
  for (int j = 0; j < gy; ++j) chan_merge(n, mm, MM, cnts[j], ws[(int64_t)j * c + ch], ws[(int64_t)(gy + j) * c + ch]);
  mean[ch] = mm;
  var_biased[ch] = n > 0.f ? MM / n : 0.f;
}

__global__ void welford_parallel_kernel(const float* __restrict__ mean_all, const float* __restrict__ var_all,
                                        const int* __restrict__ count_all, int world, int c, float eps,
                                        float* __restrict__ mean, float* __restrict__ var_u, float* __restrict__ inv_std) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  float n = 0.f, mm = 0.f, MM = 0.f;
  for (int w = 0; w < world; ++w) {
    const float nb = (float)count_all[w];
    chan_merge(n, mm, MM, nb, mean_all[(int64_t)w * c + ch], var_all[(int64_t)w * c + ch] * nb);
  }
  mean[ch] = mm;
  var_u[ch] = n > 1.f ? MM / (n - 1.f) : 0.f;
  inv_std[ch] = rsqrtf(MM / n + eps);
}

// ---------------------------------------------------------------------------------------------
// parameter access shared by the apply / backward kernels
// ---------------------------------------------------------------------------------------------
// c_last: the VEC elements of a vector are VEC consecutive channels; nchw: one channel.
template <typename TW, int VEC, bool CLAST = true>
struct ChParams {
  float mean[VEC], istd[VEC], w[VEC], b[VEC];
  __device__ __forceinline__ void load(const BnParams& p, int c0) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const int ch = CLAST ? c0 + k : c0;
      mean[k] = p.mean[ch];
      istd[k] = p.inv_std[ch];
      w[k] = p.w ? to_f(reinterpret_cast<const TW*>(p.w)[ch]) : 1.f;
      b[k] = p.b ? to_f(reinterpret_cast<const TW*>(p.b)[ch]) : 0.f;
    }
  }
};

// ---------------------------------------------------------------------------------------------
// forward apply (+z, +relu)
// ---------------------------------------------------------------------------------------------
template <typename T, typename TW, int VEC, bool CLAST>
__global__ void __launch_bounds__(256) bn_forward_kernel(const T* __restrict__ x, BnParams p, FusedRelu r,
                                                         T* __restrict__ y, int64_t total, int c, int64_t s) {
  const int64_t nvec = total / VEC;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * VEC;
    const int c0 = CLAST ? (int)(e % c) : (int)((e / s) % c);
    ChParams<TW, VEC, CLAST> q;
    q.load(p, c0);
    float v[VEC];
    load_vec<T, VEC>(v, x + e);
    float zz[VEC];
    if (r.z) load_vec<T, VEC>(zz, reinterpret_cast<const T*>(r.z) + e);
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      float o = (v[k] - q.mean[k]) * q.istd[k] * q.w[k] + q.b[k];
      if (r.z) o += zz[k];
      if (r.on) o = fmaxf(o, 0.f);
      v[k] = o;
    }
    store_vec<T, VEC>(y + e, v);
  }
}

// recompute relu(bn(x)+z) > 0 for the fused-relu backward
template <typename T, int VEC, typename Q>
__device__ __forceinline__ void relu_mask(float (&dy)[VEC], const float (&v)[VEC], const Q& q, const FusedRelu& r,
                                          int64_t e) {
  if (!r.on) return;
  float zz[VEC];
  if (r.z) load_vec<T, VEC>(zz, reinterpret_cast<const T*>(r.z) + e);
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    float o = (v[k] - q.mean[k]) * q.istd[k] * q.w[k] + q.b[k];
    if (r.z) o += zz[k];
    if (!(o > 0.f)) dy[k] = 0.f;
  }
}

template <typename T, typename TW, int VEC>
__global__ void __launch_bounds__(256) bn_relu_bw_kernel(const T* __restrict__ dy, const T* __restrict__ x, BnParams p,
                                                         FusedRelu r, T* __restrict__ out, int64_t total, int c) {
  const int64_t nvec = total / VEC;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * VEC;
    const int c0 = (int)(e % c);
    ChParams<TW, VEC> q;
    q.load(p, c0);
    float v[VEC], g[VEC];
    load_vec<T, VEC>(v, x + e);
    load_vec<T, VEC>(g, dy + e);
    relu_mask<T, VEC>(g, v, q, r, e);
    store_vec<T, VEC>(out + e, g);
  }
}

// ---------------------------------------------------------------------------------------------
// backward reductions
// ---------------------------------------------------------------------------------------------
template <typename T, typename TW, int VEC>
__global__ void __launch_bounds__(256) reduce_clast_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                           BnParams p, FusedRelu r, int64_t m, int c,
                                                           float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int TX = blockDim.x, TY = blockDim.y, tx = threadIdx.x, ty = threadIdx.y;
  const int c0 = (blockIdx.x * TX + tx) * VEC;
  const bool active = c0 < c;
  float s1[VEC], s2[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) s1[k] = s2[k] = 0.f;
  if (active) {
    ChParams<TW, VEC> q;
    q.load(p, c0);
    for (int64_t rr = (int64_t)blockIdx.y * TY + ty; rr < m; rr += (int64_t)TY * gridDim.y) {
      const int64_t e = rr * c + c0;
      float v[VEC], g[VEC];
      load_vec<T, VEC>(v, x + e);
      load_vec<T, VEC>(g, dy + e);
      relu_mask<T, VEC>(g, v, q, r, e);
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        s1[k] += g[k];
        s2[k] += g[k] * (v[k] - q.mean[k]);
      }
    }
  }
  ColSum<VEC>::stash(smem, 0, s1, tx, ty, TX, TY);
  ColSum<VEC>::stash(smem, 1, s2, tx, ty, TX, TY);
  __syncthreads();
  ColSum<VEC>::reduce_store(smem, 2, TX, TY, c, blockIdx.x * TX * VEC, ws, (int64_t)gridDim.y * c, blockIdx.y);
}

template <typename T>
__global__ void __launch_bounds__(256) reduce_nchw_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const float* __restrict__ mean, int64_t n, int c, int64_t s,
                                                          float* __restrict__ ws) {
  __shared__ float r1[4], r2[4];
  const int ch = blockIdx.x;
  const float mu = mean[ch];
  const int64_t total = n * s;
  float a = 0.f, b = 0.f;
  for (int64_t j = (int64_t)blockIdx.y * 256 + threadIdx.x; j < total; j += (int64_t)256 * gridDim.y) {
    const int64_t ni = j / s, si = j - ni * s;
    const int64_t off = (ni * c + ch) * s + si;
    const float g = to_f(dy[off]);
    a += g;
    b += g * (to_f(x[off]) - mu);
  }
  a = block_sum(a, r1);
  b = block_sum(b, r2);
  if (threadIdx.x == 0) {
    ws[(int64_t)blockIdx.y * c + ch] = a;
    ws[(int64_t)gridDim.y * c + (int64_t)blockIdx.y * c + ch] = b;
  }
}

template <typename TW>
__global__ void reduce_finalize_kernel(const float* __restrict__ ws, int gy, int c, const float* __restrict__ inv_std,
                                       float* __restrict__ sum_dy, float* __restrict__ sum_dy_xmu, TW* __restrict__ gw,
                                       TW* __restrict__ gb) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  float a = 0.f, b = 0.f;
  for (int j = 0; j < gy; ++j) {
    a += ws[(int64_t)j * c + ch];
    b += ws[(int64_t)(gy + j) * c + ch];
  }
  sum_dy[ch] = a;
  sum_dy_xmu[ch] = b;
  if (gw) gw[ch] = from_f<TW>(b * inv_std[ch]);
  if (gb) gb[ch] = from_f<TW>(a);
}

// ---------------------------------------------------------------------------------------------
// backward apply
// ---------------------------------------------------------------------------------------------
template <typename T, typename TW, int VEC, bool CLAST>
__global__ void __launch_bounds__(256) bn_backward_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          BnParams p, FusedRelu r, const float* __restrict__ sum_dy,
                                                          const float* __restrict__ sum_dy_xmu,
                                                          const int* __restrict__ count, int world,
                                                          T* __restrict__ dx, int64_t total, int c, int64_t s) {
  __shared__ float inv_n_s;
  if (threadIdx.x == 0) {
    float n = 0.f;
    for (int w = 0; w < world; ++w) n += (float)count[w];
    inv_n_s = 1.f / n;
  }
  __syncthreads();
  const float inv_n = inv_n_s;
  const int64_t nvec = total / VEC;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * VEC;
    const int c0 = CLAST ? (int)(e % c) : (int)((e / s) % c);
    ChParams<TW, VEC, CLAST> q;
    q.load(p, c0);
    float v[VEC], g[VEC];
    load_vec<T, VEC>(v, x + e);
    load_vec<T, VEC>(g, dy + e);
    relu_mask<T, VEC>(g, v, q, r, e);
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const int ch = CLAST ? c0 + k : c0;
      const float mdy = sum_dy[ch] * inv_n;
      const float mdyx = sum_dy_xmu[ch] * inv_n;
      const float xmu = v[k] - q.mean[k];
      v[k] = (g[k] - mdy - xmu * q.istd[k] * q.istd[k] * mdyx) * q.istd[k] * q.w[k];
    }
    store_vec<T, VEC>(dx + e, v);
  }
}

// ---------------------------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------------------------
static bool al16(const void* p) { return p == nullptr || ((uintptr_t)p & 15u) == 0; }

inline bool use_vec8(const BnShape& sh, std::initializer_list<const void*> ptrs) {
  const int64_t inner = sh.c_last ? sh.c : sh.s;
  if (inner % 8 != 0) return false;
  for (const void* p : ptrs)
    if (!al16(p)) return false;
  return true;
}

inline unsigned ew_grid(int64_t nvec, int cus) {
  int64_t g = (nvec + 255) / 256;
  const int64_t cap = (int64_t)cus * 8;
  if (g > cap) g = cap;
  return (unsigned)(g < 1 ? 1 : g);
}

template <typename F>
inline void dispatch_xw(int x_t, int w_t, F&& f) {
  dispatch_float(x_t, [&](auto tx) {
    dispatch_float(w_t < 0 ? kF32 : w_t, [&](auto tw) { f(tx, tw); }, "batchnorm weight");
  }, "batchnorm input");
}

}  // namespace bn

int64_t bn_workspace_floats(const BnShape& sh, int cus) {
  if (sh.c_last) {
    const bn::Tiling t = bn::clast_tiling(sh.n, sh.c, true, cus);
    const bn::Tiling t1 = bn::clast_tiling(sh.n, sh.c, false, cus);
    const int gy = t.gy > t1.gy ? t.gy : t1.gy;
    return 2 * (int64_t)gy * sh.c + gy;
  }
  const int p = bn::nchw_parts(sh.n, sh.s, sh.c, cus);
  return 2 * (int64_t)p * sh.c + (int64_t)p * sh.c;
}

void bn_welford(const void* x, int x_t, const BnShape& sh, float* mean, float* var_biased, float* ws, int cus,
                hipStream_t s) {
  if (sh.c <= 0) return;
  dispatch_float(x_t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (sh.c_last) {
      const bool v8 = bn::use_vec8(sh, {x});
      const bn::Tiling t = bn::clast_tiling(sh.n, sh.c, v8, cus);
      const size_t lds = ((t.vec == 8 ? ColSum<8>::lds_floats(t.tx, t.ty, 2) : ColSum<1>::lds_floats(t.tx, t.ty, 2)) + t.ty) * sizeof(float);
      if (v8)
        hipLaunchKernelGGL((bn::welford_clast_kernel<T, 8>), dim3(t.gx, t.gy), dim3(t.tx, t.ty), lds, s, (const T*)x,
                           sh.n, sh.c, ws);
      else
        hipLaunchKernelGGL((bn::welford_clast_kernel<T, 1>), dim3(t.gx, t.gy), dim3(t.tx, t.ty), lds, s, (const T*)x,
                           sh.n, sh.c, ws);
      hipLaunchKernelGGL(bn::welford_finalize_kernel, dim3((sh.c + 255) / 256), dim3(256), 0, s, ws, t.gy, sh.c, 0, mean,
                         var_biased);
    } else {
      const int p = bn::nchw_parts(sh.n, sh.s, sh.c, cus);
      hipLaunchKernelGGL((bn::welford_nchw_kernel<T>), dim3(sh.c, p), dim3(256), 0, s, (const T*)x, sh.n, sh.c, sh.s,
                         ws);
      hipLaunchKernelGGL(bn::welford_finalize_kernel, dim3((sh.c + 255) / 256), dim3(256), 0, s, ws, p, sh.c, 1, mean,
                         var_biased);
    }
  }, "batchnorm welford");
  check_launch("bn_welford");
}

void bn_welford_parallel(const float* mean_all, const float* var_all, const int* count_all, int world, int c,
                         float eps, float* mean, float* var_unbiased, float* inv_std, hipStream_t s) {
  if (c <= 0) return;
  hipLaunchKernelGGL(bn::welford_parallel_kernel, dim3((c + 255) / 256), dim3(256), 0, s, mean_all, var_all, count_all,
                     world, c, eps, mean, var_unbiased, inv_std);
  check_launch("bn_welford_parallel");
}

void bn_forward(const void* x, int x_t, const BnParams& p, const FusedRelu& r, void* y, const BnShape& sh, int cus,
                hipStream_t s) {
  const int64_t total = sh.n * sh.c * sh.s;
  if (total <= 0) return;
  bn::dispatch_xw(x_t, p.w_t, [&](auto tx, auto tw) {
    using T = typename decltype(tx)::type;
    using TW = typename decltype(tw)::type;
    const bool v8 = bn::use_vec8(sh, {x, y, r.z});
    const int vec = v8 ? 8 : 1;
    const unsigned g = bn::ew_grid(total / vec, cus);
    if (sh.c_last) {
      if (v8) hipLaunchKernelGGL((bn::bn_forward_kernel<T, TW, 8, true>), dim3(g), dim3(256), 0, s, (const T*)x, p, r, (T*)y, total, sh.c, sh.s);
      else hipLaunchKernelGGL((bn::bn_forward_kernel<T, TW, 1, true>), dim3(g), dim3(256), 0, s, (const T*)x, p, r, (T*)y, total, sh.c, sh.s);
    } else {
      if (v8) hipLaunchKernelGGL((bn::bn_forward_kernel<T, TW, 8, false>), dim3(g), dim3(256), 0, s, (const T*)x, p, r, (T*)y, total, sh.c, sh.s);
      else hipLaunchKernelGGL((bn::bn_forward_kernel<T, TW, 1, false>), dim3(g), dim3(256), 0, s, (const T*)x, p, r, (T*)y, total, sh.c, sh.s);
    }
  });
  check_launch("bn_forward");
}

void bn_relu_backward(const void* dy, const void* x, int x_t, const BnParams& p, const FusedRelu& r, void* dy_out,
                      const BnShape& sh, int cus, hipStream_t s) {
  const int64_t total = sh.n * sh.c * sh.s;
  if (total <= 0) return;
  bn::dispatch_xw(x_t, p.w_t, [&](auto tx, auto tw) {
    using T = typename decltype(tx)::type;
    using TW = typename decltype(tw)::type;
    const bool v8 = bn::use_vec8(sh, {x, dy, dy_out, r.z});
    const unsigned g = bn::ew_grid(total / (v8 ? 8 : 1), cus);
    if (v8) hipLaunchKernelGGL((bn::bn_relu_bw_kernel<T, TW, 8>), dim3(g), dim3(256), 0, s, (const T*)dy, (const T*)x, p, r, (T*)dy_out, total, sh.c);
    else hipLaunchKernelGGL((bn::bn_relu_bw_kernel<T, TW, 1>), dim3(g), dim3(256), 0, s, (const T*)dy, (const T*)x, p, r, (T*)dy_out, total, sh.c);
  });
  check_launch("bn_relu_backward");
}

void bn_reduce(const void* dy, const void* x, int x_t, const BnParams& p, const FusedRelu& r, float* sum_dy,
               float* sum_dy_xmu, void* grad_w, void* grad_b, const BnShape& sh, float* ws, int cus, hipStream_t s) {
  if (sh.c <= 0) return;
  bn::dispatch_xw(x_t, p.w_t, [&](auto tx, auto tw) {
    using T = typename decltype(tx)::type;
    using TW = typename decltype(tw)::type;
    int gy;
    if (sh.c_last) {
      const bool v8 = bn::use_vec8(sh, {x, dy, r.z});
      const bn::Tiling t = bn::clast_tiling(sh.n, sh.c, v8, cus);
      const size_t lds = (t.vec == 8 ? ColSum<8>::lds_floats(t.tx, t.ty, 2) : ColSum<1>::lds_floats(t.tx, t.ty, 2)) * sizeof(float);
      if (v8)
        hipLaunchKernelGGL((bn::reduce_clast_kernel<T, TW, 8>), dim3(t.gx, t.gy), dim3(t.tx, t.ty), lds, s,
                           (const T*)dy, (const T*)x, p, r, sh.n, sh.c, ws);
      else
        hipLaunchKernelGGL((bn::reduce_clast_kernel<T, TW, 1>), dim3(t.gx, t.gy), dim3(t.tx, t.ty), lds, s,
                           (const T*)dy, (const T*)x, p, r, sh.n, sh.c, ws);
      gy = t.gy;
    } else {
      gy = bn::nchw_parts(sh.n, sh.s, sh.c, cus);
      hipLaunchKernelGGL((bn::reduce_nchw_kernel<T>), dim3(sh.c, gy), dim3(256), 0, s, (const T*)dy, (const T*)x, p.mean,
                         sh.n, sh.c, sh.s, ws);
    }
    hipLaunchKernelGGL((bn::reduce_finalize_kernel<TW>), dim3((sh.c + 255) / 256), dim3(256), 0, s, ws, gy, sh.c,
                       p.inv_std, sum_dy, sum_dy_xmu, (TW*)grad_w, (TW*)grad_b);
  });
  check_launch("bn_reduce");
}

void bn_backward(const void* dy, const void* x, int x_t, const BnParams& p, const FusedRelu& r, const float* sum_dy,
                 const float* sum_dy_xmu, const int* count, int world, void* dx, const BnShape& sh, int cus,
                 hipStream_t s) {
  const int64_t total = sh.n * sh.c * sh.s;
  if (total <= 0) return;
  bn::dispatch_xw(x_t, p.w_t, [&](auto tx, auto tw) {
    using T = typename decltype(tx)::type;
    using TW = typename decltype(tw)::type;
    const bool v8 = bn::use_vec8(sh, {x, dy, dx, r.z});
    const unsigned g = bn::ew_grid(total / (v8 ? 8 : 1), cus);
    if (sh.c_last) {
      if (v8) hipLaunchKernelGGL((bn::bn_backward_kernel<T, TW, 8, true>), dim3(g), dim3(256), 0, s, (const T*)dy, (const T*)x, p, r, sum_dy, sum_dy_xmu, count, world, (T*)dx, total, sh.c, sh.s);
      else hipLaunchKernelGGL((bn::bn_backward_kernel<T, TW, 1, true>), dim3(g), dim3(256), 0, s, (const T*)dy, (const T*)x, p, r, sum_dy, sum_dy_xmu, count, world, (T*)dx, total, sh.c, sh.s);
    } else {
      if (v8) hipLaunchKernelGGL((bn::bn_backward_kernel<T, TW, 8, false>), dim3(g), dim3(256), 0, s, (const T*)dy, (const T*)x, p, r, sum_dy, sum_dy_xmu, count, world, (T*)dx, total, sh.c, sh.s);
      else hipLaunchKernelGGL((bn::bn_backward_kernel<T, TW, 1, false>), dim3(g), dim3(256), 0, s, (const T*)dy, (const T*)x, p, r, sum_dy, sum_dy_xmu, count, world, (T*)dx, total, sh.c, sh.s);
    }
  });
  check_launch("bn_backward");
}

}  // namespace apex_amd
