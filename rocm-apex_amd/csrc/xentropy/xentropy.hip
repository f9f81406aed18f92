// Softmax cross-entropy with label smoothing (forward + backward) for gfx950.
//
// Reference: apex/contrib/csrc/xentropy/xentropy_kernel.cu:391 (forward: three passes over the
// row — max+sum, sum-exp, then the loss), :554 (backward), host :583-705.
//
// gfx950 design: one 256-thread block per row; the forward is a SINGLE pass — every lane keeps
// an online (max, sum-exp) pair plus the plain sum over 8-element vectors (16-byte loads), and
// the pairs are merged with wave64 shuffles then across the 4 waves in LDS.  Vocabulary-sized
// rows (30k-50k classes) are therefore read from HBM exactly once in forward and once in
// backward.  Losses and the saved log-sum-exp are fp32.
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"

namespace apex_amd {
namespace xent {

constexpr int kThreads = 256;

__device__ __forceinline__ void merge_ms(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) {
    m = m2;
    s = s2;
    return;
  }
  if (m2 > m) {
    s = s * __expf(m - m2) + s2;
    m = m2;
  } else {
    s += s2 * __expf(m2 - m);
  }
}

template <int N>
__device__ __forceinline__ void accum(float& m, float& s, float& sum, const float (&v)[N]) {
  float lm = v[0];
#pragma unroll
  for (int k = 1; k < N; ++k) lm = fmaxf(lm, v[k]);
  float ls = 0.f;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    ls += __expf(v[k] - lm);
    sum += v[k];
  }
  merge_ms(m, s, lm, ls);
}

template <typename T, bool VEC>
__global__ void __launch_bounds__(kThreads)
xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels, float* __restrict__ losses,
                float* __restrict__ lse_out, int classes, float smoothing, int64_t padding_idx, bool use_pad) {
  __shared__ float red[3][kThreads / 64];
  const int64_t row = blockIdx.x;
  const T* x = logits + row * classes;
  float m = -INFINITY, s = 0.f, sum = 0.f;
  if (VEC) {
    const int nv = classes >> 3;
    for (int v = threadIdx.x; v < nv; v += kThreads) {
      float r[8];
      Vec8<T>::load(r, x + v * 8);
      accum<8>(m, s, sum, r);
    }
  } else {
    for (int c = threadIdx.x; c < classes; c += kThreads) {
      float r[1] = {to_f(x[c])};
      accum<1>(m, s, sum, r);
    }
  }
  // wave merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    sum += __shfl_xor(sum, o, 64);
    merge_ms(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wid] = m;
    red[1][wid] = s;
    red[2][wid] = sum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red[0][0], S = red[1][0], SUM = red[2][0];
    for (int w = 1; w < kThreads / 64; ++w) {
      merge_ms(M, S, red[0][w], red[1][w]);
      SUM += red[2][w];
    }
    const float lse = M + __logf(S);
    const int64_t lab = labels[row];
    float loss = 0.f;
    if (!(use_pad && lab == padding_idx) && lab >= 0 && lab < classes) {
      const float log_prob = to_f(x[lab]) - lse;
      loss = (lse - SUM / (float)classes) * smoothing - log_prob * (1.f - smoothing);
    }
    losses[row] = loss;
    lse_out[row] = lse;
  }
}

template <typename T, bool VEC>
__global__ void __launch_bounds__(kThreads)
xent_bwd_kernel(const float* __restrict__ grad_loss, const T* __restrict__ logits, const float* __restrict__ lse,
                const int64_t* __restrict__ labels, T* __restrict__ grad, int classes, float smoothing,
                int64_t padding_idx, bool use_pad) {
  const int64_t row = blockIdx.x;
  const int64_t lab = labels[row];
  const float g = (use_pad && lab == padding_idx) ? 0.f : grad_loss[row];
  const float c = lse[row];
  const float pos = 1.f - smoothing, neg = smoothing / (float)classes;
  const T* x = logits + row * classes;
  T* gx = grad + row * classes;
  if (VEC) {
    const int nv = classes >> 3;
    for (int v = threadIdx.x; v < nv; v += kThreads) {
      float r[8];
      Vec8<T>::load(r, x + v * 8);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int cls = v * 8 + k;
        r[k] = g * (__expf(r[k] - c) - (cls == lab ? pos : 0.f) - neg);
      }
      Vec8<T>::store(gx + v * 8, r);
    }
  } else {
    for (int cls = threadIdx.x; cls < classes; cls += kThreads)
      gx[cls] = from_f<T>(g * (__expf(to_f(x[cls]) - c) - (cls == lab ? pos : 0.f) - neg));
  }
}

}  // namespace xent

void xentropy_fwd(const void* logits, int dt, const int64_t* labels, float* losses, float* lse, int64_t rows,
                  int classes, float smoothing, int64_t padding_idx, bool use_pad, hipStream_t s) {
  if (rows <= 0) return;
  dispatch_float(dt, [&](auto tag) {
    using T = typename decltype(tag)::type;
    const bool vec = (classes % 8 == 0) && (((uintptr_t)logits & 15u) == 0);
    if (vec)
      hipLaunchKernelGGL((xent::xent_fwd_kernel<T, true>), dim3((unsigned)rows), dim3(xent::kThreads), 0, s,
                         (const T*)logits, labels, losses, lse, classes, smoothing, padding_idx, use_pad);
    else
      hipLaunchKernelGGL((xent::xent_fwd_kernel<T, false>), dim3((unsigned)rows), dim3(xent::kThreads), 0, s,
                         (const T*)logits, labels, losses, lse, classes, smoothing, padding_idx, use_pad);
  }, "xentropy forward");
  check_launch("xentropy forward");
}

void xentropy_bwd(const float* grad_loss, const void* logits, int dt, const float* lse, const int64_t* labels,
                  void* grad, int64_t rows, int classes, float smoothing, int64_t padding_idx, bool use_pad,
                  hipStream_t s) {
  if (rows <= 0) return;
  dispatch_float(dt, [&](auto tag) {
    using T = typename decltype(tag)::type;
    const bool vec = (classes % 8 == 0) && (((uintptr_t)logits & 15u) == 0) && (((uintptr_t)grad & 15u) == 0);
    if (vec)
      hipLaunchKernelGGL((xent::xent_bwd_kernel<T, true>), dim3((unsigned)rows), dim3(xent::kThreads), 0, s,
                         grad_loss, (const T*)logits, lse, labels, (T*)grad, classes, smoothing, padding_idx, use_pad);
    else
      hipLaunchKernelGGL((xent::xent_bwd_kernel<T, false>), dim3((unsigned)rows), dim3(xent::kThreads), 0, s,
                         grad_loss, (const T*)logits, lse, labels, (T*)grad, classes, smoothing, padding_idx, use_pad);
  }, "xentropy backward");
  check_launch("xentropy backward");
}

}  // namespace apex_amd
