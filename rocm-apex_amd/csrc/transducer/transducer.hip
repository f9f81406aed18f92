// RNN-T (transducer) joint and loss kernels for gfx950.
//
// Reference: apex/contrib/csrc/transducer/transducer_joint_kernel.cu (joint f[b,t] + g[b,u] with
// optional ReLU / dropout and packed output; backward = sums over u / t) and
// transducer_loss_kernel.cu (alpha / beta forward-backward over the (t, u) lattice in log space,
// gradient fused with the log-softmax backward).  Both are warp-(32)-shaped there; here:
//  * joint forward: one workgroup per (b, t) row streams all (u, h) with 16-byte vectors — the
//    f row stays in L1/L2 while every g row is read once per t (g is small).
//  * joint backward: per (b, t) / (b, u) column sums with (hvec, part) thread tiles and a
//    fixed-order LDS reduction (deterministic, no atomics).
//  * loss alpha / beta: one workgroup per (batch, direction) walks the anti-diagonals of the
//    lattice (t + u = n), all u of a diagonal in parallel, fp32 logsumexp.
//  * loss backward: one workgroup per (b, t, u) row of the vocabulary, gradient of the loss wrt
//    the logits with the softmax backward fused (or wrt log-probs when not fused).
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/transducer_api.h"

namespace apex_amd {
namespace rnnt {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

struct JointGeo {
  int64_t out_row;  // element offset of (b, t, u=0, h=0) in the output
  int64_t stride_u; // elements between consecutive u
};

__device__ __forceinline__ JointGeo joint_geo(const JointArgs& a, int b, int t) {
  JointGeo g;
  g.stride_u = a.H;
  if (a.packed) {
    const int64_t base = b == 0 ? 0 : a.batch_offset[b - 1];
    g.out_row = (base + (int64_t)t * a.g_len[b]) * a.H;
  } else {
    g.out_row = (((int64_t)b * a.T + t) * a.U) * a.H;
  }
  return g;
}

template <typename T, bool RELU, bool DROP>
__global__ void __launch_bounds__(256) joint_fwd_kernel(const JointArgs a) {
  const int t = blockIdx.x, b = blockIdx.y;
  const int fl = a.f_len[b], gl = a.g_len[b];
  if (a.packed && t >= fl) return;
  const JointGeo geo = joint_geo(a, b, t);
  const T* f = (const T*)a.f + ((int64_t)b * a.T + t) * a.H;
  const T* g = (const T*)a.g + (int64_t)b * a.U * a.H;
  T* out = (T*)a.out + geo.out_row;
  uint8_t* mask = a.mask ? a.mask + geo.out_row : nullptr;
  const int urange = a.packed ? gl : a.U;
  const uint32_t thresh = (uint32_t)fminf(a.p_drop * 4294967296.f, 4294967295.f);
  const float scale = (DROP && a.p_drop < 1.f) ? 1.f / (1.f - a.p_drop) : 1.f;
  const uint32_t smix = mix32((uint32_t)a.seed ^ mix32((uint32_t)a.offset + 0x9E3779B9u));
  if ((a.H & 7) == 0) {
    const int hv = a.H / 8;
    for (int i = threadIdx.x; i < urange * hv; i += blockDim.x) {
      const int u = i / hv, h = (i % hv) * 8;
      float r[8];
      uint8_t mk[8];
      const bool valid = t < fl && u < gl;
      if (valid) {
        float fv[8], gv[8];
        Vec8<T>::load(fv, f + h);
        Vec8<T>::load(gv, g + (int64_t)u * a.H + h);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float v = fv[e] + gv[e];
          bool keep = true;
          if (RELU) keep = v > 0.f;
          if (DROP) {
            const uint32_t idx = (uint32_t)(geo.out_row + (int64_t)u * a.H + h + e);
            const bool dk = mix32(smix ^ (idx * 0x85EBCA6Bu)) >= thresh;
            keep = keep && dk;
            v *= scale;
          }
          r[e] = keep ? v : 0.f;
          mk[e] = keep;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          r[e] = -1.f;  // finite don't-care fill (reference transducer_joint_kernel.cu:205-214)
          mk[e] = 0;
        }
      }
      Vec8<T>::store(out + (int64_t)u * a.H + h, r);
      if (mask != nullptr) {
        uint2 w;
        w.x = mk[0] | (mk[1] << 8) | (mk[2] << 16) | ((uint32_t)mk[3] << 24);
        w.y = mk[4] | (mk[5] << 8) | (mk[6] << 16) | ((uint32_t)mk[7] << 24);
        *reinterpret_cast<uint2*>(mask + (int64_t)u * a.H + h) = w;
      }
    }
  } else {
    for (int i = threadIdx.x; i < urange * a.H; i += blockDim.x) {
      const int u = i / a.H, h = i % a.H;
      float v = -1.f;
      uint8_t keep = 0;
      if (t < fl && u < gl) {
        v = to_f(f[h]) + to_f(g[(int64_t)u * a.H + h]);
        bool k = true;
        if (RELU) k = v > 0.f;
        if (DROP) {
          const uint32_t idx = (uint32_t)(geo.out_row + (int64_t)u * a.H + h);
          k = k && (mix32(smix ^ (idx * 0x85EBCA6Bu)) >= thresh);
          v *= scale;
        }
        v = k ? v : 0.f;
        keep = k;
      }
      out[(int64_t)u * a.H + h] = from_f<T>(v);
      if (mask != nullptr) mask[(int64_t)u * a.H + h] = keep;
    }
  }
}

// Column sums of the joint gradient.  SUM_U: f_grad[b,t,:] = sum_{u<gl} grad[b,t,u,:];
// else g_grad[b,u,:] = sum_{t<fl} grad[b,t,u,:].  Masked (relu/dropout) grads use mask * scale.
template <typename T, bool SUM_U, bool MASKED>
__global__ void __launch_bounds__(256) joint_bwd_kernel(const JointArgs a, const T* __restrict__ grad,
                                                        T* __restrict__ out, float scale) {
  __shared__ float red[256 * 8];
  const int x = blockIdx.x, b = blockIdx.y;
  const int fl = a.f_len[b], gl = a.g_len[b];
  const int hv = (a.H + 7) / 8;
  const int cols = hv < 256 ? hv : 256;
  const int parts = 256 / cols;
  const int col = threadIdx.x % cols, part = threadIdx.x / cols;
  const bool vec = (a.H & 7) == 0;
  const int n = SUM_U ? gl : fl;              // summed extent
  const bool row_valid = SUM_U ? (x < fl) : (x < gl);
  T* dst = out + ((int64_t)b * (SUM_U ? a.T : a.U) + x) * a.H;
  for (int h0 = 0; h0 < hv; h0 += cols) {
    const int h = (h0 + col) * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (row_valid && part < parts && h0 + col < hv) {
      for (int j = part; j < n; j += parts) {
        const int t = SUM_U ? x : j, u = SUM_U ? j : x;
        const JointGeo geo = joint_geo(a, b, t);
        const int64_t off = geo.out_row + (int64_t)u * a.H + h;
        float gv[8];
        if (vec) {
          Vec8<T>::load(gv, grad + off);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) gv[e] = (h + e < a.H) ? to_f(grad[off + e]) : 0.f;
        }
        if (MASKED) {
#pragma unroll
          for (int e = 0; e < 8; ++e) gv[e] *= (h + e < a.H && a.mask[off + e]) ? scale : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += gv[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = acc[e];
    __syncthreads();
    if (part == 0 && h0 + col < hv) {
      float s[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] = 0.f;
      for (int p = 0; p < parts; ++p)
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += red[(p * cols + col) * 8 + e];
      if (vec) {
        Vec8<T>::store(dst + h, s);
      } else {
        for (int e = 0; e < 8 && h + e < a.H; ++e) dst[h + e] = from_f<T>(s[e]);
      }
    }
    __syncthreads();
  }
}

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  return m + logf(expf(a - m) + expf(b - m));
}

struct LossGeo {
  int64_t base;  // row (t=0, u=0) of batch b in x (in vocabulary rows)
  int64_t st;    // rows between consecutive t
};
__device__ __forceinline__ LossGeo loss_geo(const LossArgs& a, int b) {
  LossGeo g;
  const int gl = a.y_len[b] + 1;
  if (a.packed) {
    g.base = b == 0 ? 0 : a.batch_offset[b - 1];
    g.st = gl;
  } else {
    g.base = (int64_t)b * a.T * a.U;
    g.st = a.U;
  }
  return g;
}

// blockIdx.x: 0 = alpha, 1 = beta; blockIdx.y = batch
template <typename T>
__global__ void __launch_bounds__(1024) loss_fwd_kernel(const LossArgs a) {
  const int b = blockIdx.y;
  const int fl = a.f_len[b], gl = a.y_len[b] + 1;
  const LossGeo geo = loss_geo(a, b);
  const T* x = (const T*)a.x;
  const int* lab = a.label + (int64_t)b * (a.U - 1);
  const int64_t V = a.V;
  auto X = [&](int t, int u, int v) { return to_f(x[(geo.base + (int64_t)t * geo.st + u) * V + v]); };
  float* al = a.alpha + (int64_t)b * a.T * a.U;
  float* be = a.beta + (int64_t)b * a.T * a.U;
  if (fl <= 0) {
    if (blockIdx.x == 1 && threadIdx.x == 0) a.loss[b] = 0.f;
    return;
  }
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) al[0] = 0.f;
    __syncthreads();
    for (int n = 1; n < fl + gl - 1; ++n) {
      for (int u = threadIdx.x; u < gl; u += blockDim.x) {
        const int t = n - u;
        if (t < 0 || t >= fl) continue;
        float v;
        if (u == 0) v = al[(t - 1) * a.U] + X(t - 1, 0, a.blank);
        else if (t == 0) v = al[u - 1] + X(0, u - 1, lab[u - 1]);
        else
          v = lse2(al[(t - 1) * a.U + u] + X(t - 1, u, a.blank), al[t * a.U + u - 1] + X(t, u - 1, lab[u - 1]));
        al[t * a.U + u] = v;
      }
      __syncthreads();
    }
  } else {
    if (threadIdx.x == 0) be[(fl - 1) * a.U + gl - 1] = X(fl - 1, gl - 1, a.blank);
    __syncthreads();
    for (int n = fl + gl - 3; n >= 0; --n) {
      for (int u = threadIdx.x; u < gl; u += blockDim.x) {
        const int t = n - u;
        if (t < 0 || t >= fl) continue;
        float v;
        if (u == gl - 1) v = be[(t + 1) * a.U + u] + X(t, u, a.blank);
        else if (t == fl - 1) v = be[t * a.U + u + 1] + X(t, u, lab[u]);
        else v = lse2(be[(t + 1) * a.U + u] + X(t, u, a.blank), be[t * a.U + u + 1] + X(t, u, lab[u]));
        be[t * a.U + u] = v;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) a.loss[b] = -be[0];
  }
}

// one workgroup per (u, t, b) vocabulary row
template <typename T, bool FUSED>
__global__ void __launch_bounds__(256) loss_bwd_kernel(const LossArgs a, const float* __restrict__ loss_grad,
                                                       T* __restrict__ xg) {
  const int u = blockIdx.x, t = blockIdx.y, b = blockIdx.z;
  const int fl = a.f_len[b], gl = a.y_len[b] + 1;
  const LossGeo geo = loss_geo(a, b);
  const int64_t V = a.V;
  if (a.packed && (t >= fl || u >= gl)) return;
  T* g = xg + (geo.base + (int64_t)t * geo.st + u) * V;
  if (t >= fl || u >= gl) {
    for (int64_t v = threadIdx.x; v < V; v += blockDim.x) g[v] = from_f<T>(0.f);
    return;
  }
  const T* x = (const T*)a.x + (geo.base + (int64_t)t * geo.st + u) * V;
  const float* al = a.alpha + (int64_t)b * a.T * a.U;
  const float* be = a.beta + (int64_t)b * a.T * a.U;
  const float common = logf(loss_grad[b]) + al[t * a.U + u] - be[0];
  const float b_tu = be[t * a.U + u];
  const float b_tu1 = (u + 1 < gl) ? be[t * a.U + u + 1] : 0.f;
  const float b_t1u = (t + 1 < fl) ? be[(t + 1) * a.U + u] : 0.f;
  const int lab = (u < gl - 1) ? a.label[(int64_t)b * (a.U - 1) + u] : -1;
  for (int64_t v = threadIdx.x; v < V; v += blockDim.x) {
    const float gr = common + to_f(x[v]);
    float r = FUSED ? expf(gr + b_tu) : 0.f;
    if (v == lab) r -= expf(gr + b_tu1);
    else if (v == a.blank) {
      if (t == fl - 1 && u == gl - 1) r -= expf(gr);
      else if (t != fl - 1) r -= expf(gr + b_t1u);
    }
    g[v] = from_f<T>(r);
  }
}

}  // namespace rnnt

void transducer_joint_fwd(const JointArgs& a, hipStream_t s) {
  dispatch_float(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    const dim3 grid(a.T, a.B);
    if (a.relu && a.dropout) hipLaunchKernelGGL((rnnt::joint_fwd_kernel<T, true, true>), grid, dim3(256), 0, s, a);
    else if (a.relu) hipLaunchKernelGGL((rnnt::joint_fwd_kernel<T, true, false>), grid, dim3(256), 0, s, a);
    else if (a.dropout) hipLaunchKernelGGL((rnnt::joint_fwd_kernel<T, false, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((rnnt::joint_fwd_kernel<T, false, false>), grid, dim3(256), 0, s, a);
  }, "transducer_joint_fwd");
  check_launch("transducer_joint_fwd");
}

void transducer_joint_bwd(const JointArgs& a, const void* grad, void* f_grad, void* g_grad, float scale,
                          hipStream_t s) {
  dispatch_float(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    const T* gr = (const T*)grad;
    if (a.mask != nullptr) {
      hipLaunchKernelGGL((rnnt::joint_bwd_kernel<T, true, true>), dim3(a.T, a.B), dim3(256), 0, s, a, gr, (T*)f_grad,
                         scale);
      hipLaunchKernelGGL((rnnt::joint_bwd_kernel<T, false, true>), dim3(a.U, a.B), dim3(256), 0, s, a, gr, (T*)g_grad,
                         scale);
    } else {
      hipLaunchKernelGGL((rnnt::joint_bwd_kernel<T, true, false>), dim3(a.T, a.B), dim3(256), 0, s, a, gr,
                         (T*)f_grad, scale);
      hipLaunchKernelGGL((rnnt::joint_bwd_kernel<T, false, false>), dim3(a.U, a.B), dim3(256), 0, s, a, gr,
                         (T*)g_grad, scale);
    }
  }, "transducer_joint_bwd");
  check_launch("transducer_joint_bwd");
}

void transducer_loss_fwd(const LossArgs& a, hipStream_t s) {
  dispatch_float(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    int threads = 64;
    while (threads < a.U && threads < 1024) threads *= 2;
    hipLaunchKernelGGL((rnnt::loss_fwd_kernel<T>), dim3(2, a.B), dim3(threads), 0, s, a);
  }, "transducer_loss_fwd");
  check_launch("transducer_loss_fwd");
}

void transducer_loss_bwd(const LossArgs& a, const float* loss_grad, void* x_grad, bool fused, hipStream_t s) {
  dispatch_float(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    const dim3 grid(a.U, a.T, a.B);
    if (fused) hipLaunchKernelGGL((rnnt::loss_bwd_kernel<T, true>), grid, dim3(256), 0, s, a, loss_grad, (T*)x_grad);
    else hipLaunchKernelGGL((rnnt::loss_bwd_kernel<T, false>), grid, dim3(256), 0, s, a, loss_grad, (T*)x_grad);
  }, "transducer_loss_bwd");
  check_launch("transducer_loss_bwd");
}

}  // namespace apex_amd
