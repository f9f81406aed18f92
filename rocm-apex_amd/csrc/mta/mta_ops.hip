// Multi-tensor elementwise + reduction ops for gfx950 (the amp_C family).
//
// Reference semantics (what each op computes) come from the reference's csrc/multi_tensor_*.cu;
// the execution model is our own: one persistent launch per op over a cached device work table
// (mta.h), 8 elements per lane per step, reductions finalized in-launch by the last block.
#include <cstring>

#include "apex_amd/mta_api.h"

#include <type_traits>
#include "apex_amd/dispatch.h"

namespace apex_amd {

// =============================================================================================
// table upload without host staging memory: the bytes travel as kernel arguments, so building a
// work table is capturable in a hipGraph (no pinned-allocator events, no memcpy node)
// =============================================================================================
constexpr int kUploadChunk = 2048;
struct UploadPayload {
  uint32_t w[kUploadChunk / 4];
};

__global__ void __launch_bounds__(256) mta_upload_kernel(uint32_t* __restrict__ dst, int nwords, UploadPayload p) {
  for (int i = threadIdx.x; i < nwords; i += 256) dst[i] = p.w[i];
}

void mta_upload_bytes(void* dst, const void* src, size_t bytes, hipStream_t s) {
  // tables are 8-byte aligned and sized in 8-byte units
  const uint8_t* in = static_cast<const uint8_t*>(src);
  uint8_t* out = static_cast<uint8_t*>(dst);
  for (size_t off = 0; off < bytes; off += kUploadChunk) {
    const size_t n = bytes - off < (size_t)kUploadChunk ? bytes - off : (size_t)kUploadChunk;
    UploadPayload p;
    std::memcpy(p.w, in + off, n);
    hipLaunchKernelGGL(mta_upload_kernel, dim3(1), dim3(256), 0, s, reinterpret_cast<uint32_t*>(out + off),
                       (int)((n + 3) / 4), p);
  }
  check_launch("mta_upload");
}

// =============================================================================================
// scale / axpby / check_finite
// =============================================================================================
struct ScaleOp : MtaOpBase {
  static constexpr unsigned kRead = 0b01, kWrite = 0b10;
  static constexpr bool kSkipOnNoop = false;
  DevScalar scale;
  struct TS { float s; };
  __device__ __forceinline__ TS tensor_state(int) const { return {scale.get()}; }
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[2][N], const TS& ts, bool& bad, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      bad |= !is_finite(r[0][k]);
      r[1][k] = r[0][k] * ts.s;
    }
  }
};

void mt_scale(const MtaMeta& m, int in_t, int out_t, int* noop, DevScalar scale, const Launch& L) {
  ScaleOp op;
  op.scale = scale;
  const int grid = mta_grid_work(m, L.max_blocks);
  dispatch_float(in_t, [&](auto ti) {
    dispatch_float(out_t, [&](auto to) {
      using TI = typename decltype(ti)::type;
      using TO = typename decltype(to)::type;
      mta_elementwise_kernel<ScaleOp, TI, TO><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
    }, "multi_tensor_scale(out)");
  }, "multi_tensor_scale(in)");
  check_launch("multi_tensor_scale");
}

struct AxpbyOp : MtaOpBase {
  static constexpr unsigned kRead = 0b011, kWrite = 0b100;
  static constexpr bool kSkipOnNoop = false;
  float a, b;
  int check;  // -1 both, 0 x, 1 y
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[3][N], const TS&, bool& bad, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const float x = r[0][k], y = r[1][k];
      r[2][k] = a * x + b * y;
      if (check == -1) bad |= !(is_finite(x) && is_finite(y));
      else if (check == 0) bad |= !is_finite(x);
      else if (check == 1) bad |= !is_finite(y);
    }
  }
};

void mt_axpby(const MtaMeta& m, int x_t, int y_t, int out_t, int* noop, float a, float b, int arg_to_check,
              const Launch& L) {
  AxpbyOp op;
  op.a = a;
  op.b = b;
  op.check = arg_to_check;
  const int grid = mta_grid_work(m, L.max_blocks);
  dispatch_float(x_t, [&](auto tx) {
    dispatch_float(y_t, [&](auto ty) {
      dispatch_float(out_t, [&](auto to) {
        using TX = typename decltype(tx)::type;
        using TY = typename decltype(ty)::type;
        using TO = typename decltype(to)::type;
        mta_elementwise_kernel<AxpbyOp, TX, TY, TO><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
      }, "multi_tensor_axpby(out)");
    }, "multi_tensor_axpby(y)");
  }, "multi_tensor_axpby(x)");
  check_launch("multi_tensor_axpby");
}

struct CheckFiniteOp : MtaOpBase {
  static constexpr unsigned kRead = 0b1, kWrite = 0b0;
  static constexpr bool kSkipOnNoop = false;
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[1][N], const TS&, bool& bad, float*) const {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < N; ++k) s += r[0][k] * 0.f;  // NaN/inf propagate, finite -> 0
    bad |= (s != 0.f) | (s != s);
  }
};

void mt_check_finite(const MtaMeta& m, int t, int* noop, const Launch& L) {
  const int grid = mta_grid_work(m, L.max_blocks);
  dispatch_float(t, [&](auto tt) {
    using T = typename decltype(tt)::type;
    mta_elementwise_kernel<CheckFiniteOp, T><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, CheckFiniteOp{});
  }, "multi_tensor_check_finite");
  check_launch("multi_tensor_check_finite");
}

// =============================================================================================
// norms: l2 / max-abs, optional scaled copy-out, optional per-tensor EMA blend (NovoGrad)
// =============================================================================================
template <int D, bool SKIP>
struct NormOp {
  static constexpr int kNumAcc = 1;
  static constexpr bool kCheckPartial = true;
  __device__ __forceinline__ bool acc_is_max() const { return mode == 1; }
  static constexpr unsigned kRead = 0b01, kWrite = (D == 2) ? 0b10 : 0b0;
  static constexpr bool kSkipOnNoop = SKIP;
  int mode;  // 0 l2 (sum of squares), 1 max-abs
  DevScalar scale;
  float* total;
  float* per_tensor;
  bool blend;
  float alpha, beta;
  struct TS { float s; };
  __device__ __forceinline__ TS tensor_state(int) const { return {scale.get()}; }
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[D][N], const TS& ts, bool& bad, float* acc) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const float x = r[0][k];
      if (mode == 0) acc[0] += x * x;
      else {  // fmaxf drops NaN, so flag non-finite inputs directly
        acc[0] = fmaxf(acc[0], fabsf(x));
        bad |= !is_finite(x);
      }
      if constexpr (D == 2) r[1][k] = x * ts.s;
    }
  }
  __device__ void finalize(const MtaMeta& m, unsigned tag) const {
    __shared__ float red[kMtaBlock / 64];
    const bool is_max = mode == 1;
    float mine = 0.f;
    for (int t = threadIdx.x; t < m.ntensors; t += blockDim.x) {
      const float s = mta_tensor_reduce(m, 0, t, is_max, tag);
      mine = is_max ? fmaxf(mine, s) : mine + s;
      if (per_tensor) {
        if (blend) {
          const float old = per_tensor[t];
          per_tensor[t] = is_max ? alpha * old + beta * s : sqrtf(alpha * old * old + beta * s);
        } else {
          per_tensor[t] = is_max ? s : sqrtf(s);
        }
      }
    }
    const float tot = is_max ? block_max(mine, red) : block_sum(mine, red);
    if (threadIdx.x == 0 && total) *total = is_max ? tot : sqrtf(tot);
  }
  __device__ void finalize_skipped(const MtaMeta& m) const {
    if (threadIdx.x == 0 && total) *total = 0.f;
    if (per_tensor && !blend)
      for (int t = threadIdx.x; t < m.ntensors; t += blockDim.x) per_tensor[t] = 0.f;
  }
};

template <int D, bool SKIP>
static void launch_norm(const MtaMeta& m, int in_t, int out_t, int* noop, const NormOp<D, SKIP>& op, int grid,
                        hipStream_t s) {
  dispatch_float(in_t, [&](auto ti) {
    using TI = typename decltype(ti)::type;
    if constexpr (D == 2) {
      dispatch_float(out_t, [&](auto to) {
        using TO = typename decltype(to)::type;
        mta_elementwise_kernel<NormOp<D, SKIP>, TI, TO><<<grid, kMtaBlock, 0, s>>>(m, noop, op);
      }, "multi_tensor_l2norm_scale(out)");
    } else {
      mta_elementwise_kernel<NormOp<D, SKIP>, TI><<<grid, kMtaBlock, 0, s>>>(m, noop, op);
    }
  }, "multi_tensor_norm");
}

void mt_norm(const MtaMeta& m, int in_t, int out_t, int* noop, float* total, float* per_tensor, int mode,
             bool skip_on_noop, DevScalar scale, bool blend, float alpha, float beta, const Launch& L) {
  const int grid = mta_grid_work(m, L.max_blocks, false);
  auto fill = [&](auto& op) {
    op.mode = mode;
    op.scale = scale;
    op.total = total;
    op.per_tensor = per_tensor;
    op.blend = blend;
    op.alpha = alpha;
    op.beta = beta;
  };
  if (out_t >= 0) {
    if (skip_on_noop) { NormOp<2, true> op; fill(op); launch_norm(m, in_t, out_t, noop, op, grid, L.stream); }
    else { NormOp<2, false> op; fill(op); launch_norm(m, in_t, out_t, noop, op, grid, L.stream); }
  } else {
    if (skip_on_noop) { NormOp<1, true> op; fill(op); launch_norm(m, in_t, out_t, noop, op, grid, L.stream); }
    else { NormOp<1, false> op; fill(op); launch_norm(m, in_t, out_t, noop, op, grid, L.stream); }
  }
  check_launch("multi_tensor_norm");
}

// Optimizer math at the reference's precision: its multi-tensor and optimizer kernels are built
// with --use_fast_math (reference setup.py:167,210,352,375), i.e. approximate divide and sqrt.  Here
// that is one v_rcp_f32 / v_sqrt_f32 (1 ulp) instead of the ~10-instruction IEEE sequences, and a
// per-tensor divisor (bias correction) becomes a multiply by its reciprocal, computed once per chunk:
// Adam drops from ~60 to ~15 VALU ops per element, so its waves spend their time on memory.
// (APEX_MTA_IEEE=1: variant build with IEEE sqrt / divide, for the A/B in tools/mta_bench.py)
#if APEX_MTA_IEEE
__device__ __forceinline__ float fm_sqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ float fm_rcp(float x) { return 1.f / x; }
#else
__device__ __forceinline__ float fm_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float fm_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
#endif

// =============================================================================================
// Adam / AdamW (reference csrc/multi_tensor_adam.cu:24-127 for the math; op order kept so the
// python fallback and this kernel agree to rounding)
// =============================================================================================
template <int D, bool SKIP>
struct AdamOp : MtaOpBase {
  static constexpr unsigned kRead = 0b1111, kWrite = (D == 5) ? 0b11110 : 0b1110;
  static constexpr bool kSkipOnNoop = SKIP;
  AdamArgs a;
  struct TS { float lr, inv, rbc1, rbc2; };  // reciprocal bias corrections
  __device__ __forceinline__ TS tensor_state(int) const {
    TS s;
    s.lr = a.lr.get();
    s.inv = a.inv_scale.get();
    float bc1 = a.bc1, bc2 = a.bc2;
    if (a.step_dev && a.bias_correction) {
      const float st = *a.step_dev;
      bc1 = 1.f - powf(a.beta1, st);
      bc2 = 1.f - powf(a.beta2, st);
    }
    s.rbc1 = 1.f / bc1;
    s.rbc2 = 1.f / bc2;
    return s;
  }
  // the step's update m^/(sqrt(v^)+eps), shared with AdamUndoOp so the undo inverts it exactly
  static __device__ __forceinline__ float update(float mm, float vv, const TS& s, float eps) {
    return (mm * s.rbc1) * fm_rcp(fm_sqrt(vv * s.rbc2) + eps);
  }
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[D][N], const TS& s, bool&, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      float g = r[0][k] * s.inv;
      float p = r[1][k], mm = r[2][k], vv = r[3][k];
      if (a.mode == 0) {
        g = g + a.weight_decay * p;
        mm = a.beta1 * mm + (1.f - a.beta1) * g;
        vv = a.beta2 * vv + (1.f - a.beta2) * g * g;
        p = p - s.lr * update(mm, vv, s, a.eps);
      } else {
        mm = a.beta1 * mm + (1.f - a.beta1) * g;
        vv = a.beta2 * vv + (1.f - a.beta2) * g * g;
        p = p - s.lr * (update(mm, vv, s, a.eps) + a.weight_decay * p);
      }
      r[1][k] = p;
      r[2][k] = mm;
      r[3][k] = vv;
      if constexpr (D == 5) r[4][k] = p;
    }
  }
};

template <int D, bool SKIP>
static void launch_adam(const MtaMeta& m, int g_t, int p_t, int out_t, int* noop, const AdamArgs& a, int grid,
                        hipStream_t s) {
  AdamOp<D, SKIP> op;
  op.a = a;
  dispatch_float(g_t, [&](auto tg) {
    using TG = typename decltype(tg)::type;
    if constexpr (D == 5) {
      dispatch_model_out(out_t, [&](auto to) {
        using TO = typename decltype(to)::type;
        mta_elementwise_kernel<AdamOp<D, SKIP>, TG, float, float, float, TO><<<grid, kMtaBlock, 0, s>>>(m, noop, op);
      }, "multi_tensor_adam(model out)");
    } else {
      dispatch_float(p_t, [&](auto tp) {
        using TP = typename decltype(tp)::type;
        mta_elementwise_kernel<AdamOp<D, SKIP>, TG, TP, TP, TP><<<grid, kMtaBlock, 0, s>>>(m, noop, op);
      }, "multi_tensor_adam(param)");
    }
  }, "multi_tensor_adam(grad)");
}

void mt_adam(const MtaMeta& m, int g_t, int p_t, int out_t, int* noop, const AdamArgs& a, const Launch& L) {
  const int grid = mta_grid_work(m, L.max_blocks);
  if (m.depth == 5) {
    if (p_t != kF32) throw std::runtime_error("multi_tensor_adam: master params must be fp32 with a model copy");
    if (a.skip_on_noop) launch_adam<5, true>(m, g_t, p_t, out_t, noop, a, grid, L.stream);
    else launch_adam<5, false>(m, g_t, p_t, out_t, noop, a, grid, L.stream);
  } else {
    if (a.skip_on_noop) launch_adam<4, true>(m, g_t, p_t, out_t, noop, a, grid, L.stream);
    else launch_adam<4, false>(m, g_t, p_t, out_t, noop, a, grid, L.stream);
  }
  check_launch("multi_tensor_adam");
}

// ---------------------------------------------------------------------------------------------
// Adam undo (capability of the reference's maybe_adam_undo, apex/contrib/csrc/optimizers/
// fused_adam_cuda_kernel.cu:657): given the gradient g of the step just taken and the post-step
// p, m, v, recompute that step's update from (m, v) and invert it in place, so a step can be
// rolled back without keeping copies of the master / moment shards.  Exact for p up to fp32
// rounding; m and v are recovered up to the cancellation in (m - (1-b1) g) / b1 (v is clamped
// at 0).  Skipped entirely when *noop (the reverted step's skip flag) is set.
// ---------------------------------------------------------------------------------------------
template <int D>
struct AdamUndoOp : MtaOpBase {
  static constexpr unsigned kRead = 0b1111, kWrite = (D == 5) ? 0b11110 : 0b1110;
  static constexpr bool kSkipOnNoop = true;
  AdamArgs a;
  using TS = typename AdamOp<D, true>::TS;
  __device__ __forceinline__ TS tensor_state(int t) const {
    AdamOp<D, true> fwd;
    fwd.a = a;
    return fwd.tensor_state(t);
  }
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[D][N], const TS& s, bool&, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      float g = r[0][k] * s.inv;
      const float p = r[1][k], mm = r[2][k], vv = r[3][k];
      const float upd = AdamOp<D, true>::update(mm, vv, s, a.eps);
      float p0;
      if (a.mode == 0) {
        p0 = p + s.lr * upd;
        g = g + a.weight_decay * p0;
      } else {
        p0 = (p + s.lr * upd) / (1.f - s.lr * a.weight_decay);
      }
      r[1][k] = p0;
      r[2][k] = (mm - (1.f - a.beta1) * g) / a.beta1;
      r[3][k] = fmaxf((vv - (1.f - a.beta2) * g * g) / a.beta2, 0.f);
      if constexpr (D == 5) r[4][k] = p0;
    }
  }
};

void mt_adam_undo(const MtaMeta& m, int g_t, int out_t, int* noop, const AdamArgs& a, const Launch& L) {
  const int grid = mta_grid_work(m, L.max_blocks);
  dispatch_float(g_t, [&](auto tg) {
    using TG = typename decltype(tg)::type;
    if (m.depth == 5) {
      dispatch_model_out(out_t, [&](auto to) {
        using TO = typename decltype(to)::type;
        AdamUndoOp<5> op;
        op.a = a;
        mta_elementwise_kernel<AdamUndoOp<5>, TG, float, float, float, TO><<<grid, kMtaBlock, 0, L.stream>>>(m, noop,
                                                                                                           op);
      }, "multi_tensor_adam_undo(model out)");
    } else {
      AdamUndoOp<4> op;
      op.a = a;
      mta_elementwise_kernel<AdamUndoOp<4>, TG, float, float, float><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
    }
  }, "multi_tensor_adam_undo(grad)");
  check_launch("multi_tensor_adam_undo");
}

// =============================================================================================
// SGD with momentum (reference csrc/multi_tensor_sgd_kernel.cu:29-139)
// =============================================================================================
template <int D>
struct SgdOp : MtaOpBase {
  static constexpr unsigned kRead = 0b0111, kWrite = (D == 4) ? 0b1110 : 0b0110;
  static constexpr bool kSkipOnNoop = true;
  SgdArgs a;
  struct TS { float lr, scale; };
  __device__ __forceinline__ TS tensor_state(int) const { return {a.lr.get(), a.scale.get()}; }
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[D][N], const TS& s, bool&, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      float g = r[0][k] * s.scale;
      const float w = r[1][k];
      float mom = r[2][k];
      if (a.wd != 0.f && !a.wd_after_momentum) g += a.wd * w;
      if (a.momentum != 0.f) {
        if (!a.first_run) mom = mom * a.momentum + (1.f - a.dampening) * g;
        else mom = g;
        if (a.nesterov) g += a.momentum * mom;
        else g = mom;
      }
      if (a.wd != 0.f && a.wd_after_momentum) g += a.wd * w;
      const float nw = w + (-s.lr * g);
      r[1][k] = nw;
      r[2][k] = mom;
      if constexpr (D == 4) r[3][k] = nw;
    }
  }
};

void mt_sgd(const MtaMeta& m, int g_t, int w_t, int out_t, int* noop, const SgdArgs& a, const Launch& L) {
  const int grid = mta_grid_work(m, L.max_blocks);
  dispatch_float(g_t, [&](auto tg) {
    using TG = typename decltype(tg)::type;
    dispatch_float(w_t, [&](auto tw) {
      using TW = typename decltype(tw)::type;
      if (m.depth == 4) {
        SgdOp<4> op;
        op.a = a;
        dispatch_model_out(out_t, [&](auto to) {
          using TO = typename decltype(to)::type;
          mta_elementwise_kernel<SgdOp<4>, TG, TW, TW, TO><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
        }, "multi_tensor_sgd(model out)");
      } else {
        SgdOp<3> op;
        op.a = a;
        mta_elementwise_kernel<SgdOp<3>, TG, TW, TW><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
      }
    }, "multi_tensor_sgd(weight)");
  }, "multi_tensor_sgd(grad)");
  check_launch("multi_tensor_sgd");
}

// =============================================================================================
// Adagrad (reference csrc/multi_tensor_adagrad.cu:24-84)
// =============================================================================================
struct AdagradOp : MtaOpBase {
  static constexpr unsigned kRead = 0b111, kWrite = 0b110;
  static constexpr bool kSkipOnNoop = false;
  float lr, eps, wd;
  int mode;
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[3][N], const TS&, bool&, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      float g = r[0][k], p = r[1][k], h = r[2][k];
      if (mode == 0) {
        g = g + wd * p;
        h = h + g * g;
        p = p - lr * (g * fm_rcp(fm_sqrt(h) + eps));
      } else {
        h = h + g * g;
        p = p - lr * (g * fm_rcp(fm_sqrt(h) + eps) + wd * p);
      }
      r[1][k] = p;
      r[2][k] = h;
    }
  }
};

void mt_adagrad(const MtaMeta& m, int t, int* noop, float lr, float eps, int mode, float wd, const Launch& L) {
  AdagradOp op;
  op.lr = lr;
  op.eps = eps;
  op.wd = wd;
  op.mode = mode;
  const int grid = mta_grid_work(m, L.max_blocks);
  dispatch_float(t, [&](auto tt) {
    using T = typename decltype(tt)::type;
    mta_elementwise_kernel<AdagradOp, T, T, T><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
  }, "multi_tensor_adagrad");
  check_launch("multi_tensor_adagrad");
}

// =============================================================================================
// NovoGrad update (reference csrc/multi_tensor_novograd.cu:33-127); norms blended beforehand
// =============================================================================================
struct NovoOp : MtaOpBase {
  static constexpr unsigned kRead = 0b111, kWrite = 0b110;
  static constexpr bool kSkipOnNoop = false;
  NovoArgs a;
  struct TS { float gn; };
  __device__ __forceinline__ TS tensor_state(int t) const { return {a.grad_norms[t]}; }
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[3][N], const TS& s, bool&, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      float g = r[0][k], p = r[1][k], mm = r[2][k];
      if (a.mode == 0) {
        const float denom = s.gn / a.bc2 + a.eps;
        g = (g / denom) + (a.weight_decay * p);
        mm = a.beta1 * mm + a.beta3 * g;
        p = p - (a.lr * (mm / a.bc1));
      } else {
        mm = a.beta1 * mm + a.beta3 * g;
        const float denom = s.gn / a.bc2 + a.eps;
        p = p - (a.lr * (((mm / a.bc1) / denom) + (a.weight_decay * p)));
      }
      r[1][k] = p;
      r[2][k] = mm;
    }
  }
};

void mt_novograd(const MtaMeta& m, int t, int* noop, const NovoArgs& a, const Launch& L) {
  NovoOp op;
  op.a = a;
  const int grid = mta_grid_work(m, L.max_blocks);
  dispatch_float(t, [&](auto tt) {
    using T = typename decltype(tt)::type;
    mta_elementwise_kernel<NovoOp, T, T, T><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
  }, "multi_tensor_novograd");
  check_launch("multi_tensor_novograd");
}

// =============================================================================================
// LAMB. Stage 1 computes the Adam-style update (written into g) AND both per-tensor norms
// (||p||, ||update||) in the same pass — the reference needs two extra l2norm launches plus two
// cleanup launches for those (csrc/multi_tensor_lamb.cu:370,394).
// =============================================================================================
template <bool SKIP>
struct LambStage1Op {
  static constexpr int kNumAcc = 2;
  static constexpr bool kCheckPartial = false;
  __device__ __forceinline__ bool acc_is_max() const { return false; }
  static constexpr unsigned kRead = 0b1111, kWrite = 0b1101;
  static constexpr bool kSkipOnNoop = SKIP;
  LambArgs a;
  struct TS { float gscale, rbc1, rbc2; };  // inv_scale / clip and reciprocal bias corrections
  __device__ __forceinline__ TS tensor_state(int) const {
    TS s;
    const float gn = *a.global_grad_norm;
    const float mx = a.max_grad_norm.get();
    const float clip = (mx > 0.f && gn > mx) ? gn / mx : 1.f;
    s.gscale = a.inv_scale.get() / clip;
    float bc1 = a.bc1, bc2 = a.bc2;
    if (a.step_dev && a.bias_correction) {
      const float st = *a.step_dev;
      bc1 = 1.f - powf(a.beta1, st);
      bc2 = 1.f - powf(a.beta2, st);
    }
    s.rbc1 = 1.f / bc1;
    s.rbc2 = 1.f / bc2;
    return s;
  }
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[4][N], const TS& s, bool&, float* acc) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const float p = r[1][k];
      float mm = r[2][k], vv = r[3][k];
      float sg = r[0][k] * s.gscale;
      const float pd = a.weight_decay != 0.f ? p : 0.f;
      float upd;
      if (a.mode == 0) {
        sg = sg + a.weight_decay * pd;
        mm = mm * a.beta1 + a.beta3 * sg;
        vv = vv * a.beta2 + (1.f - a.beta2) * sg * sg;
        upd = (mm * s.rbc1) * fm_rcp(fm_sqrt(vv * s.rbc2) + a.eps);
      } else {
        mm = mm * a.beta1 + a.beta3 * sg;
        vv = vv * a.beta2 + (1.f - a.beta2) * sg * sg;
        upd = (mm * s.rbc1) * fm_rcp(fm_sqrt(vv * s.rbc2) + a.eps) + a.weight_decay * pd;
      }
      acc[0] += p * p;
      acc[1] += upd * upd;
      r[0][k] = upd;
      r[2][k] = mm;
      r[3][k] = vv;
    }
  }
  __device__ void finalize(const MtaMeta& m, unsigned tag) const {
    for (int t = threadIdx.x; t < m.ntensors; t += blockDim.x) {
      a.param_norm[t] = sqrtf(mta_tensor_reduce(m, 0, t, false, tag));
      a.update_norm[t] = sqrtf(mta_tensor_reduce(m, 1, t, false, tag));
    }
  }
  __device__ void finalize_skipped(const MtaMeta&) const {}
};

template <int D, bool SKIP>
struct LambStage2Op : MtaOpBase {
  static constexpr unsigned kRead = 0b011, kWrite = (D == 3) ? 0b110 : 0b010;
  static constexpr bool kSkipOnNoop = SKIP;
  LambArgs a;
  struct TS { float ratio; };
  __device__ __forceinline__ TS tensor_state(int t) const {
    const float lr = a.lr.get();
    float ratio = lr;
    if (a.use_nvlamb || a.weight_decay != 0.f) {
      const float pn = a.param_norm[t], un = a.update_norm[t];
      ratio = (un != 0.f && pn != 0.f) ? lr * (pn / un) : lr;
    }
    return {ratio};
  }
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[D][N], const TS& s, bool&, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const float p = r[1][k] - s.ratio * r[0][k];
      r[1][k] = p;
      if constexpr (D == 3) r[2][k] = p;
    }
  }
};

void mt_lamb_stage1(const MtaMeta& m, int g_t, int p_t, int* noop, const LambArgs& a, const Launch& L) {
  const int grid = mta_grid_work(m, L.max_blocks, false);
  auto go = [&](auto skip_tag) {
    constexpr bool S = decltype(skip_tag)::value;
    LambStage1Op<S> op;
    op.a = a;
    dispatch_float(g_t, [&](auto tg) {
      dispatch_float(p_t, [&](auto tp) {
        using TG = typename decltype(tg)::type;
        using TP = typename decltype(tp)::type;
        mta_elementwise_kernel<LambStage1Op<S>, TG, TP, TP, TP><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
      }, "multi_tensor_lamb(param)");
    }, "multi_tensor_lamb(grad)");
  };
  if (a.skip_on_noop) go(std::true_type{});
  else go(std::false_type{});
  check_launch("multi_tensor_lamb_stage1");
}

void mt_lamb_stage2(const MtaMeta& m, int u_t, int p_t, int out_t, int* noop, const LambArgs& a,
                    const Launch& L) {
  const int grid = mta_grid_work(m, L.max_blocks);
  auto go = [&](auto skip_tag) {
    constexpr bool S = decltype(skip_tag)::value;
    dispatch_float(u_t, [&](auto tu) {
      dispatch_float(p_t, [&](auto tp) {
        using TU = typename decltype(tu)::type;
        using TP = typename decltype(tp)::type;
        if (m.depth == 3) {
          LambStage2Op<3, S> op;
          op.a = a;
          dispatch_model_out(out_t, [&](auto to) {
            using TO = typename decltype(to)::type;
            mta_elementwise_kernel<LambStage2Op<3, S>, TU, TP, TO><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
          }, "multi_tensor_lamb(model out)");
        } else {
          LambStage2Op<2, S> op;
          op.a = a;
          mta_elementwise_kernel<LambStage2Op<2, S>, TU, TP><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
        }
      }, "multi_tensor_lamb(param)");
    }, "multi_tensor_lamb(update)");
  };
  if (a.skip_on_noop) go(std::true_type{});
  else go(std::false_type{});
  check_launch("multi_tensor_lamb_stage2");
}

// ---------------------------------------------------------------------------------------------
// Legacy LAMB pair (per-tensor decay, reference csrc/multi_tensor_lamb_stage_1.cu:17-151 and
// csrc/multi_tensor_lamb_stage_2.cu:20-125).  Lists stage1: g, p, m, v, update.  stage2: p, update.
// ---------------------------------------------------------------------------------------------
// DEV: the capturable form (DistributedFusedLAMB's sync-free step) — the whole launch is a no-op
// when *noop (the device skip flag) is set, and the bias corrections come from the device step
// counter (reference apex/contrib/optimizers/distributed_fused_lamb.py:702-712 keeps is_finite
// and _step on the device the same way)
template <bool DEV>
struct LambLegacy1Op : MtaOpBase {
  static constexpr unsigned kRead = 0b01111, kWrite = 0b11100;
  static constexpr bool kSkipOnNoop = DEV;
  const float* decay;
  float beta1, beta2, beta3, bc1, bc2, eps, max_norm;
  const float* gnorm;
  const float* step;  // DEV: device step count (after this step's increment)
  int bias_correction;
  struct TS { float rclip, decay, rbc1, rbc2; };  // reciprocals of the clip and bias corrections
  __device__ __forceinline__ TS tensor_state(int t) const {
    const float gn = *gnorm;
    float b1 = bc1, b2 = bc2;
    if constexpr (DEV) {
      const float st = *step;
      b1 = bias_correction ? 1.f - powf(beta1, st) : 1.f;
      b2 = bias_correction ? 1.f - powf(beta2, st) : 1.f;
    }
    return {(gn > max_norm) ? max_norm / gn : 1.f, decay[t], 1.f / b1, 1.f / b2};
  }
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[5][N], const TS& s, bool&, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const float sg = r[0][k] * s.rclip;
      const float mm = r[2][k] * beta1 + beta3 * sg;
      const float vv = r[3][k] * beta2 + (1.f - beta2) * sg * sg;
      r[4][k] = (mm * s.rbc1) * fm_rcp(fm_sqrt(vv * s.rbc2) + eps) + s.decay * r[1][k];
      r[2][k] = mm;
      r[3][k] = vv;
    }
  }
};

void mt_lamb_legacy_stage1(const MtaMeta& m, int g_t, int p_t, int* noop, const float* per_tensor_decay,
                           float beta1, float beta2, float beta3, float bc1, float bc2, float eps,
                           const float* global_grad_norm, float max_global_grad_norm, const Launch& L,
                           const float* step_dev, int bias_correction) {
  auto fill = [&](auto& op) {
    op.decay = per_tensor_decay;
    op.beta1 = beta1;
    op.beta2 = beta2;
    op.beta3 = beta3;
    op.bc1 = bc1;
    op.bc2 = bc2;
    op.eps = eps;
    op.gnorm = global_grad_norm;
    op.max_norm = max_global_grad_norm;
    op.step = step_dev;
    op.bias_correction = bias_correction;
  };
  const int grid = mta_grid_work(m, L.max_blocks);
  dispatch_float(g_t, [&](auto tg) {
    dispatch_float(p_t, [&](auto tp) {
      using TG = typename decltype(tg)::type;
      using TP = typename decltype(tp)::type;
      if (step_dev) {
        LambLegacy1Op<true> op;
        fill(op);
        mta_elementwise_kernel<LambLegacy1Op<true>, TG, TP, TP, TP, TP><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
      } else {
        LambLegacy1Op<false> op;
        fill(op);
        mta_elementwise_kernel<LambLegacy1Op<false>, TG, TP, TP, TP, TP><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
      }
    }, "multi_tensor_lamb_stage1(param)");
  }, "multi_tensor_lamb_stage1(grad)");
  check_launch("multi_tensor_lamb_stage1_cuda");
}

// D == 3: the updated master is also written to a model-dtype (16-bit or fp8) copy.  DEV: skip-
// gated launch (kSkipOnNoop) with the learning rate read from the device
template <int D, bool DEV>
struct LambLegacy2Op : MtaOpBase {
  static constexpr unsigned kRead = 0b011, kWrite = (D == 3) ? 0b101 : 0b001;
  static constexpr bool kSkipOnNoop = DEV;
  const float* pn;
  const float* un;
  const float* lr_dev;
  float lr, wd;
  bool nv;
  struct TS { float ratio; };
  __device__ __forceinline__ TS tensor_state(int t) const {
    const float l = DEV ? *lr_dev : lr;
    float ratio = l;
    if (nv || wd != 0.f) {
      const float a = pn[t], b = un[t];
      ratio = (a != 0.f && b != 0.f) ? l * (a / b) : l;
    }
    return {ratio};
  }
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[D][N], const TS& s, bool&, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      r[0][k] = r[0][k] - s.ratio * r[1][k];
      if constexpr (D == 3) r[2][k] = r[0][k];
    }
  }
};

void mt_lamb_legacy_stage2(const MtaMeta& m, int p_t, int u_t, int out_t, int* noop,
                           const float* per_tensor_param_norm, const float* per_tensor_update_norm, float lr,
                           float weight_decay, bool use_nvlamb, const Launch& L, const float* lr_dev) {
  auto fill = [&](auto& op) {
    op.pn = per_tensor_param_norm;
    op.un = per_tensor_update_norm;
    op.lr = lr;
    op.lr_dev = lr_dev;
    op.wd = weight_decay;
    op.nv = use_nvlamb;
  };
  const int grid = mta_grid_work(m, L.max_blocks);
  auto run = [&](auto dev_tag) {
    constexpr bool DEV = decltype(dev_tag)::value;
    dispatch_float(p_t, [&](auto tp) {
      dispatch_float(u_t, [&](auto tu) {
        using TP = typename decltype(tp)::type;
        using TU = typename decltype(tu)::type;
        if (out_t < 0) {
          LambLegacy2Op<2, DEV> op;
          fill(op);
          mta_elementwise_kernel<LambLegacy2Op<2, DEV>, TP, TU><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
        } else {
          auto go = [&](auto to) {
            using TO = typename decltype(to)::type;
            LambLegacy2Op<3, DEV> op;
            fill(op);
            mta_elementwise_kernel<LambLegacy2Op<3, DEV>, TP, TU, TO><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, op);
          };
          // fp32 model copies too (a ZeRO shard of fp32 parameters: flat_param is fp32)
          if (out_t == kF32) go(Tag<float>{});
          else dispatch_model_out(out_t, go, "multi_tensor_lamb_stage2(model out)");
        }
      }, "multi_tensor_lamb_stage2(update)");
    }, "multi_tensor_lamb_stage2(param)");
  };
  if (lr_dev) run(std::true_type{});
  else run(std::false_type{});
  check_launch("multi_tensor_lamb_stage2_cuda");
}

// =============================================================================================
// plain cast copy (also the master->model copy) : out = in
// =============================================================================================
struct CastOp : MtaOpBase {
  static constexpr unsigned kRead = 0b01, kWrite = 0b10;
  static constexpr bool kSkipOnNoop = false;
  template <int N>
  __device__ __forceinline__ void apply(float (&r)[2][N], const TS&, bool&, float*) const {
#pragma unroll
    for (int k = 0; k < N; ++k) r[1][k] = r[0][k];
  }
};

void mt_cast(const MtaMeta& m, int in_t, int out_t, int* noop, const Launch& L) {
  const int grid = mta_grid_work(m, L.max_blocks);
  dispatch_any(in_t, [&](auto ti) {
    dispatch_any(out_t, [&](auto to) {
      using TI = typename decltype(ti)::type;
      using TO = typename decltype(to)::type;
      mta_elementwise_kernel<CastOp, TI, TO><<<grid, kMtaBlock, 0, L.stream>>>(m, noop, CastOp{});
    }, "multi_tensor_cast(out)");
  }, "multi_tensor_cast(in)");
  check_launch("multi_tensor_cast");
}

// =============================================================================================
// device-side dynamic loss scaler (reference apex/amp/scaler.py:206-226, minus the .item() sync)
// state: [0] scale, [1] inv_scale_used (1/scale that produced this step's grads),
//        [2] unskipped (as float), [3] total skipped steps
// =============================================================================================
__global__ void amp_update_scale_kernel(const int* overflow, int* skip_flag, float* st, float growth,
                                        float backoff, int interval, float min_scale, float max_scale,
                                        int dynamic) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const float scale = st[0];
  st[1] = 1.f / scale;
  const int ovf = *overflow != 0;
  const int skip = dynamic && ovf;
  *skip_flag = skip;
  if (!dynamic) {
    st[2] = st[2] + 1.f;
    return;
  }
  float ns = scale;
  float unsk = st[2];
  if (skip) {
    ns = scale * backoff;
    if (min_scale > 0.f) ns = fmaxf(min_scale, ns);
    unsk = 0.f;
    st[3] = st[3] + 1.f;
  } else {
    unsk = unsk + 1.f;
  }
  if ((int)unsk == interval) {
    ns = fminf(max_scale, ns * growth);
    unsk = 0.f;
  }
  st[0] = ns;
  st[2] = unsk;
}

void amp_update_scale(const int* overflow, int* skip_flag, float* state, float growth_factor, float backoff,
                      int growth_interval, float min_scale, float max_scale, bool dynamic, hipStream_t s) {
  amp_update_scale_kernel<<<1, 64, 0, s>>>(overflow, skip_flag, state, growth_factor, backoff, growth_interval,
                                          min_scale, max_scale, dynamic ? 1 : 0);
  check_launch("amp_update_scale");
}

}  // namespace apex_amd
