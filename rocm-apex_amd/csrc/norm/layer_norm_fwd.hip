// LayerNorm / RMSNorm forward for gfx950.
//
// Reference: csrc/layer_norm_cuda_kernel.cu:336 (cuApplyLayerNorm, Welford per row, one 32-lane
// warp-shaped block per row) and its launcher :690-718.  This kernel is register-resident:
// the row is loaded once with 16-byte vector loads, mean and variance are two exact passes
// over registers, and the normalized row is written with 16-byte stores.  Rows are owned by
// W wave64s (norm_common.h), several rows per 256-thread block for small widths so a launch
// has >> 256 workgroups for realistic n1.
#include "norm_common.h"

namespace apex_amd {
namespace norm {

template <typename TI, typename TW, typename TO, int W, int VPT>
__global__ void __launch_bounds__(block_threads<W>())
ln_fwd_kernel(const TI* __restrict__ x, const TW* __restrict__ gamma, const TW* __restrict__ beta,
              TO* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ invvar_out, int64_t n1,
              int n2, float eps, bool rms) {
  constexpr int NT = block_threads<W>();
  constexpr int RPB = NT / 64 / W;  // rows per block
  // wide rows (16 waves, 1024 threads => <= 128 VGPRs): gamma / beta are re-read per row (L2 /
  // L1 hits) instead of held in registers, and an fp32 row at 8 vectors per lane is not
  // double-buffered (64 raw words per row)
  constexpr bool GREG = W * VPT <= 32;
  constexpr bool PF = !(sizeof(TI) == 4 && VPT > 4);
  constexpr int GV = GREG ? VPT : 1;
  __shared__ float red[2 * RPB * W];
  const int wave = threadIdx.x >> 6;
  const int row_in_block = wave / W;
  const int wave_in_row = wave % W;
  const int li = wave_in_row * 64 + (threadIdx.x & 63);  // lane index within the row
  const int nv = n2 >> 3;
  const int64_t ngroups = (n1 + RPB - 1) / RPB;
  const float inv_n = 1.f / (float)n2;

  // gamma / beta are the same for every row this lane visits: loaded once (GREG)
  float g[GV][8], b[GV][8];
  auto load_gb = [&](int j, float (&gj)[8], float (&bj)[8]) {
    const int v = j * W * 64 + li;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      gj[k] = 1.f;
      bj[k] = 0.f;
    }
    if (v < nv) {
      if (gamma != nullptr) Vec8<TW>::load(gj, gamma + v * 8);
      if (beta != nullptr) Vec8<TW>::load(bj, beta + v * 8);
    }
  };
  if constexpr (GREG) {
#pragma unroll
    for (int j = 0; j < VPT; ++j) load_gb(j, g[j], b[j]);
  }
  // persistent, software-pipelined: the next row-group's input is loaded raw while the current
  // row is reduced and stored (two rows' bytes in flight per lane)
  Raw8<TI> px[VPT];
  auto prefetch = [&](int64_t grp) {
    const int64_t row = grp * RPB + row_in_block;
    const bool ok = grp < ngroups && row < n1;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = j * W * 64 + li;
      if (ok && v < nv) px[j].load(x + row * (int64_t)n2 + v * 8);
      else px[j].zero();
    }
  };
  if constexpr (PF) prefetch(blockIdx.x);
  for (int64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int64_t row = grp * RPB + row_in_block;
    const bool valid = row < n1;
    if constexpr (!PF) prefetch(grp);
    float r[VPT][8];
#pragma unroll
    for (int j = 0; j < VPT; ++j) px[j].unpack(r[j]);
    if constexpr (PF) prefetch(grp + gridDim.x);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) s += r[j][k];
    float mu = 0.f;
    if (!rms) mu = row_sum<W>(s, red, row_in_block, wave_in_row) * inv_n;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = j * W * 64 + li;
      if (v < nv) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = r[j][k] - mu;
          q += d * d;
        }
      }
    }
    q = row_sum<W>(q, red + RPB * W, row_in_block, wave_in_row);
    const float iv = rsqrtf(q * inv_n + eps);
    if (!valid) continue;
    if (li == 0) {
      if (!rms) mean_out[row] = mu;
      invvar_out[row] = iv;
    }
    TO* yr = y + row * (int64_t)n2;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = j * W * 64 + li;
      if (v < nv) {
        float gl[8], bl[8];
        if constexpr (!GREG) load_gb(j, gl, bl);
        const float* gj = GREG ? g[j < GV ? j : 0] : gl;
        const float* bj = GREG ? b[j < GV ? j : 0] : bl;
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = (r[j][k] - mu) * iv * gj[k] + bj[k];
        Vec8<TO>::store(yr + v * 8, o);
      }
    }
  }
}

// Generic path (any n2, any alignment): one 256-thread block per row, scalar loads, three
// passes over the row (the re-reads hit L1/L2).
template <typename TI, typename TW, typename TO>
__global__ void __launch_bounds__(256)
ln_fwd_generic_kernel(const TI* __restrict__ x, const TW* __restrict__ gamma, const TW* __restrict__ beta,
                      TO* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ invvar_out, int64_t n1,
                      int n2, float eps, bool rms) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  const TI* xr = x + row * (int64_t)n2;
  float s = 0.f;
  if (!rms)
    for (int i = threadIdx.x; i < n2; i += 256) s += to_f(xr[i]);
  const float mu = rms ? 0.f : block_sum(s, red) / (float)n2;
  float q = 0.f;
  for (int i = threadIdx.x; i < n2; i += 256) {
    const float d = to_f(xr[i]) - mu;
    q += d * d;
  }
  const float iv = rsqrtf(block_sum(q, red + 4) / (float)n2 + eps);
  if (threadIdx.x == 0) {
    if (!rms) mean_out[row] = mu;
    invvar_out[row] = iv;
  }
  TO* yr = y + row * (int64_t)n2;
  for (int i = threadIdx.x; i < n2; i += 256) {
    float o = (to_f(xr[i]) - mu) * iv;
    if (gamma != nullptr) o *= to_f(gamma[i]);
    if (beta != nullptr) o += to_f(beta[i]);
    yr[i] = from_f<TO>(o);
  }
}

template <typename TI, typename TW, typename TO, int W, int VPT>
static void launch_fwd(const NormFwdArgs& a, int cus, hipStream_t s) {
  constexpr int NT = block_threads<W>();
  constexpr int RPB = NT / 64 / W;
  const int64_t ngroups = (a.n1 + RPB - 1) / RPB;
  const int64_t cap = (int64_t)cus * (W == 16 ? 1 : W == 8 ? 2 : 4);  // resident blocks per CU (persistent grid)
  const int64_t grid = ngroups < cap ? ngroups : cap;
  hipLaunchKernelGGL((ln_fwd_kernel<TI, TW, TO, W, VPT>), dim3((unsigned)grid), dim3(NT), 0, s,
                     (const TI*)a.x, (const TW*)a.gamma, (const TW*)a.beta, (TO*)a.y, a.mean, a.invvar, a.n1,
                     a.n2, a.eps, a.rms);
}

static bool aligned16(const void* p) { return p == nullptr || ((uintptr_t)p & 15u) == 0; }

void norm_fwd_impl(const NormFwdArgs& a, int cus, hipStream_t s) {
  if (a.n1 <= 0 || a.n2 <= 0) return;
  const Cfg c = pick_cfg(a.n2);
  const bool fast = c.W > 0 && (a.n2 % 8 == 0) && aligned16(a.x) && aligned16(a.y) && aligned16(a.gamma) &&
                    aligned16(a.beta);
  dispatch_norm_types(a.in_t, a.w_t, a.out_t, [&](auto ti, auto tw, auto to) {
    using TI = typename decltype(ti)::type;
    using TW = typename decltype(tw)::type;
    using TO = typename decltype(to)::type;
    if (!fast) {
      hipLaunchKernelGGL((ln_fwd_generic_kernel<TI, TW, TO>), dim3((unsigned)a.n1), dim3(256), 0, s,
                         (const TI*)a.x, (const TW*)a.gamma, (const TW*)a.beta, (TO*)a.y, a.mean, a.invvar, a.n1,
                         a.n2, a.eps, a.rms);
      return;
    }
    if (c.W == 1 && c.VPT == 1) launch_fwd<TI, TW, TO, 1, 1>(a, cus, s);
    else if (c.W == 1 && c.VPT == 2) launch_fwd<TI, TW, TO, 1, 2>(a, cus, s);
    else if (c.W == 1 && c.VPT == 4) launch_fwd<TI, TW, TO, 1, 4>(a, cus, s);
    else if (c.W == 4 && c.VPT == 2) launch_fwd<TI, TW, TO, 4, 2>(a, cus, s);
    else if (c.W == 4 && c.VPT == 4) launch_fwd<TI, TW, TO, 4, 4>(a, cus, s);
    else if (c.W == 8) launch_fwd<TI, TW, TO, 8, 4>(a, cus, s);
    else if (c.VPT == 4) launch_fwd<TI, TW, TO, 16, 4>(a, cus, s);
    else launch_fwd<TI, TW, TO, 16, 8>(a, cus, s);
  });
  check_launch("layer_norm forward");
}

}  // namespace norm

void norm_fwd(const NormFwdArgs& a, int cus, hipStream_t s) { norm::norm_fwd_impl(a, cus, s); }

}  // namespace apex_amd
