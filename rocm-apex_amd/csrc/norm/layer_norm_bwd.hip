// LayerNorm / RMSNorm backward for gfx950.
//
// Reference: csrc/layer_norm_cuda_kernel.cu:430 (cuComputePartGradGammaBeta), :498
// (cuComputeGradGammaBeta), :549 (cuComputeGradInput), launcher :753-833 — three kernels, and
// dy/x are read twice (once for dgamma/dbeta, once for dx).
//
// Here dx and the dgamma/dbeta partials come out of ONE persistent pass: a lane owns a fixed
// set of columns (the same for every row it visits), so while it computes dx for a row it also
// accumulates dy*xhat and dy for its columns in registers.  Each workgroup leaves one fp32
// partial row per quantity; a small column-reduce kernel sums the partials in a fixed order
// (bitwise deterministic, no float atomics).
#include "norm_common.h"
#include "apex_amd/launch_plan.h"

#include <cstdlib>

namespace apex_amd {
namespace norm {

// Persistent grid: enough resident blocks to saturate HBM, few enough that the partial slab
// stays small relative to the activations.
// APEX_AMD_LN_BWD_BPC = 3 | 4: that many resident blocks per CU instead of the plan's 2 (A/B knob;
// the workspace holds max(2 * cus, 1024) partial rows, so the grid stays within it)
inline int bwd_grid(int64_t ngroups, int cus) {
  static const int bpc = [] {
    const char* e = std::getenv("APEX_AMD_LN_BWD_BPC");
    const int v = e ? std::atoi(e) : 2;
    return v >= 2 && v <= 4 ? v : 2;
  }();
  if (bpc == 2) return plan::ln_bwd_grid(ngroups, cus);
  int64_t cap = (int64_t)cus * bpc;
  const int64_t ws_rows = (int64_t)cus * 2 > 1024 ? (int64_t)cus * 2 : 1024;
  if (cap > ws_rows) cap = ws_rows;
  return (int)(ngroups < cap ? (ngroups > 0 ? ngroups : 1) : cap);
}

template <typename TI, typename TW, typename TO, int W, int VPT>
__global__ void __launch_bounds__(block_threads<W>())
ln_bwd_kernel(const TO* __restrict__ dy, const TI* __restrict__ x, const float* __restrict__ mean,
              const float* __restrict__ invvar, const TW* __restrict__ gamma, TI* __restrict__ dx,
              float* __restrict__ part_g, float* __restrict__ part_b, int64_t n1, int n2, bool rms,
              bool want_dgamma, bool want_dbeta, const TO* __restrict__ dres) {
  constexpr int NT = block_threads<W>();
  constexpr int RPB = NT / 64 / W;
  __shared__ float red[2 * RPB * W];
  const int wave = threadIdx.x >> 6;
  const int row_in_block = wave / W;
  const int wave_in_row = wave % W;
  const int li = wave_in_row * 64 + (threadIdx.x & 63);
  const int nv = n2 >> 3;
  const int64_t ngroups = (n1 + RPB - 1) / RPB;
  const float inv_n = 1.f / (float)n2;

  float g[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int v = j * W * 64 + li;
    if (gamma != nullptr && v < nv) {
      Vec8<TW>::load(g[j], gamma + v * 8);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) g[j][k] = 1.f;
    }
  }
  float ag[VPT][8], ab[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ag[j][k] = 0.f;
      ab[j][k] = 0.f;
    }

  // software pipeline: the next row-group's x / dy (and statistics) are loaded raw while the
  // current one is reduced and written, so every lane keeps two rows' bytes in flight
  Raw8<TI> px[VPT];
  Raw8<TO> pd[VPT];
  Raw8<TO> pr[VPT];  // dres (a residual branch's gradient summed into dx), when given
  float pmu = 0.f, piv = 0.f;
  auto prefetch = [&](int64_t grp) {
    const int64_t row = grp * RPB + row_in_block;
    const bool ok = grp < ngroups && row < n1;
    const int64_t rr = ok ? row : 0;
    pmu = (rms || !ok) ? 0.f : mean[rr];
    piv = ok ? invvar[rr] : 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = j * W * 64 + li;
      if (ok && v < nv) {
        px[j].load(x + rr * n2 + v * 8);
        pd[j].load(dy + rr * n2 + v * 8);
        if (dres != nullptr) pr[j].load(dres + rr * n2 + v * 8);
      } else {
        px[j].zero();
        pd[j].zero();
        pr[j].zero();
      }
    }
  };
  prefetch(blockIdx.x);
  for (int64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int64_t row = grp * RPB + row_in_block;
    const bool valid = row < n1;
    const int64_t rr = valid ? row : 0;
    const float mu = pmu, iv = piv;
    float xh[VPT][8], d[VPT][8], rsd[VPT][8];
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      px[j].unpack(xh[j]);
      pd[j].unpack(d[j]);
      if (dres != nullptr) pr[j].unpack(rsd[j]);
    }
    prefetch(grp + gridDim.x);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = j * W * 64 + li;
      if (valid && v < nv) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xh[j][k] = (xh[j][k] - mu) * iv;
          const float gd = d[j][k] * g[j][k];
          s1 += gd;
          s2 += gd * xh[j][k];
          ag[j][k] += d[j][k] * xh[j][k];
          ab[j][k] += d[j][k];
        }
      }
    }
    row_sum2<W>(s1, s2, red, row_in_block, wave_in_row);
    const float m1 = rms ? 0.f : s1 * inv_n;
    const float m2 = s2 * inv_n;
    if (valid) {
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int v = j * W * 64 + li;
        if (v < nv) {
          float o[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = iv * (d[j][k] * g[j][k] - m1 - xh[j][k] * m2);
          if (dres != nullptr) {
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] += rsd[j][k];
          }
          Vec8<TI>::store(dx + rr * n2 + v * 8, o);
        }
      }
    }
  }

  if (!want_dgamma && !want_dbeta) return;
  // Combine the RPB rows-per-block lanes that own the same columns, then write one partial row.
  // LDS image: [RPB][n2] floats, reused for dgamma then dbeta.
  extern __shared__ __attribute__((aligned(16))) float cmb[];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if ((q == 0 && !want_dgamma) || (q == 1 && !want_dbeta)) continue;
    float* out = (q == 0 ? part_g : part_b) + (int64_t)blockIdx.x * n2;
    if constexpr (RPB == 1) {
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int v = j * W * 64 + li;
        if (v < nv) Vec8<float>::store(out + v * 8, q == 0 ? ag[j] : ab[j]);
      }
    } else {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int v = j * W * 64 + li;
        if (v < nv) Vec8<float>::store(cmb + (int64_t)row_in_block * n2 + v * 8, q == 0 ? ag[j] : ab[j]);
      }
      __syncthreads();
      for (int c = threadIdx.x; c < n2; c += NT) {
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < RPB; ++i) sum += cmb[i * n2 + c];
        out[c] = sum;
      }
    }
  }
}

// Wide rows (16384 < n2 <= 65536): one 1024-thread workgroup (16 waves, <= 128 VGPRs) per row,
// persistent over rows.  x and dy stay raw (16-bit: 4 words per 8 elements) in registers and are
// unpacked in each of the two passes; gamma is re-read per row (L1 / L2 hits).  With GB (VPT 2,
// n2 <= 16384) the lane also accumulates dy * xhat and dy of its 16 columns (32 registers) and the
// workgroup leaves one partial row, as the narrow kernels do; at VPT 4 / 8 those accumulators do
// not fit beside the row at 16 waves (VPT 4 spills), so ln_bwd_gb_wide_kernel makes the partials
// in a column-tiled pass (x and dy read once more).  The narrow 8-wave kernel holds gamma and the
// accumulators of 4 vectors per lane and spills: rows past 8192 take this kernel.
template <typename TI, typename TW, typename TO, int VPT, bool GB>
__global__ void __launch_bounds__(1024)
ln_bwd_wide_kernel(const TO* __restrict__ dy, const TI* __restrict__ x, const float* __restrict__ mean,
                   const float* __restrict__ invvar, const TW* __restrict__ gamma, TI* __restrict__ dx,
                   float* __restrict__ part_g, float* __restrict__ part_b, int64_t n1, int n2, bool rms,
                   const TO* __restrict__ dres) {
  constexpr int W = 16;
  constexpr int GV = GB ? VPT : 1;
  __shared__ float red[2 * W];
  const int li = threadIdx.x;
  const int wave = li >> 6;
  const int nv = n2 >> 3;
  const float inv_n = 1.f / (float)n2;
  float ag[GV][8], ab[GV][8];
#pragma unroll
  for (int j = 0; j < GV; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) ag[j][k] = ab[j][k] = 0.f;
  auto gload = [&](int v, float (&gj)[8]) {
    if (gamma != nullptr) {
      Vec8<TW>::load(gj, gamma + v * 8);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) gj[k] = 1.f;
    }
  };
  for (int64_t row = blockIdx.x; row < n1; row += gridDim.x) {
    const float mu = rms ? 0.f : mean[row], iv = invvar[row];
    Raw8<TI> px[VPT];
    Raw8<TO> pd[VPT];
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = j * W * 64 + li;
      if (v < nv) {
        px[j].load(x + row * n2 + v * 8);
        pd[j].load(dy + row * n2 + v * 8);
      } else {
        px[j].zero();
        pd[j].zero();
      }
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = j * W * 64 + li;
      if (v < nv) {
        float xh[8], d[8], gj[8];
        px[j].unpack(xh);
        pd[j].unpack(d);
        gload(v, gj);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xh[k] = (xh[k] - mu) * iv;
          const float gd = d[k] * gj[k];
          s1 += gd;
          s2 += gd * xh[k];
          if constexpr (GB) {
            ag[j < GV ? j : 0][k] += d[k] * xh[k];
            ab[j < GV ? j : 0][k] += d[k];
          }
        }
      }
      // one vector's gamma / unpacked values live at a time (the scheduler would otherwise hoist
      // every vector's gamma load and spill at 16 waves)
      __builtin_amdgcn_sched_barrier(0);
    }
    row_sum2<W>(s1, s2, red, 0, wave);
    const float m1 = rms ? 0.f : s1 * inv_n;
    const float m2 = s2 * inv_n;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = j * W * 64 + li;
      if (v < nv) {
        float xh[8], d[8], gj[8], o[8];
        px[j].unpack(xh);
        pd[j].unpack(d);
        gload(v, gj);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = iv * (d[k] * gj[k] - m1 - (xh[k] - mu) * iv * m2);
        if (dres != nullptr) {
          float rs[8];
          Vec8<TO>::load(rs, dres + row * n2 + v * 8);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += rs[k];
        }
        Vec8<TI>::store(dx + row * n2 + v * 8, o);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (GB) {
    if (part_g == nullptr) return;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = j * W * 64 + li;
      if (v < nv) {
        Vec8<float>::store(part_g + (int64_t)blockIdx.x * n2 + v * 8, ag[j]);
        Vec8<float>::store(part_b + (int64_t)blockIdx.x * n2 + v * 8, ab[j]);
      }
    }
  }
}

// dgamma / dbeta partials of wide rows: grid (n2 / 2048 column blocks, P row parts); a thread owns
// 8 columns (16-byte loads) over rows p, p + P, ...; partial row p of each quantity out.
template <typename TI, typename TO>
__global__ void __launch_bounds__(256)
ln_bwd_gb_wide_kernel(const TO* __restrict__ dy, const TI* __restrict__ x, const float* __restrict__ mean,
                      const float* __restrict__ invvar, float* __restrict__ part_g, float* __restrict__ part_b,
                      int64_t n1, int n2, bool rms) {
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v >= (n2 >> 3)) return;
  float sg[8], sb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sg[k] = sb[k] = 0.f;
  for (int64_t r = blockIdx.y; r < n1; r += gridDim.y) {
    const float mu = rms ? 0.f : mean[r], iv = invvar[r];
    float xv[8], d[8];
    Vec8<TI>::load(xv, x + r * n2 + v * 8);
    Vec8<TO>::load(d, dy + r * n2 + v * 8);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sg[k] += d[k] * ((xv[k] - mu) * iv);
      sb[k] += d[k];
    }
  }
  Vec8<float>::store(part_g + (int64_t)blockIdx.y * n2 + v * 8, sg);
  Vec8<float>::store(part_b + (int64_t)blockIdx.y * n2 + v * 8, sb);
}

// dgamma[c] = sum_b part[b][c] in fixed b order.  Block = 64 columns x 4 row-groups.
template <typename TW>
__global__ void __launch_bounds__(256)
ln_col_reduce_kernel(const float* __restrict__ part_g, const float* __restrict__ part_b, TW* __restrict__ dgamma,
                     TW* __restrict__ dbeta, int nparts, int n2) {
  __shared__ float red[16][17];
  const float* part = blockIdx.y == 0 ? part_g : part_b;
  TW* out = blockIdx.y == 0 ? dgamma : dbeta;
  if (out == nullptr) return;  // uniform over the block
  const float v = colreduce16(part, nparts, n2, red);
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  if ((threadIdx.x >> 4) == 0 && c < n2) out[c] = from_f<TW>(v);
}

// Generic path: dx per row (block per row) and dgamma/dbeta partials by a column-tiled pass.
template <typename TI, typename TW, typename TO>
__global__ void __launch_bounds__(256)
ln_bwd_dx_generic_kernel(const TO* __restrict__ dy, const TI* __restrict__ x, const float* __restrict__ mean,
                         const float* __restrict__ invvar, const TW* __restrict__ gamma, TI* __restrict__ dx,
                         int64_t n1, int n2, bool rms, const TO* __restrict__ dres) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  const float mu = rms ? 0.f : mean[row];
  const float iv = invvar[row];
  const TI* xr = x + row * n2;
  const TO* dr = dy + row * n2;
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < n2; i += 256) {
    const float gd = to_f(dr[i]) * (gamma ? to_f(gamma[i]) : 1.f);
    s1 += gd;
    s2 += gd * (to_f(xr[i]) - mu) * iv;
  }
  s1 = block_sum(s1, red);
  s2 = block_sum(s2, red + 4);
  const float m1 = rms ? 0.f : s1 / (float)n2, m2 = s2 / (float)n2;
  for (int i = threadIdx.x; i < n2; i += 256) {
    const float gd = to_f(dr[i]) * (gamma ? to_f(gamma[i]) : 1.f);
    const float xh = (to_f(xr[i]) - mu) * iv;
    dx[row * n2 + i] = from_f<TI>(iv * (gd - m1 - xh * m2) + (dres ? to_f(dres[row * n2 + i]) : 0.f));
  }
}

template <typename TI, typename TO>
__global__ void __launch_bounds__(256)
ln_bwd_gb_generic_kernel(const TO* __restrict__ dy, const TI* __restrict__ x, const float* __restrict__ mean,
                         const float* __restrict__ invvar, float* __restrict__ part_g, float* __restrict__ part_b,
                         int64_t n1, int n2, bool rms) {
  // grid (ceil(n2/256), nparts): each thread owns one column over a strided subset of rows
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n2) return;
  float sg = 0.f, sb = 0.f;
  for (int64_t r = blockIdx.y; r < n1; r += gridDim.y) {
    const float d = to_f(dy[r * n2 + c]);
    const float xh = (to_f(x[r * n2 + c]) - (rms ? 0.f : mean[r])) * invvar[r];
    sg += d * xh;
    sb += d;
  }
  part_g[(int64_t)blockIdx.y * n2 + c] = sg;
  part_b[(int64_t)blockIdx.y * n2 + c] = sb;
}

template <typename TI, typename TW, typename TO, int W, int VPT>
static int launch_bwd(const NormBwdArgs& a, int cus, hipStream_t s) {
  constexpr int NT = block_threads<W>();
  constexpr int RPB = NT / 64 / W;
  const int64_t ngroups = (a.n1 + RPB - 1) / RPB;
  const int grid = bwd_grid(ngroups, cus);
  const bool wg = a.dgamma != nullptr, wb = a.dbeta != nullptr;
  const size_t lds = (RPB > 1 && (wg || wb)) ? (size_t)RPB * a.n2 * sizeof(float) : 0;
  float* pg = a.workspace;
  float* pb = a.workspace + (int64_t)grid * a.n2;
  hipLaunchKernelGGL((ln_bwd_kernel<TI, TW, TO, W, VPT>), dim3(grid), dim3(NT), lds, s, (const TO*)a.dy,
                     (const TI*)a.x, a.mean, a.invvar, (const TW*)a.gamma, (TI*)a.dx, pg, pb, a.n1, a.n2, a.rms,
                     wg, wb, (const TO*)a.dres);
  return grid;
}

// the raw x / dy words a lane of the wide kernel keeps per row must stay <= 64 of its 128 VGPRs
// (fp32 rows at 8 vectors per lane take the generic kernels)
template <typename TI, typename TO, int VPT>
constexpr bool wide_ok() { return VPT * 2 * (int)(sizeof(TI) + sizeof(TO)) <= 64; }

template <typename TI, typename TW, typename TO, int VPT>
static int launch_bwd_wide(const NormBwdArgs& a, int cus, hipStream_t s) {
  const bool want = a.dgamma != nullptr || a.dbeta != nullptr;
  const int grid = (int)(a.n1 < cus ? a.n1 : cus);
  constexpr bool GB = VPT <= 2;
  float* pg = want && GB ? a.workspace : nullptr;
  float* pb = want && GB ? a.workspace + (int64_t)grid * a.n2 : nullptr;
  hipLaunchKernelGGL((ln_bwd_wide_kernel<TI, TW, TO, VPT, GB>), dim3(grid), dim3(1024), 0, s, (const TO*)a.dy,
                     (const TI*)a.x, a.mean, a.invvar, (const TW*)a.gamma, (TI*)a.dx, pg, pb, a.n1, a.n2, a.rms,
                     (const TO*)a.dres);
  if (!want) return 0;
  if (GB) return grid;
  const int cb = (a.n2 / 8 + 255) / 256;
  int64_t p = ((int64_t)cus * 4 + cb - 1) / cb;
  if (p > a.n1) p = a.n1;
  if (p > 1024) p = 1024;
  const int parts = (int)(p < 1 ? 1 : p);
  hipLaunchKernelGGL((ln_bwd_gb_wide_kernel<TI, TO>), dim3(cb, parts), dim3(256), 0, s, (const TO*)a.dy,
                     (const TI*)a.x, a.mean, a.invvar, a.workspace, a.workspace + (int64_t)parts * a.n2, a.n1, a.n2,
                     a.rms);
  return parts;
}

static bool aligned16(const void* p) { return p == nullptr || ((uintptr_t)p & 15u) == 0; }

static int generic_parts(int64_t n1, int n2, int cus) {
  const int64_t col_blocks = (n2 + 255) / 256;
  int64_t p = ((int64_t)cus * 4 + col_blocks - 1) / col_blocks;
  if (p > n1) p = n1;
  if (p > 1024) p = 1024;
  return (int)(p < 1 ? 1 : p);
}

void norm_bwd_impl(const NormBwdArgs& a, int cus, hipStream_t s) {
  if (a.n1 <= 0 || a.n2 <= 0) return;
  const Cfg c = pick_cfg(a.n2);
  const bool fast = c.W > 0 && (a.n2 % 8 == 0) && aligned16(a.x) && aligned16(a.dy) && aligned16(a.dx) && aligned16(a.dres) &&
                    aligned16(a.gamma);
  const bool want = a.dgamma != nullptr || a.dbeta != nullptr;
  dispatch_norm_types(a.in_t, a.w_t, a.out_t, [&](auto ti, auto tw, auto to) {
    using TI = typename decltype(ti)::type;
    using TW = typename decltype(tw)::type;
    using TO = typename decltype(to)::type;
    int nparts = 0;
    const bool wide_fits = c.W < 16 || (c.VPT == 4 ? wide_ok<TI, TO, 4>() : wide_ok<TI, TO, 8>());
    // rows of 8193 .. 16384 (the forward's 8-wave geometry): the 16-wave kernel at 2 vectors per
    // lane (see ln_bwd_wide_kernel)
    const bool wide2 = c.W == 8;
    if (fast && wide_fits) {
      if (c.W == 1 && c.VPT == 1) nparts = launch_bwd<TI, TW, TO, 1, 1>(a, cus, s);
      else if (c.W == 1 && c.VPT == 2) nparts = launch_bwd<TI, TW, TO, 1, 2>(a, cus, s);
      else if (c.W == 1 && c.VPT == 4) nparts = launch_bwd<TI, TW, TO, 1, 4>(a, cus, s);
      else if (c.W == 4 && c.VPT == 2) nparts = launch_bwd<TI, TW, TO, 4, 2>(a, cus, s);
      else if (c.W == 4 && c.VPT == 4) nparts = launch_bwd<TI, TW, TO, 4, 4>(a, cus, s);
      else if (wide2) nparts = launch_bwd_wide<TI, TW, TO, 2>(a, cus, s);
      else if (c.VPT == 4) nparts = launch_bwd_wide<TI, TW, TO, 4>(a, cus, s);
      else if constexpr (wide_ok<TI, TO, 8>()) nparts = launch_bwd_wide<TI, TW, TO, 8>(a, cus, s);
    } else {
      hipLaunchKernelGGL((ln_bwd_dx_generic_kernel<TI, TW, TO>), dim3((unsigned)a.n1), dim3(256), 0, s,
                         (const TO*)a.dy, (const TI*)a.x, a.mean, a.invvar, (const TW*)a.gamma, (TI*)a.dx, a.n1,
                         a.n2, a.rms, (const TO*)a.dres);
      if (want) {
        nparts = generic_parts(a.n1, a.n2, cus);
        hipLaunchKernelGGL((ln_bwd_gb_generic_kernel<TI, TO>), dim3((a.n2 + 255) / 256, nparts), dim3(256), 0, s,
                           (const TO*)a.dy, (const TI*)a.x, a.mean, a.invvar, a.workspace,
                           a.workspace + (int64_t)nparts * a.n2, a.n1, a.n2, a.rms);
      }
    }
    if (want) {
      hipLaunchKernelGGL((ln_col_reduce_kernel<TW>), dim3((a.n2 + 15) / 16, 2), dim3(256), 0, s, a.workspace,
                         a.workspace + (int64_t)nparts * a.n2, (TW*)a.dgamma, (TW*)a.dbeta, nparts, a.n2);
    }
  });
  check_launch("layer_norm backward");
}

}  // namespace norm

int64_t norm_bwd_workspace_floats(int64_t n1, int n2, int cus) {
  const int64_t fast_parts = (int64_t)cus * 2;
  const int64_t gen_parts = 1024;
  const int64_t parts = fast_parts > gen_parts ? fast_parts : gen_parts;
  return 2 * parts * (int64_t)n2;
}

void norm_bwd(const NormBwdArgs& a, int cus, hipStream_t s) { norm::norm_bwd_impl(a, cus, s); }

}  // namespace apex_amd
