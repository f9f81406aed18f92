// Spatial-tile 3x3 convolution, 64 -> 64 channels, stride 1 (ResNet-50 stage 1: conv2 forward
// and its data gradient, the flipped-weight forward), for gfx950.
//
// Why a separate kernel: the tap GEMMs of conv_igemm.hip gather the A tile once per tap from
// global memory (9 LDS-DMA passes over the same input rows per output tile).  At 64 channels a
// K-step is only 64 deep, so per MFMA the workgroup moves ~0.6 KB into LDS and reads ~1.5 KB back
// out — the LDS, not the MFMA pipe, sets the pace (fprop2 F2Cfg<256,64,8,1,2>: ~106 us for 59
// GFLOP at 56 x 56, ~22 % of the bf16 peak; profiles/resnet50_node_r04u.md).  Here a workgroup
// owns an 8 x 32 output-pixel tile of one image:
//   * the 10 x 34 x 64 input halo is staged into LDS ONCE per tile (zero outside the image: the
//     padding taps are exact zeros) and every tap reads its shifted window from it;
//   * the whole [64][9 x 64] weight tensor sits in LDS for the workgroup's lifetime (persistent
//     grid over the tiles), its rows permuted so that each lane's accumulators hold 16
//     CONSECUTIVE output channels of one pixel (32-byte epilogue stores straight from registers);
//   * 4 waves x (2 output rows x 64 channels): per 16-deep k-step 2 weight and 2 activation
//     fragments (ds_read_b128, conflict-free 144-B / 1168-B row strides) feed 4 MFMAs — 1 KB of
//     LDS per MFMA;
//   * the next tile's halo is fetched into registers under the current tile's 144 MFMAs per wave
//     and committed to LDS between two LDS-only barriers; the epilogue's stores follow the commit,
//     so neither they nor the prefetch are drained at a barrier.
// Optional epilogue: BN statistics partials (sum / sum of squares of y - shift) per workgroup,
// rows = the persistent grid size (conv_sp_grid), for the consuming batch norm's finalize.
#include "apex_amd/conv_api.h"
#include "apex_amd/conv_halo.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/mfma.h"

#include <cstdlib>
#include <stdexcept>

namespace apex_amd {
namespace csp {
using namespace mfma;

constexpr int C = 64;                  // input channels
constexpr int KO = 64;                 // output channels
constexpr int TH = 8, TW = 32;         // output tile
constexpr int HH = TH + 2, HW = TW + 2;  // halo
constexpr int PS = C + 8;              // halo pixel stride (elements): 144 B, rows 16 B apart in bank space
constexpr int WS = 9 * C + 8;          // weight row stride (elements): 1168 B
constexpr int HALO = HH * HW * PS;     // elements
constexpr int NT = 256;
constexpr int HCH = HH * HW * (C / 8);          // 16-byte chunks of the halo
constexpr int HPT = (HCH + NT - 1) / NT;        // per thread
constexpr size_t LDS = (size_t)(HALO + KO * WS) * 2;

struct Args {
  const uint16_t* x;  // [n][h][w][64]
  const uint16_t* w;  // [64][9][64]  (k = tap * 64 + c)
  uint16_t* y;        // [n][h][w][64]
  int n, h, wd, tiles_x, tiles_y, ntiles;
  int toff[9];        // per tap: (dh * HW + dw) * PS, the halo offset of the tap's window
  float* stats;       // nullable: [2][gridDim.x][64]
  const float* shift; // nullable
  const float* pcoef; // PRO: [2][64] x' = relu(x * pcoef[c] + pcoef[64 + c]) (the producing BN + ReLU)
};

// LDS-only barrier: this wave's LDS accesses complete, then a raw s_barrier (__syncthreads()
// would also drain the halo prefetch and the epilogue's global stores)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// output channel held by accumulator row j of a 32-row block: lane half lh of the C^T tile then
// holds channels 16 lh .. 16 lh + 15 in register order (crow(r, lh) -> 16 lh + r)
__device__ __forceinline__ int chan_of_row(int j) { return 16 * ((j >> 2) & 1) + (j & 3) + 4 * (j >> 3); }

// PRO: the next tile's halo is transformed in registers (one 16-byte chunk per k-step in the
// second half of the current tile's MFMA loop, when its loads have landed); the padding taps and
// out-of-image slots stay exact zeros (the mask is the fetch's)
template <typename T, bool STATS, bool PRO>
__global__ void __launch_bounds__(NT, 1) fprop_kernel(const Args p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* halo = lds;
  uint16_t* wimg = lds + HALO;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, lr = lane & 31, lh = lane >> 5;

  // weights -> LDS once (row permutation above)
  for (int i = tid; i < KO * (9 * C / 8); i += NT) {
    const int row = i / (9 * C / 8), c8 = (i % (9 * C / 8)) * 8;
    const int co = (row & ~31) + chan_of_row(row & 31);
    *reinterpret_cast<uint4*>(wimg + row * WS + c8) = *reinterpret_cast<const uint4*>(p.w + (int64_t)co * 9 * C + c8);
  }

  const int tiles_img = p.tiles_x * p.tiles_y;
  uint4 hr[HPT];
  uint32_t hok = 0;  // bit i: chunk i of the fetched halo lies inside the image
  // a thread's halo chunks all hold channels 8 (tid & 7) .. + 7 (NT % 8 == 0)
  float ps[PRO ? 8 : 1], pb[PRO ? 8 : 1];
  if constexpr (PRO) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ps[e] = p.pcoef[(tid & 7) * 8 + e];
      pb[e] = p.pcoef[C + (tid & 7) * 8 + e];
    }
  }
  auto xform = [&](int i) {
    if constexpr (PRO) {
      if ((hok >> i) & 1u) {
        float v[8];
        Vec8<T>::load(v, reinterpret_cast<const T*>(&hr[i]));
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(fmaf(v[e], ps[e], pb[e]), 0.f);
        Vec8<T>::store(reinterpret_cast<T*>(&hr[i]), v);
      } else {
        hr[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  // halo of tile `tile` -> registers (zero outside the image; every load unconditional on a
  // clamped address, the zero chosen after)
  auto fetch = [&](int tile) {
    const int img = tile / tiles_img, rem = tile - img * tiles_img;
    const int ty = rem / p.tiles_x, tx = rem - ty * p.tiles_x;
    const int y0 = ty * TH - 1, x0 = tx * TW - 1;
    const uint16_t* xb = p.x + (int64_t)img * p.h * p.wd * C;
    hok = 0;
#pragma unroll
    for (int i = 0; i < HPT; ++i) {
      const int q = tid + NT * i;
      const int pix = q >> 3, c8 = (q & 7) * 8;
      const int hy = pix / HW, hx = pix - hy * HW;
      const int iy = y0 + hy, ix = x0 + hx;
      const bool ok = q < HCH && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.wd;
      const int cy = min(max(iy, 0), p.h - 1), cx = min(max(ix, 0), p.wd - 1);
      const uint4 v = *reinterpret_cast<const uint4*>(xb + ((int64_t)cy * p.wd + cx) * C + c8);
      hok |= ok ? 1u << i : 0u;
      if constexpr (PRO) hr[i] = v;  // the mask is applied with the transform (xform)
      else hr[i] = ok ? v : make_uint4(0, 0, 0, 0);
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < HPT; ++i) {
      const int q = tid + NT * i;
      if (q < HCH) *reinterpret_cast<uint4*>(halo + (q >> 3) * PS + (q & 7) * 8) = hr[i];
    }
  };

  float s1[2][16], s2[2][16], sh[2][16];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s1[cb][r] = s2[cb][r] = 0.f;
      sh[cb][r] = (STATS && p.shift) ? p.shift[32 * cb + 16 * lh + r] : 0.f;
    }

  int tile = blockIdx.x;
  const int tlast = p.ntiles - 1;
  fetch(min(tile, tlast));
#pragma unroll
  for (int i = 0; i < HPT; ++i) xform(i);
  commit();
  __syncthreads();
  // this lane's B-fragment base: output row 2 wid + b of the tile, column lr, halo (+1, +1)
  const int bbase = ((2 * wid + 1) * HW + lr + 1) * PS + 8 * lh;
  const int abase = lr * WS + 8 * lh;
  while (tile < p.ntiles) {
    const int next = tile + gridDim.x;
    fetch(min(next, tlast));  // in flight under the MFMAs below

    f32x16 acc[2][2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) acc[b][cb] = zero16();
    // 36 k-steps (9 taps x 4 channel steps); the fragments of step i + 2 are read while step i's
    // MFMAs run (a 3-slot register ring: one wave per SIMD has no other wave to hide the LDS
    // latency behind)
    constexpr int NS = 9 * (C / 16);
    s16x8 fw[3][2], fx[3][2];
    auto rd = [&](int st, int slot) {
      const int t = st / (C / 16), kk = st % (C / 16);
      const int to = p.toff[t];
      fw[slot][0] = *reinterpret_cast<const s16x8*>(wimg + abase + t * C + 16 * kk);
      fw[slot][1] = *reinterpret_cast<const s16x8*>(wimg + abase + 32 * WS + t * C + 16 * kk);
      fx[slot][0] = *reinterpret_cast<const s16x8*>(halo + bbase + to + 16 * kk);
      fx[slot][1] = *reinterpret_cast<const s16x8*>(halo + bbase + HW * PS + to + 16 * kk);
    };
    rd(0, 0);
    rd(1, 1);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      if (st + 2 < NS) rd(st + 2, (st + 2) % 3);
      // keep the read-ahead where it is (the scheduler would otherwise sink each read next to
      // its MFMA, exposing the LDS latency at every k-step)
      __builtin_amdgcn_sched_barrier(0);
      const int sl = st % 3;
      acc[0][0] = mma<T>(fw[sl][0], fx[sl][0], acc[0][0]);
      acc[0][1] = mma<T>(fw[sl][1], fx[sl][0], acc[0][1]);
      acc[1][0] = mma<T>(fw[sl][0], fx[sl][1], acc[1][0]);
      acc[1][1] = mma<T>(fw[sl][1], fx[sl][1], acc[1][1]);
      // PRO: one chunk of the next tile's halo per k-step from step 20 on (its loads have had 20
      // steps of MFMAs to land), VALU under the MFMA pipe
      if constexpr (PRO) {
        if (st >= 20 && st - 20 < HPT) xform(st - 20);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    static_assert(!PRO || 20 + HPT <= NS, "halo transform steps");

    // every wave is done reading this tile's halo: commit the next one (the compiler waits for
    // the prefetch loads only), then the epilogue — its stores stay in flight under the next
    // tile's MFMAs
    lds_barrier();
    commit();
    // epilogue straight from the accumulators: lane (lr, lh) of block (b, cb) holds pixel lr of
    // tile row 2 wid + b, channels 32 cb + 16 lh .. + 15
    {
      const int img = tile / tiles_img, rem = tile - img * tiles_img;
      const int ty = rem / p.tiles_x, tx = rem - ty * p.tiles_x;
      const int ox = tx * TW + lr;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oy = ty * TH + 2 * wid + b;
        const bool ok = oy < p.h && ox < p.wd;
        T* yp = reinterpret_cast<T*>(p.y) + (((int64_t)img * p.h + oy) * p.wd + ox) * KO + 16 * lh;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          uint32_t wv[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const T lo = from_f<T>(acc[b][cb][2 * e]), hi = from_f<T>(acc[b][cb][2 * e + 1]);
            wv[e] = (uint32_t)lo.x | ((uint32_t)hi.x << 16);
            if constexpr (STATS) {
              if (ok) {
                const float d0 = to_f(lo) - sh[cb][2 * e], d1 = to_f(hi) - sh[cb][2 * e + 1];
                s1[cb][2 * e] += d0;
                s2[cb][2 * e] = fmaf(d0, d0, s2[cb][2 * e]);
                s1[cb][2 * e + 1] += d1;
                s2[cb][2 * e + 1] = fmaf(d1, d1, s2[cb][2 * e + 1]);
              }
            }
          }
          if (ok) {
            *reinterpret_cast<uint4*>(yp + 32 * cb) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
            *reinterpret_cast<uint4*>(yp + 32 * cb + 8) = make_uint4(wv[4], wv[5], wv[6], wv[7]);
          }
        }
      }
    }
    tile = next;
    lds_barrier();  // the next tile's halo is in LDS
  }

  if constexpr (STATS) {
    // sum over the 32 pixels (lanes) of each half, then over the 4 waves, fixed order
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int m = 1; m < 32; m <<= 1) {
          s1[cb][r] += __shfl_xor(s1[cb][r], m, 64);
          s2[cb][r] += __shfl_xor(s2[cb][r], m, 64);
        }
    float* red = reinterpret_cast<float*>(lds);  // [4 waves][2][64] (the halo is dead now)
    if (lr == 0) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          red[(wid * 2 + 0) * KO + 32 * cb + 16 * lh + r] = s1[cb][r];
          red[(wid * 2 + 1) * KO + 32 * cb + 16 * lh + r] = s2[cb][r];
        }
    }
    __syncthreads();
    if (tid < 2 * KO) {
      const int which = tid / KO, ch = tid % KO;
      float v = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) v += red[(w4 * 2 + which) * KO + ch];
      p.stats[((int64_t)which * gridDim.x + blockIdx.x) * KO + ch] = v;
    }
  }
}

}  // namespace csp

static bool sp_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("APEX_AMD_CONV_SP");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool conv_sp_supported(const ConvTapArgs& a) {
  if (a.c != csp::C || a.kout != csp::KO || a.ntaps != 9) return false;
  if (a.ish != 1 || a.isw != 1 || a.osh != 1 || a.osw != 1 || a.oph != 0 || a.opw != 0) return false;
  if (a.oh != a.ih || a.ow != a.iw || a.oht != a.oh || a.owt != a.ow) return false;
  if (a.scale || a.bias || a.residual || a.mask || a.relu) return false;
  for (int t = 0; t < 9; ++t)
    if (a.dh[t] < -1 || a.dh[t] > 1 || a.dw[t] < -1 || a.dw[t] > 1) return false;
  return ((uintptr_t)a.in % 16) == 0 && ((uintptr_t)a.wt % 16) == 0 && ((uintptr_t)a.out % 16) == 0;
}

bool conv_sp_default(const ConvTapArgs& a) { return sp_enabled() && conv_sp_supported(a); }

int conv_sp_grid(const ConvTapArgs& a, int cus) {
  const int64_t tiles = (int64_t)a.n * ((a.ih + csp::TH - 1) / csp::TH) * ((a.iw + csp::TW - 1) / csp::TW);
  return (int)std::min<int64_t>(tiles, cus);
}

void conv_sp_fprop(const ConvTapArgs& a, int cus, hipStream_t s) { conv_sp_fprop_pro(a, nullptr, cus, s); }

void conv_sp_fprop_pro(const ConvTapArgs& a, const float* pcoef, int cus, hipStream_t s) {
  if (!conv_sp_supported(a)) throw std::runtime_error("conv_sp_fprop: unsupported shape / epilogue");
  csp::Args p;
  p.x = static_cast<const uint16_t*>(a.in);
  p.w = static_cast<const uint16_t*>(a.wt);
  p.y = static_cast<uint16_t*>(a.out);
  p.n = a.n;
  p.h = a.ih;
  p.wd = a.iw;
  p.tiles_x = (a.iw + csp::TW - 1) / csp::TW;
  p.tiles_y = (a.ih + csp::TH - 1) / csp::TH;
  const int64_t nt = (int64_t)a.n * p.tiles_x * p.tiles_y;
  if (nt >= (1ll << 31)) throw std::runtime_error("conv_sp_fprop: too many tiles");
  p.ntiles = (int)nt;
  for (int t = 0; t < 9; ++t) p.toff[t] = (a.dh[t] * csp::HW + a.dw[t]) * csp::PS;
  p.stats = a.stats;
  p.shift = a.stats_shift;
  p.pcoef = pcoef;
  const int grid = conv_sp_grid(a, cus);
  dispatch_16(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    // (the LDS opt-in is set on every launch: one flag per kernel would need one static per
    // template instance, and the call is cheap next to the launch)
    auto go = [&](auto kern) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)csp::LDS);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(csp::NT), csp::LDS, s, p);
    };
    if (pcoef) {
      if (a.stats) go(csp::fprop_kernel<T, true, true>);
      else go(csp::fprop_kernel<T, false, true>);
    } else {
      if (a.stats) go(csp::fprop_kernel<T, true, false>);
      else go(csp::fprop_kernel<T, false, false>);
    }
  }, "conv_sp_fprop");
  check_launch("conv_sp_fprop");
}

}  // namespace apex_amd
