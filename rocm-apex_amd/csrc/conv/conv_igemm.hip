// Implicit-GEMM convolutions on NHWC activations for gfx950 (MFMA 32x32x16, LDS-DMA staging).
//
// Reference capability: the fused NHWC convolutions of apex/contrib/bottleneck (cudnn-frontend
// execution plans, apex/contrib/csrc/bottleneck/bottleneck.cpp:2472-2485); the reference builds
// none of it on ROCm.  Here they are the ResNet 3x3 / strided convolutions, which MIOpen runs at
// 20-30 % of their MFMA roofline on MI355X (profiles/conv_shapes_miopen_r02.jsonl).
//
// fprop ("tap" GEMM, forward and data-gradient, conv_api.h):
//   M = n * oh * ow output pixels, N = kout, K = ntaps * c.  256 x BN x 64 tile per 512-thread
//   workgroup (8 waves; BN = 256 / 128 / 64 picked per shape so the launch fills 256 CUs), each
//   wave a (256/WM) x (BN/WN) block of 32x32 accumulators.  Per K-step (one tap, 64 channels)
//   the A tile is GATHERED by LDS-DMA (global_load_lds_dwordx4): every lane fetches 16 B of one
//   output pixel's shifted input row, taps that fall into the zero padding (and rows past M)
//   read a zero page instead — no im2col buffer, no bounds branch around the DMA.  The B tile is
//   the weight slice [BN][64] (k contiguous).  Both images are k-major [rows][64] with the bank
//   swizzle applied on the SOURCE address (16-B chunk c of row r at c ^ ((r >> 1) & 7)), the
//   next K-step's DMA is in flight under the current step's MFMAs, one barrier per step.
//   Epilogue: fp32 accumulators staged through LDS, 16-byte row stores at the (possibly
//   strided, phase-shifted) output pixel.
//
// wgrad: dW[k][t][c] = sum over pixels of dY[p][k] * X[p shifted by tap t][c].  Both operands
//   are pixel-major ([pixel][channels], channels contiguous), so the reduction dim is the ROW of
//   both LDS images; fragments are read with ds_read_b64_tr_b16 (hardware transpose).  The
//   pixel range is split over workgroups (the output is only kout x 9c), each writes an fp32
//   partial tile, and a reduce pass sums the partials in a fixed order (deterministic) and
//   converts to the weight dtype.
#include "apex_amd/conv_api.h"
#include "apex_amd/conv_halo.h"
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/fastdiv.h"
#include "apex_amd/launch_plan.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace apex_amd {
namespace conv {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// 128 bytes of zeros: the DMA source for padding taps and rows past the end
__device__ __attribute__((aligned(16))) uint16_t g_zero[64];

struct Geo {
  int n, h, w, c, oh, ow, oht, owt, kout, ish, isw, osh, osw, oph, opw, ntaps, m;
  int dh[kConvMaxTaps], dw[kConvMaxTaps];
  int tapoff[kConvMaxTaps];  // byte offset of tap t in the input image: (dh * w + dw) * c * 2
  FastDiv div_ohw, div_ow;
  int ident;                 // output pixel == M row (stride-1 placement over the whole tensor)
  int xbytes, wbytes;        // buffer-descriptor ranges (< 2^31: fprop2 only)
  const float* scale;
  const float* bias;
  const uint16_t* res;
  const uint16_t* mask;
  int relu;
  float* stats;         // nullable: BN statistics partials [2][tiles_m][kout] of the stored output
  const float* shift;   //   about this per-channel shift (nullable = 0)
  const uint16_t* rx;   // nullable: BN backward reduction mode (ConvTapArgs::red_x) — stats then
  const float* rcoef;   //   holds sum(g) / sum(g (x - mean)) of the masked gradient g
  const float* rmean;
};

inline Geo make_geo(const ConvTapArgs& a) {
  Geo g;
  g.n = a.n; g.h = a.ih; g.w = a.iw; g.c = a.c; g.oh = a.oh; g.ow = a.ow; g.oht = a.oht; g.owt = a.owt;
  g.kout = a.kout; g.ish = a.ish; g.isw = a.isw; g.osh = a.osh; g.osw = a.osw; g.oph = a.oph; g.opw = a.opw;
  g.ntaps = a.ntaps;
  g.m = a.n * a.oh * a.ow;
  g.scale = a.scale;
  g.bias = a.bias;
  g.res = reinterpret_cast<const uint16_t*>(a.residual);
  g.stats = a.stats;
  g.shift = a.stats_shift;
  g.mask = reinterpret_cast<const uint16_t*>(a.mask);
  g.relu = a.relu;
  g.rx = reinterpret_cast<const uint16_t*>(a.red_x);
  g.rcoef = a.red_coef;
  g.rmean = a.red_mean;
  for (int t = 0; t < kConvMaxTaps; ++t) {
    g.dh[t] = t < a.ntaps ? a.dh[t] : 0;
    g.dw[t] = t < a.ntaps ? a.dw[t] : 0;
    g.tapoff[t] = (g.dh[t] * a.iw + g.dw[t]) * a.c * 2;
  }
  g.div_ohw = make_fastdiv((uint32_t)(a.oh * a.ow));
  g.div_ow = make_fastdiv((uint32_t)a.ow);
  g.ident = a.osh == 1 && a.osw == 1 && a.oph == 0 && a.opw == 0 && a.oht == a.oh && a.owt == a.ow;
  const int64_t xb = (int64_t)a.n * a.ih * a.iw * a.c * 2, wb = (int64_t)a.kout * a.ntaps * a.c * 2;
  g.xbytes = xb < (1ll << 31) ? (int)xb : -1;
  g.wbytes = wb < (1ll << 31) ? (int)wb : -1;
  return g;
}

__device__ __forceinline__ void dma16(const uint16_t* src, uint16_t* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

template <typename T>
__device__ __forceinline__ f32x16 mfma(s16x8 a, s16x8 b, f32x16 c);
template <>
__device__ __forceinline__ f32x16 mfma<bf16_t>(s16x8 a, s16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}
template <>
__device__ __forceinline__ f32x16 mfma<f16_t>(s16x8 a, s16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

// XCD-aware, bijective remap of the linear workgroup id (consecutive ids share an XCD's L2:
// neighbouring output-pixel tiles re-read overlapping input rows through it)
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// =============================================================================================
// fprop
// =============================================================================================
constexpr int BM = 256, BK = 64;  // fprop_kernel output-pixel tile, K step
constexpr int STAGES = 3;  // wgrad LDS ring depth

// Tile configuration: BN output channels per workgroup, WM x WN waves, S-deep LDS ring.
template <int BN_, int WM_, int WN_, int S_>
struct FCfg {
  static constexpr int BN = BN_, WM = WM_, WN = WN_, S = S_;
  static constexpr int NW = WM * WN, THREADS = NW * 64;
  static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;   // 32x32 MFMA tiles per wave
  static constexpr int PA = BM / 8 / NW, PB = BN / 8 / NW;     // 1-KB DMA pieces per wave
  static constexpr size_t OPS = (size_t)S * (BM * BK + BN * BK) * 2;
  static constexpr size_t EPI = (size_t)128 * (BN + 4) * 4;
  static constexpr size_t LDS = OPS > EPI ? OPS : EPI;
  static_assert(PA >= 1 && PB >= 1 && TM >= 1 && TN >= 1, "bad tile configuration");
};

// Epilogue of one EH-row chunk of an fprop tile whose fp32 accumulators are staged in ``cs``
// ([EH][BN + 4] floats): fused scale / bias / residual / ReLU / mask, 16-byte row stores.  The
// consuming BN's statistics of the stored values accumulate in the caller's st1 / st2 (8
// columns per thread) over all chunks of the tile; stats_fold writes the tile's row.
// RED: the BN backward reduction mode (Geo::rx) — a compile-time variant: the runtime branch alone
// cost the plain epilogue its occupancy (stage-2 F2Cfg<256,64,8,1,2> 97 -> 136 us in the step,
// profiles/r06/resnet50_step_timeline_r06m.md vs _r06f.md)
template <typename T, int BN, int THREADS, int EH, bool RED = false>
__device__ __forceinline__ void epi_chunk(const Geo& g, uint16_t* __restrict__ Y, const float* cs, int row0c,
                                          int col0, int tid, float (&st1)[8], float (&st2)[8]) {
  constexpr int CST = BN + 4;
  constexpr int CPR = BN / 8;               // 8-column chunks per row
  constexpr int RP = THREADS / CPR;         // rows per pass
  static_assert(EH % RP == 0 || RP > EH, "epilogue row passes");
  const int ch = tid % CPR, rsub = tid / CPR;
  const int gc = col0 + ch * 8;
  float sc[8], bi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = 1.f;
    bi[e] = 0.f;
  }
  if (g.scale) Vec8<float>::load(sc, g.scale + gc);
  if (g.bias) Vec8<float>::load(bi, g.bias + gc);
  const bool affine = g.scale || g.bias;
  float sft[8], rsc[RED ? 8 : 1], rsh[RED ? 8 : 1];
#pragma unroll
  for (int e = 0; e < 8; ++e) sft[e] = 0.f;
  if (g.stats && g.shift && !RED) Vec8<float>::load(sft, g.shift + gc);
  if constexpr (RED) {  // BN backward reduction: sft = the BN's mean, rsc / rsh its forward apply coefficients
    Vec8<float>::load(sft, g.rmean + gc);
    Vec8<float>::load(rsc, g.rcoef + gc);
    Vec8<float>::load(rsh, g.rcoef + g.kout + gc);
  }
  const int ohw = g.oh * g.ow;
#pragma unroll
  for (int it = 0; it < (EH + RP - 1) / RP; ++it) {
    const int rl = rsub + RP * it;
    const int m = row0c + rl;
    if (rl < EH && m < g.m) {
      int64_t pix = m;
      if (!g.ident) {
        const int nimg = (int)fdiv((uint32_t)m, g.div_ohw), rem = m - nimg * ohw;
        const int oy = (int)fdiv((uint32_t)rem, g.div_ow), ox = rem - oy * g.ow;
        pix = ((int64_t)nimg * g.oht + oy * g.osh + g.oph) * g.owt + ox * g.osw + g.opw;
      }
      float v[8];
      const float4 lo = *reinterpret_cast<const float4*>(cs + rl * CST + ch * 8);
      const float4 hi = *reinterpret_cast<const float4*>(cs + rl * CST + ch * 8 + 4);
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
      v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      if (affine) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaf(v[e], sc[e], bi[e]);
      }
      if (g.res) {
        float r[8];
        Vec8<T>::load(r, reinterpret_cast<const T*>(g.res) + pix * g.kout + gc);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e];
      }
      if (g.relu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (g.mask) {
        float mk[8];
        Vec8<T>::load(mk, reinterpret_cast<const T*>(g.mask) + pix * g.kout + gc);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = mk[e] > 0.f ? v[e] : 0.f;
      }
      if constexpr (RED) {
        // the stored (rounded) gradient, masked by the BN's forward ReLU recomputed from its
        // input: what the standalone reduction pass would read back and sum
        float xv[8];
        Vec8<T>::load(xv, reinterpret_cast<const T*>(g.rx) + pix * g.kout + gc);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gq = fmaf(xv[e], rsc[e], rsh[e]) > 0.f ? to_f(from_f<T>(v[e])) : 0.f;
          v[e] = gq;
          st1[e] += gq;
          st2[e] = fmaf(gq, xv[e] - sft[e], st2[e]);
        }
      }
      Vec8<T>::store(reinterpret_cast<T*>(Y) + pix * g.kout + gc, v);
      if (g.stats && !RED) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[e] - sft[e];
          st1[e] += d;
          st2[e] = fmaf(d, d, st2[e]);
        }
      }
    }
  }
}

// fixed-order fold of the thread groups sharing each 8-column chunk -> statistics row ``srow``
// of [2][rows][kout] (rows = the launch's M tiles: conv_tap_stats_tiles).  Uses ``red`` (LDS,
// 2 x min(RP, rows_per_tile) x BN floats) — the caller has barriered after its last read of it.
template <int BN, int THREADS>
__device__ __forceinline__ void stats_fold(const Geo& g, float* red, int srow, int rows, int col0, int tid,
                                           const float (&st1)[8], const float (&st2)[8]) {
  constexpr int CPR = BN / 8, RP = THREADS / CPR;
  const int ch = tid % CPR, rsub = tid / CPR;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[(rsub * 2 + 0) * BN + ch * 8 + e] = st1[e];
    red[(rsub * 2 + 1) * BN + ch * 8 + e] = st2[e];
  }
  __syncthreads();
  for (int i = tid; i < 2 * BN; i += THREADS) {
    const int which = i / BN, col = i % BN;
    float acc2 = 0.f;
    for (int r = 0; r < RP; ++r) acc2 += red[(r * 2 + which) * BN + col];
    g.stats[((int64_t)which * rows + srow) * g.kout + col0 + col] = acc2;
  }
}

// k-major fragment of a 32-row subtile at k-step kk from a swizzled [rows][64] image
__device__ __forceinline__ s16x8 frag_k(const uint16_t* tile, int rowbase, int kk, int lane) {
  const int row = rowbase + (lane & 31);
  const int c = (2 * kk + (lane >> 5)) ^ ((row >> 1) & 7);
  return *reinterpret_cast<const s16x8*>(tile + row * BK + 8 * c);
}

template <typename T, typename C, bool RED = false>
__global__ void __launch_bounds__(C::THREADS, 1)
fprop_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y, Geo g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  constexpr int BN = C::BN, WM = C::WM, WN = C::WN, NW = C::NW, TM = C::TM, TN = C::TN;
  constexpr int PA = C::PA, PB = C::PB, S = C::S;
  constexpr int TA = BM * BK, TB = BN * BK;
  auto a_buf = [&](int b) { return lds + b * (TA + TB); };
  auto b_buf = [&](int b) { return lds + b * (TA + TB) + TA; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (g.m + BM - 1) / BM, tiles_n = g.kout / BN;
  const int wg = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  // N-fastest order: the BN-column tiles of one pixel tile run back to back (A panel reuse)
  const int bm = wg / tiles_n, bn = wg % tiles_n;
  const int row0 = bm * BM, col0 = bn * BN;
  const int ohw = g.oh * g.ow;
  const int64_t kw = (int64_t)g.ntaps * g.c;  // weight row length

  // this lane's PA A rows (fixed for the whole K loop): image base + input origin of the pixel
  int64_t abase[PA];
  int aih[PA], aiw[PA], asrc[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int row = 8 * (i * NW + wave) + (lane >> 3);
    const int m = row0 + row;
    asrc[i] = 8 * ((lane & 7) ^ ((row >> 1) & 7));
    if (m < g.m) {
      const int nimg = m / ohw, rem = m - nimg * ohw;
      const int oy = rem / g.ow, ox = rem - oy * g.ow;
      abase[i] = (int64_t)nimg * g.h * g.w * g.c;
      aih[i] = oy * g.ish;
      aiw[i] = ox * g.isw;
    } else {
      abase[i] = 0;
      aih[i] = -(1 << 28);  // every tap lands outside: zero page
      aiw[i] = 0;
    }
  }
  const int cblocks = g.c / BK;
  const int nk = g.ntaps * cblocks;

  auto issue = [&](int kt, int buf) {
    const int t = kt / cblocks, c0 = (kt - t * cblocks) * BK;
    const int dh = g.dh[t], dw = g.dw[t];
    uint16_t* adst = a_buf(buf);
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int ih = aih[i] + dh, iw = aiw[i] + dw;
      const bool ok = (unsigned)ih < (unsigned)g.h && (unsigned)iw < (unsigned)g.w;
      // branch-free select: every lane issues exactly one DMA per piece (a divergent branch
      // would issue the instruction twice and break the counted vmcnt)
      const uintptr_t real = (uintptr_t)(X + abase[i] + ((int64_t)ih * g.w + iw) * g.c + c0 + asrc[i]);
      const uintptr_t zero = (uintptr_t)(g_zero + asrc[i]);
      const uintptr_t msk = (uintptr_t)0 - (uintptr_t)ok;
      dma16((const uint16_t*)((real & msk) | (zero & ~msk)), adst + (i * NW + wave) * 512);
    }
    uint16_t* bdst = b_buf(buf);
    const int64_t k0 = (int64_t)t * g.c + c0;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int j = i * NW + wave;
      const int row = 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      dma16(Wt + (int64_t)(col0 + row) * kw + k0 + 8 * c, bdst + j * 512);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // S-stage ring (cdna_hip_programming.md "Pipelining across barriers"): the DMA of step
  // kt+S-1 is issued while step kt computes.  Each wave waits only for ITS OWN DMA of step kt
  // (counted vmcnt: newer steps stay in flight), then a raw s_barrier publishes every wave's
  // pieces (a __syncthreads would drain vmcnt to 0).  The buffer refilled at step kt was last
  // read at step kt-1, which every wave finished before this barrier.
  constexpr int PER_STEP = PA + PB;  // DMA instructions per wave per K-step
#pragma unroll
  for (int p = 0; p < S - 1; ++p)
    if (p < nk) issue(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = nk - 1 - kt < S - 2 ? nk - 1 - kt : S - 2;  // younger steps in flight
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_STEP) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + S - 1 < nk) issue(kt + S - 1, (kt + S - 1) % S);
    const int cur = kt % S;
    const uint16_t* at = a_buf(cur);
    const uint16_t* bt = b_buf(cur);
    // all of this step's fragments first (the reads of later k-slices overlap the MFMAs of
    // earlier ones; the compiler's counted lgkmcnt waits release them one slice at a time)
    s16x8 af[BK / 16][TM], bf[BK / 16][TN];
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
#pragma unroll
      for (int i = 0; i < TM; ++i) af[kk][i] = frag_k(at, wm * (BM / WM) + 32 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[kk][j] = frag_k(bt, wn * (BN / WN) + 32 * j, kk, lane);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma<T>(af[kk][i], bf[kk][j], acc[i][j]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: 128-row chunks staged as fp32 through LDS, 16-byte row stores ----
  float* cs = reinterpret_cast<float*>(lds);
  constexpr int BMT = BM;
  float st1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, st2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int half = 0; half < BM / 128; ++half) {
    const int wr0 = wm * (BM / WM);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rb = wr0 + 32 * i;
      if (rb / 128 != half) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = rb - 128 * half + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          cs[rl * (BN + 4) + wn * (BN / WN) + 32 * j + (lane & 31)] = acc[i][j][r];
        }
    }
    __syncthreads();
    epi_chunk<T, BN, C::THREADS, 128, RED>(g, Y, cs, row0 + 128 * half, col0, tid, st1, st2);
    __syncthreads();
  }
  if (g.stats) stats_fold<BN, C::THREADS>(g, cs, bm, (g.m + BMT - 1) / BMT, col0, tid, st1, st2);
}

// ---------------------------------------------------------------------------------------------
// fprop2: the same tap GEMM with the operand staging rebuilt for a low VALU count per MFMA.
//   * A rows are fetched with buffer_load ... lds through a range-checked descriptor: a padding
//     tap or a row past M gets an out-of-range offset and the hardware writes zeros (no zero
//     page, no 64-bit address math).  Each lane precomputes, once, its rows' byte offsets and a
//     ntaps-bit validity mask, so a K-step costs ~4 VALU per 1-KiB piece (bit test, add, select)
//     instead of ~20 (64-bit address, two range compares, select).
//   * B (weights) offsets are a per-lane constant plus the step's scalar k offset.
//   * Pixel decomposition (setup and epilogue) by multiply-high (FastDiv), the epilogue skips
//     it entirely for the identity output placement.
//   * BM x BN tiles with 64 x 64 (or 128 x 64) per wave: every A fragment feeds TN MFMAs and every
//     B fragment TM (the 32 x 64 per-wave tiles of fprop_kernel re-read B for every 2 MFMAs).
// Requires the input and weight tensors to be < 2 GiB (buffer ranges); fprop_kernel otherwise.
// ---------------------------------------------------------------------------------------------
template <int BM_, int BN_, int WM_, int WN_, int S_>
struct F2Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, S = S_;
  static constexpr int NW = WM * WN, THREADS = NW * 64;
  static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static constexpr int PA = BM / 8 / NW, PB = BN / 8 / NW;
  static constexpr size_t OPS = (size_t)S * (BM * BK + BN * BK) * 2;
  static constexpr size_t EPI = (size_t)128 * (BN + 4) * 4;
  static constexpr size_t LDS = OPS > EPI ? OPS : EPI;
  static_assert(PA >= 1 && PB >= 1 && TM >= 1 && TN >= 1 && BM % 128 == 0, "bad fprop2 tile configuration");
};

__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint16_t* lds_dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff, 0, 0,
                                           0);
}

template <typename T, typename C, bool RED = false>
__global__ void __launch_bounds__(C::THREADS, 1)
fprop2_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y, Geo g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  constexpr int BM2 = C::BM, BN = C::BN, WM = C::WM, WN = C::WN, NW = C::NW, TM = C::TM, TN = C::TN;
  constexpr int PA = C::PA, PB = C::PB, S = C::S;
  constexpr int TA = BM2 * BK, TB = BN * BK;
  auto a_buf = [&](int b) { return lds + b * (TA + TB); };
  auto b_buf = [&](int b) { return lds + b * (TA + TB) + TA; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (g.m + BM2 - 1) / BM2, tiles_n = g.kout / BN;
  const int wg = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int bm = wg / tiles_n, bn = wg % tiles_n;
  const int row0 = bm * BM2, col0 = bn * BN;
  const int ohw = g.oh * g.ow;
  const int kw = g.ntaps * g.c;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)X, 0, __builtin_amdgcn_readfirstlane(g.xbytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)Wt, 0, __builtin_amdgcn_readfirstlane(g.wbytes), 0x00020000);

  // this lane's A rows: byte offset of (pixel origin, its 16-byte chunk) + tap validity bits
  uint32_t aoff[PA], amask[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int row = 8 * (i * NW + wave) + (lane >> 3);
    const int m = row0 + row;
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    aoff[i] = 0;
    amask[i] = 0;
    if (m < g.m) {
      const int nimg = (int)fdiv((uint32_t)m, g.div_ohw), rem = m - nimg * ohw;
      const int oy = (int)fdiv((uint32_t)rem, g.div_ow), ox = rem - oy * g.ow;
      const int ih0 = oy * g.ish, iw0 = ox * g.isw;
      aoff[i] = (uint32_t)((((nimg * g.h + ih0) * g.w + iw0) * g.c + 8 * chunk) * 2);
      uint32_t mk = 0;
      for (int t = 0; t < g.ntaps; ++t) {
        const int ih = ih0 + g.dh[t], iw = iw0 + g.dw[t];
        mk |= ((unsigned)ih < (unsigned)g.h && (unsigned)iw < (unsigned)g.w) ? (1u << t) : 0u;
      }
      amask[i] = mk;
    }
  }
  uint32_t boff[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int row = 8 * (i * NW + wave) + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    boff[i] = (uint32_t)(((col0 + row) * kw + 8 * chunk) * 2);
  }
  const int cblocks = g.c / BK;
  const int nk = g.ntaps * cblocks;

  auto issue = [&](int kt, int buf) {
    const int t = kt / cblocks, c0 = (kt - t * cblocks) * BK;
    const uint32_t toff = (uint32_t)(g.tapoff[t] + c0 * 2);
    uint16_t* adst = a_buf(buf);
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const uint32_t voff = ((amask[i] >> t) & 1u) ? aoff[i] + toff : 0x80000000u;  // OOB -> zeros
      bdma16(xr, voff, adst + (i * NW + wave) * 512);
    }
    uint16_t* bdst = b_buf(buf);
    const uint32_t k0b = (uint32_t)((t * g.c + c0) * 2);
#pragma unroll
    for (int i = 0; i < PB; ++i) bdma16(wr, boff[i] + k0b, bdst + (i * NW + wave) * 512);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int PER_STEP = PA + PB;
#pragma unroll
  for (int p = 0; p < S - 1; ++p)
    if (p < nk) issue(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = nk - 1 - kt < S - 2 ? nk - 1 - kt : S - 2;
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_STEP) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + S - 1 < nk) issue(kt + S - 1, (kt + S - 1) % S);
    const int cur = kt % S;
    const uint16_t* at = a_buf(cur);
    const uint16_t* bt = b_buf(cur);
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      s16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag_k(at, wm * (BM2 / WM) + 32 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = frag_k(bt, wn * (BN / WN) + 32 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma<T>(af[i], bf[j], acc[i][j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  float* cs = reinterpret_cast<float*>(lds);
  constexpr int BMT = BM2;
  float st1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, st2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int half = 0; half < BM2 / 128; ++half) {
    const int wr0 = wm * (BM2 / WM);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rb = wr0 + 32 * i;
      if (rb / 128 != half) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = rb - 128 * half + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          cs[rl * (BN + 4) + wn * (BN / WN) + 32 * j + (lane & 31)] = acc[i][j][r];
        }
    }
    __syncthreads();
    epi_chunk<T, BN, C::THREADS, 128, RED>(g, Y, cs, row0 + 128 * half, col0, tid, st1, st2);
    __syncthreads();
  }
  if (g.stats) stats_fold<BN, C::THREADS>(g, cs, bm, (g.m + BMT - 1) / BMT, col0, tid, st1, st2);
}

// ---------------------------------------------------------------------------------------------
// fprop3: persistent tap GEMM with the accumulators transposed (D[channel][pixel]) and the
// epilogue straight from registers.
//   * Workgroup (n, p) of a P x tiles_n grid owns output-channel block n and the contiguous
//     pixel-tile range [p T / P, (p+1) T / P): the LDS-DMA ring (fprop2's buffer-load staging) runs
//     across tile boundaries, so the next tile's operands stream in while the current tile's
//     last K-steps and its epilogue run — no per-tile pipeline fill / drain (the 9-step K loop
//     of a 64-channel 3x3 conv spends most of its time there otherwise).
//   * MFMA operands swapped (a = weight fragment, b = activation fragment): lane l holds, for
//     pixel (l & 31) of a 32-pixel subtile, 4 consecutive channels per register group, so the
//     epilogue writes 8-byte channel runs per pixel directly from the accumulators (no LDS
//     staging, no barrier) and the LDS ring is never repurposed.
//   * BN statistics of the output accumulate per lane over all the workgroup's tiles; one
//     cross-lane + cross-wave fold per workgroup writes statistics row p ([2][rows][kout];
//     rows >= P are zero-filled).
// ---------------------------------------------------------------------------------------------
template <int BM_, int BN_, int WM_, int WN_, int S_>
struct F3Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, S = S_;
  static constexpr int NW = WM * WN, THREADS = NW * 64;
  static constexpr int TPX = BM / WM / 32, TCH = BN / WN / 32;  // 32-pixel / 32-channel subtiles per wave
  static constexpr int PA = BM / 8 / NW, PB = BN / 8 / NW;
  static constexpr size_t LDS = (size_t)S * (BM * BK + BN * BK) * 2;
  static_assert(PA >= 1 && PB >= 1 && TPX >= 1 && TCH >= 1, "bad fprop3 tile configuration");
  static_assert(LDS >= (size_t)2 * WM * BN * 4, "statistics fold needs 2 x WM x BN floats of LDS");
};

struct F3Sched {
  int P, rows;  // workgroups per channel block (balanced split of the pixel tiles), stats rows
};

template <typename T, typename C, bool STATS>
__global__ void __launch_bounds__(C::THREADS, 1)
fprop3_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y, Geo g,
              F3Sched sc) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  constexpr int BMX = C::BM, BN = C::BN, WM = C::WM, WN = C::WN, NW = C::NW, TPX = C::TPX, TCH = C::TCH;
  constexpr int PA = C::PA, PB = C::PB, S = C::S;
  constexpr int TA = BMX * BK, TB = BN * BK;
  auto a_buf = [&](int b) { return lds + b * (TA + TB); };
  auto b_buf = [&](int b) { return lds + b * (TA + TB) + TA; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (g.m + BMX - 1) / BMX, tiles_n = g.kout / BN;
  const int wg = xcd_remap(blockIdx.x, sc.P * tiles_n);
  const int bn = wg % tiles_n, p = wg / tiles_n;
  const int t_begin = (int)((int64_t)p * tiles_m / sc.P), t_end = (int)((int64_t)(p + 1) * tiles_m / sc.P);
  const int ntile = max(0, t_end - t_begin);
  const int col0 = bn * BN;
  const int ohw = g.oh * g.ow;
  const int kw = g.ntaps * g.c;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)X, 0, __builtin_amdgcn_readfirstlane(g.xbytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)Wt, 0, __builtin_amdgcn_readfirstlane(g.wbytes), 0x00020000);
  const int cblocks = g.c / BK;
  const int nk = g.ntaps * cblocks;
  const int nsteps = ntile * nk;

  // issue-side state: this lane's A rows of the tile being ISSUED (recomputed at its first step)
  uint32_t aoff[PA], amask[PA];
  auto set_rows = [&](int tile) {
    const int row0 = tile * BMX;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int row = 8 * (i * NW + wave) + (lane >> 3);
      const int m = row0 + row;
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      aoff[i] = 0;
      amask[i] = 0;
      if (m < g.m) {
        const int nimg = (int)fdiv((uint32_t)m, g.div_ohw), rem = m - nimg * ohw;
        const int oy = (int)fdiv((uint32_t)rem, g.div_ow), ox = rem - oy * g.ow;
        const int ih0 = oy * g.ish, iw0 = ox * g.isw;
        aoff[i] = (uint32_t)((((nimg * g.h + ih0) * g.w + iw0) * g.c + 8 * chunk) * 2);
        uint32_t mk = 0;
        for (int t = 0; t < g.ntaps; ++t) {
          const int ih = ih0 + g.dh[t], iw = iw0 + g.dw[t];
          mk |= ((unsigned)ih < (unsigned)g.h && (unsigned)iw < (unsigned)g.w) ? (1u << t) : 0u;
        }
        amask[i] = mk;
      }
    }
  };
  uint32_t boff[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int row = 8 * (i * NW + wave) + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    boff[i] = (uint32_t)(((col0 + row) * kw + 8 * chunk) * 2);
  }
  int issue_tile = -1;
  auto issue = [&](int gs, int buf) {
    const int tl = gs / nk, kt = gs - tl * nk;
    if (tl != issue_tile) {
      issue_tile = tl;
      set_rows(t_begin + tl);
    }
    const int t = kt / cblocks, c0 = (kt - t * cblocks) * BK;
    const uint32_t toff = (uint32_t)(g.tapoff[t] + c0 * 2);
    uint16_t* adst = a_buf(buf);
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const uint32_t voff = ((amask[i] >> t) & 1u) ? aoff[i] + toff : 0x80000000u;
      bdma16(xr, voff, adst + (i * NW + wave) * 512);
    }
    uint16_t* bdst = b_buf(buf);
    const uint32_t k0b = (uint32_t)((t * g.c + c0) * 2);
#pragma unroll
    for (int i = 0; i < PB; ++i) bdma16(wr, boff[i] + k0b, bdst + (i * NW + wave) * 512);
  };

  // epilogue constants of this lane's channels: channel of register r of subtile ci =
  // chw + 32 ci + 8 (r >> 2) + 4 (lane >> 5) + (r & 3)
  const int chw = col0 + wn * (BN / WN);
  // (statistics registers only in the STATS instantiation: the others keep the occupancy)
  constexpr int SR = STATS ? 16 : 1;
  float st1[TCH][SR], st2[TCH][SR], sft[TCH][SR];
#pragma unroll
  for (int ci = 0; ci < TCH; ++ci)
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      st1[ci][r] = st2[ci][r] = 0.f;
      sft[ci][r] = (STATS && g.shift) ? g.shift[chw + 32 * ci + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3)] : 0.f;
    }

  f32x16 acc[TCH][TPX];
#pragma unroll
  for (int i = 0; i < TCH; ++i)
#pragma unroll
    for (int j = 0; j < TPX; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int PER_STEP = PA + PB;
#pragma unroll
  for (int q = 0; q < S - 1; ++q)
    if (q < nsteps) issue(q, q);
  int gs = 0;
  for (int tl = 0; tl < ntile; ++tl) {
  for (int kt = 0; kt < nk; ++kt, ++gs) {
    const int ahead = nsteps - 1 - gs < S - 2 ? nsteps - 1 - gs : S - 2;
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_STEP) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (gs + S - 1 < nsteps) issue(gs + S - 1, (gs + S - 1) % S);
    const int cur = gs % S;
    const uint16_t* at = a_buf(cur);
    const uint16_t* bt = b_buf(cur);
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      s16x8 wf[TCH], xf[TPX];
#pragma unroll
      for (int i = 0; i < TCH; ++i) wf[i] = frag_k(bt, wn * (BN / WN) + 32 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TPX; ++j) xf[j] = frag_k(at, wm * (BMX / WM) + 32 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TCH; ++i)
#pragma unroll
        for (int j = 0; j < TPX; ++j) acc[i][j] = mfma<T>(wf[i], xf[j], acc[i][j]);
    }
  }
    // ---- tile epilogue from registers (no LDS): 8-byte channel runs per pixel ----
    const int tile = t_begin + tl;
#pragma unroll
    for (int j = 0; j < TPX; ++j) {
      const int m = tile * BMX + wm * (BMX / WM) + 32 * j + (lane & 31);
      if (m >= g.m) continue;
      int64_t pix = m;
      if (!g.ident) {
        const int nimg = (int)fdiv((uint32_t)m, g.div_ohw), rem = m - nimg * ohw;
        const int oy = (int)fdiv((uint32_t)rem, g.div_ow), ox = rem - oy * g.ow;
        pix = ((int64_t)nimg * g.oht + oy * g.osh + g.oph) * g.owt + ox * g.osw + g.opw;
      }
#pragma unroll
      for (int i = 0; i < TCH; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ch = chw + 32 * i + 8 * q + 4 * (lane >> 5);
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
          if (g.scale || g.bias) {
            const float4 s4 = g.scale ? *reinterpret_cast<const float4*>(g.scale + ch) : make_float4(1.f, 1.f, 1.f, 1.f);
            const float4 b4 = g.bias ? *reinterpret_cast<const float4*>(g.bias + ch) : make_float4(0.f, 0.f, 0.f, 0.f);
            v[0] = fmaf(v[0], s4.x, b4.x); v[1] = fmaf(v[1], s4.y, b4.y);
            v[2] = fmaf(v[2], s4.z, b4.z); v[3] = fmaf(v[3], s4.w, b4.w);
          }
          const int64_t off = pix * g.kout + ch;
          if (g.res) {
            const uint2 rr = *reinterpret_cast<const uint2*>(g.res + off);
            v[0] += to_f(T{(uint16_t)(rr.x & 0xffffu)}); v[1] += to_f(T{(uint16_t)(rr.x >> 16)});
            v[2] += to_f(T{(uint16_t)(rr.y & 0xffffu)}); v[3] += to_f(T{(uint16_t)(rr.y >> 16)});
          }
          if (g.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          if (g.mask) {
            const uint2 mm = *reinterpret_cast<const uint2*>(g.mask + off);
            const uint16_t mk[4] = {(uint16_t)(mm.x & 0xffffu), (uint16_t)(mm.x >> 16), (uint16_t)(mm.y & 0xffffu),
                                    (uint16_t)(mm.y >> 16)};
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = to_f(T{mk[e]}) > 0.f ? v[e] : 0.f;
          }
          uint2 o;
          o.x = (uint32_t)from_f<T>(v[0]).x | ((uint32_t)from_f<T>(v[1]).x << 16);
          o.y = (uint32_t)from_f<T>(v[2]).x | ((uint32_t)from_f<T>(v[3]).x << 16);
          *reinterpret_cast<uint2*>(Y + off) = o;
          if constexpr (STATS) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float d = v[e] - sft[i][4 * q + e];
              st1[i][4 * q + e] += d;
              st2[i][4 * q + e] = fmaf(d, d, st2[i][4 * q + e]);
            }
          }
        }
    }
#pragma unroll
    for (int i = 0; i < TCH; ++i)
#pragma unroll
      for (int j = 0; j < TPX; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  }
  if constexpr (!STATS) return;
  // ---- statistics: fold the 32 pixels of each half-wave (xor shuffles), then the WM wave rows
  // sharing a channel range through LDS in a fixed order, one row per workgroup ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TCH; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int sh = 1; sh < 32; sh <<= 1) {
        st1[i][r] += __shfl_xor(st1[i][r], sh);
        st2[i][r] += __shfl_xor(st2[i][r], sh);
      }
    }
  float* red = reinterpret_cast<float*>(lds);  // [2][WM][BN]
  if ((lane & 31) == 0) {
#pragma unroll
    for (int i = 0; i < TCH; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = wn * (BN / WN) + 32 * i + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
        red[(0 * WM + wm) * BN + c] = st1[i][r];
        red[(1 * WM + wm) * BN + c] = st2[i][r];
      }
  }
  __syncthreads();
  for (int i = tid; i < 2 * BN; i += C::THREADS) {
    const int which = i / BN, c = i % BN;
    float v = 0.f;
    for (int w = 0; w < WM; ++w) v += red[(which * WM + w) * BN + c];
    g.stats[((int64_t)which * sc.rows + p) * g.kout + col0 + c] = v;
    // rows past the schedule's P are zero (the finalize sums every row)
    for (int r2 = p + sc.P; r2 < sc.rows; r2 += sc.P) g.stats[((int64_t)which * sc.rows + r2) * g.kout + col0 + c] = 0.f;
  }
}

// =============================================================================================
// wgrad
// =============================================================================================
constexpr int WG_THREADS = 256, WG_BK = plan::kWgradBK;

// quarter-of-a-bank-row swizzle for pixel-major images read by ds_read_b64_tr_b16: the four
// consecutive rows a 16-lane group reads land in four different 64-byte bank quarters
template <int W>
__device__ __forceinline__ int tr_swz(int r) {
  return W == 64 ? ((r >> 1) & 1) : (r & 3);
}

__device__ __forceinline__ s16x4 tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)((__attribute__((address_space(3))) uint16_t*)p));
}

// fragment of a 32-column subtile (MFMA rows) at reduction step kk from a [64][W] pixel-major
// image: lane (g, q, p) reads 4 consecutive columns of rows kb + q and kb + 4 + q transposed
template <int W>
__device__ __forceinline__ s16x8 frag_t(const uint16_t* tile, int colbase, int kk, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int kb = 16 * kk + 8 * (g >> 1);
  const int col = colbase + 16 * (g & 1) + 4 * p;
  const int ck = col >> 3, off = col & 7;
  const int r0 = kb + q, r1 = kb + 4 + q;
  const s16x4 lo = tr_read(tile + r0 * W + ((ck ^ (tr_swz<W>(r0) << 2)) << 3) + off);
  const s16x4 hi = tr_read(tile + r1 * W + ((ck ^ (tr_swz<W>(r1) << 2)) << 3) + off);
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// BMW x BNW output tile (kout rows x channel columns of one tap), 4 waves in 2 x 2
template <typename T, int BMW, int BNW>
__global__ void __launch_bounds__(WG_THREADS, BMW == 128 ? 1 : 2)
wgrad_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ DY, float* __restrict__ part, Geo g,
             int chunk) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  constexpr int TA = WG_BK * BMW, TB = WG_BK * BNW;
  constexpr int TM = BMW / 2 / 32, TN = BNW / 2 / 32;
  auto a_buf = [&](int b) { return lds + b * (TA + TB); };
  auto b_buf = [&](int b) { return lds + b * (TA + TB) + TA; };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_m = g.kout / BMW, tiles_n = g.ntaps * g.c / BNW;
  const int tiles = tiles_m * tiles_n;
  const int tile = xcd_remap(blockIdx.x, tiles), split = blockIdx.y;
  const int bm = tile / tiles_n, bn = tile % tiles_n;
  const int k0 = bm * BMW;                       // output-channel rows
  const int j0 = bn * BNW;                       // (tap, channel) columns
  const int t = j0 / g.c, c0 = j0 - t * g.c;
  const int dh = g.dh[t], dw = g.dw[t];
  const int ohw = g.oh * g.ow;
  const int p_begin = split * chunk;
  const int p_end = min(g.m, p_begin + chunk);
  const int nk = (p_end - p_begin + WG_BK - 1) / WG_BK;

  // DMA pieces: 1 KB = (1024 / row bytes) pixel rows of one image
  constexpr int RA = 512 / BMW, RB = 512 / BNW;  // rows per piece
  auto issue = [&](int kt, int buf) {
    const int pbase = p_begin + kt * WG_BK;
    uint16_t* adst = a_buf(buf);
#pragma unroll
    for (int i = 0; i < TA / 512 / 4; ++i) {
      const int piece = i * 4 + wave;
      const int row = piece * RA + lane / (BMW / 8);
      const int slot = lane % (BMW / 8);
      const int c = slot ^ (tr_swz<BMW>(row) << 2);
      const int p = pbase + row;
      const uintptr_t real = (uintptr_t)(DY + (int64_t)p * g.kout + k0 + 8 * c);
      const uintptr_t zero = (uintptr_t)(g_zero + 8 * (c & 7));
      const uintptr_t msk = (uintptr_t)0 - (uintptr_t)(p < p_end);
      dma16((const uint16_t*)((real & msk) | (zero & ~msk)), adst + piece * 512);
    }
    uint16_t* bdst = b_buf(buf);
#pragma unroll
    for (int i = 0; i < TB / 512 / 4; ++i) {
      const int piece = i * 4 + wave;
      const int row = piece * RB + lane / (BNW / 8);
      const int slot = lane % (BNW / 8);
      const int c = slot ^ (tr_swz<BNW>(row) << 2);
      const int p = pbase + row;
      const int nimg = p / ohw, rem = p - nimg * ohw;
      const int oy = rem / g.ow, ox = rem - oy * g.ow;
      const int ih = oy * g.ish + dh, iw = ox * g.isw + dw;
      const bool ok = p < p_end && (unsigned)ih < (unsigned)g.h && (unsigned)iw < (unsigned)g.w;
      const uintptr_t real = (uintptr_t)(X + (((int64_t)nimg * g.h + ih) * g.w + iw) * g.c + c0 + 8 * c);
      const uintptr_t zero = (uintptr_t)(g_zero + 8 * (c & 7));
      const uintptr_t msk = (uintptr_t)0 - (uintptr_t)ok;
      dma16((const uint16_t*)((real & msk) | (zero & ~msk)), bdst + piece * 512);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // same 3-stage ring as fprop (counted vmcnt, raw barrier)
  constexpr int PER_STEP = TA / 512 / 4 + TB / 512 / 4;
  if (nk > 0) issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) issue(kt + 2, (kt + 2) % STAGES);
    const int cur = kt % STAGES;
    const uint16_t* at = a_buf(cur);
    const uint16_t* bt = b_buf(cur);
#pragma unroll
    for (int kk = 0; kk < WG_BK / 16; ++kk) {
      s16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag_t<BMW>(at, wm * (BMW / 2) + 32 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = frag_t<BNW>(bt, wn * (BNW / 2) + 32 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma<T>(af[i], bf[j], acc[i][j]);
    }
  }

  // fp32 partial tile straight from the accumulators: each register row is 32 consecutive
  // columns across the lanes (128-byte segments)
  const int64_t ldp = (int64_t)g.ntaps * g.c;
  float* dst = part + (int64_t)split * g.kout * ldp;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = k0 + wm * (BMW / 2) + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = j0 + wn * (BNW / 2) + 32 * j + (lane & 31);
        dst[(int64_t)row * ldp + col] = acc[i][j][r];
      }
}

// wgrad2: the same split-pixel weight gradient with cheap operand addressing — buffer_load ...
// lds through range-checked descriptors (out-of-range offsets zero-fill), DY offsets advanced by a
// uniform stride per K-step, the pixel -> (image, row, col) decomposition of the X rows by
// FastDiv (4 VALU per divide instead of ~30) — and W x W tiles per wave that feed 2 x 2 MFMAs
// per fragment pair.  BMW x BNW output tile, 4 waves in WMW x WNW.
template <typename T, int BMW, int BNW, int WMW, int WNW>
__global__ void __launch_bounds__(WG_THREADS, 1)
wgrad2_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ DY, float* __restrict__ part, Geo g,
              int chunk, int dybytes) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  static_assert(WMW * WNW == 4, "wgrad2 runs 4 waves");
  constexpr int TA = WG_BK * BMW, TB = WG_BK * BNW;
  constexpr int TM = BMW / WMW / 32, TN = BNW / WNW / 32;
  constexpr int PA = TA / 512 / 4, PB = TB / 512 / 4;  // 1-KiB DMA pieces per wave per step
  auto a_buf = [&](int b) { return lds + b * (TA + TB); };
  auto b_buf = [&](int b) { return lds + b * (TA + TB) + TA; };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;
  const int tiles_m = g.kout / BMW, tiles_n = g.ntaps * g.c / BNW;
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n), split = blockIdx.y;
  const int bm = tile / tiles_n, bn = tile % tiles_n;
  const int k0 = bm * BMW;
  const int j0 = bn * BNW;
  const int t = j0 / g.c, c0 = j0 - t * g.c;
  const int dh = g.dh[t], dw = g.dw[t];
  const int ohw = g.oh * g.ow;
  const int p_begin = split * chunk;
  const int p_end = min(g.m, p_begin + chunk);
  const int nk = (p_end - p_begin + WG_BK - 1) / WG_BK;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)X, 0, __builtin_amdgcn_readfirstlane(g.xbytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)DY, 0, __builtin_amdgcn_readfirstlane(dybytes), 0x00020000);

  constexpr int RA = 512 / BMW, RB = 512 / BNW;  // pixel rows per piece
  // A (DY) pieces: fixed column chunk per lane, pixel row advanced by WG_BK per step
  int arow[PA];
  uint32_t aoff[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int piece = i * 4 + wave;
    const int row = piece * RA + lane / (BMW / 8);
    const int cc = (lane % (BMW / 8)) ^ (tr_swz<BMW>(row) << 2);
    arow[i] = row;
    aoff[i] = (uint32_t)(((p_begin + row) * g.kout + k0 + 8 * cc) * 2);
  }
  const uint32_t astep = (uint32_t)(WG_BK * g.kout * 2);
  int brow[PB], bcol[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int piece = i * 4 + wave;
    brow[i] = piece * RB + lane / (BNW / 8);
    bcol[i] = 8 * ((lane % (BNW / 8)) ^ (tr_swz<BNW>(brow[i]) << 2));
  }

  auto issue = [&](int kt, int buf) {
    const int pbase = p_begin + kt * WG_BK;
    uint16_t* adst = a_buf(buf);
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const uint32_t voff = pbase + arow[i] < p_end ? aoff[i] + (uint32_t)kt * astep : 0x80000000u;
      bdma16(dr, voff, adst + (i * 4 + wave) * 512);
    }
    uint16_t* bdst = b_buf(buf);
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int p = pbase + brow[i];
      const int nimg = (int)fdiv((uint32_t)p, g.div_ohw), rem = p - nimg * ohw;
      const int oy = (int)fdiv((uint32_t)rem, g.div_ow), ox = rem - oy * g.ow;
      const int ih = oy * g.ish + dh, iw = ox * g.isw + dw;
      const bool ok = p < p_end && (unsigned)ih < (unsigned)g.h && (unsigned)iw < (unsigned)g.w;
      const uint32_t voff = ok ? (uint32_t)((((nimg * g.h + ih) * g.w + iw) * g.c + c0 + bcol[i]) * 2) : 0x80000000u;
      bdma16(xr, voff, bdst + (i * 4 + wave) * 512);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int PER_STEP = PA + PB;
  if (nk > 0) issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) issue(kt + 2, (kt + 2) % STAGES);
    const int cur = kt % STAGES;
    const uint16_t* at = a_buf(cur);
    const uint16_t* bt = b_buf(cur);
#pragma unroll
    for (int kk = 0; kk < WG_BK / 16; ++kk) {
      s16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag_t<BMW>(at, wm * (BMW / WMW) + 32 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = frag_t<BNW>(bt, wn * (BNW / WNW) + 32 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma<T>(af[i], bf[j], acc[i][j]);
    }
  }

  const int64_t ldp = (int64_t)g.ntaps * g.c;
  float* dst = part + (int64_t)split * g.kout * ldp;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = k0 + wm * (BMW / WMW) + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = j0 + wn * (BNW / WNW) + 32 * j + (lane & 31);
        dst[(int64_t)row * ldp + col] = acc[i][j][r];
      }
}

// fixed-order sum of the split partials: a block owns 16 consecutive 8-element vectors and its 16
// thread groups each sum every 16th split, folded in LDS in a fixed order (S / 16 loads per
// thread and n / 128 blocks — one thread per vector over all S splits left the chip idle)
template <typename TO>
__global__ void __launch_bounds__(256) wgrad_reduce(const float* __restrict__ part, int splits, int64_t n,
                                                    TO* __restrict__ out) {
  __shared__ float red[16][16 * 8 + 4];
  const int v = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t i = ((int64_t)blockIdx.x * 16 + v) * 8;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < n)
    for (int q = grp; q < splits; q += 16) {
      float t8[8];
      Vec8<float>::load(t8, part + (int64_t)q * n + i);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += t8[k];
    }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[grp][v * 8 + k] = a[k];
  __syncthreads();
  if (grp != 0 || i >= n) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = 0.f;
  for (int g2 = 0; g2 < 16; ++g2)
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += red[g2][v * 8 + k];
  Vec8<TO>::store(out + i, a);
}

using plan::WgPlan;

}  // namespace conv

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

bool conv_tap_supported(const ConvTapArgs& a) {
  if (a.dtype != kBF16 && a.dtype != kF16) return false;
  if (a.c % 64 || a.kout % 64 || a.c <= 0 || a.kout <= 0) return false;
  if (a.ntaps < 1 || a.ntaps > kConvMaxTaps) return false;
  if (a.n <= 0 || a.oh <= 0 || a.ow <= 0) return false;
  if ((int64_t)a.n * a.oh * a.ow >= (1ll << 31) || (int64_t)a.n * a.ih * a.iw >= (1ll << 31)) return false;
  if ((a.scale && !aligned16(a.scale)) || (a.bias && !aligned16(a.bias)) || (a.residual && !aligned16(a.residual)) ||
      (a.mask && !aligned16(a.mask)))
    return false;
  return aligned16(a.in) && aligned16(a.wt) && aligned16(a.out);
}

// fprop tile configurations (APEX_AMD_CONV_CFG=<index> forces one, for A/B sweeps):
//   0: BN 128, 8 waves 4x2 (64x64 each), 3 stages   1: BN 64, 8 waves 8x1 (32x64), 3 stages
//   2: BN 128, 4 waves 2x2 (128x64), 3 stages         3: BN 64, 4 waves 4x1 (64x64), 3 stages
//   4: BN 128, 8 waves, 2 stages                       5: BN 64, 8 waves, 2 stages
//   6: BN 256, 8 waves 2x4 (128x64), 2 stages
using FC0 = conv::FCfg<128, 4, 2, 3>;
using FC1 = conv::FCfg<64, 8, 1, 3>;
using FC2 = conv::FCfg<128, 2, 2, 3>;
using FC3 = conv::FCfg<64, 4, 1, 3>;
using FC4 = conv::FCfg<128, 4, 2, 2>;
using FC5 = conv::FCfg<64, 8, 1, 2>;
using FC6 = conv::FCfg<256, 2, 4, 2>;
// fprop2 (BM, BN, WM x WN waves, stages)
using F7 = conv::F2Cfg<256, 64, 8, 1, 2>;
using F8 = conv::F2Cfg<256, 64, 4, 1, 2>;
using F9 = conv::F2Cfg<256, 128, 4, 2, 2>;
using F10 = conv::F2Cfg<128, 128, 2, 2, 3>;
using F11 = conv::F2Cfg<128, 128, 2, 2, 2>;
using F12 = conv::F2Cfg<256, 256, 2, 4, 2>;
using F13 = conv::F2Cfg<128, 256, 2, 4, 2>;
// fprop3 (persistent, transposed accumulators): BM pixels, BN channels, WM x WN waves, stages
using F14 = conv::F3Cfg<256, 64, 8, 1, 2>;
using F15 = conv::F3Cfg<128, 64, 4, 1, 2>;
using F16 = conv::F3Cfg<128, 128, 4, 2, 2>;
using F17 = conv::F3Cfg<128, 128, 2, 2, 2>;
using F18 = conv::F3Cfg<256, 128, 4, 2, 2>;
using F19 = conv::F3Cfg<128, 256, 2, 4, 2>;
using F20 = conv::F3Cfg<256, 64, 4, 1, 2>;

static int g_forced_cfg = [] {
  const char* e = std::getenv("APEX_AMD_CONV_CFG");
  return e ? std::atoi(e) : -1;
}();

void conv_force_fprop_cfg(int cfg) { g_forced_cfg = cfg; }

static int fprop_cfg(const ConvTapArgs& a, int cus) { return plan::conv_fprop_cfg(a, cus, g_forced_cfg); }

// the spatial-tile 64-channel kernel (conv3x3_sp.hip): forced as configuration 21, else taken
// wherever it applies unless another configuration is forced
constexpr int kSpCfg = 21;
static bool use_sp(const ConvTapArgs& a) {
  if (a.red_x) return false;  // the BN backward reduction epilogue is the tap kernels' (epi_chunk)
  if (g_forced_cfg == kSpCfg) return conv_sp_supported(a);
  return g_forced_cfg < 0 && conv_sp_default(a);
}

// the halo-tile kernel (conv3x3_halo.hip) for stride-1 3x3 at C % 64, K % 128 unless another
// configuration is forced
static bool use_hfp(const ConvTapArgs& a) { return !a.red_x && g_forced_cfg < 0 && conv_hfp_default(a); }

int conv_tap_stats_tiles(const ConvTapArgs& a, int cus) {
  if (use_sp(a)) return conv_sp_grid(a, cus);
  if (use_hfp(a)) return conv_hfp_stats_rows(a, cus);
  const int bm = plan::conv_fprop_bm(fprop_cfg(a, cus));
  return (int)(((int64_t)a.n * a.oh * a.ow + bm - 1) / bm);
}

void conv_tap_fprop(const ConvTapArgs& a, int cus, hipStream_t s) {
  if (!conv_tap_supported(a)) throw std::runtime_error("conv_tap_fprop: unsupported shape / dtype / alignment");
  if (use_sp(a)) {
    conv_sp_fprop(a, cus, s);
    return;
  }
  if (use_hfp(a)) {
    conv_hfp(a, nullptr, cus, s);
    return;
  }
  const conv::Geo g = conv::make_geo(a);
  int cfg = fprop_cfg(a, cus);
  // the reduction epilogue lives in epi_chunk (fprop / fprop2); the persistent fprop3 writes from
  // registers: take the fprop2 choice of the shape instead
  if (a.red_x && cfg >= 14) cfg = plan::conv_fprop_cfg(a, cus, -1);
  if (a.red_x && (!a.stats || a.stats_shift || a.mask || a.residual || a.relu || a.scale || a.bias))
    throw std::runtime_error("conv_tap_fprop: the BN backward reduction takes stats only (no other epilogue)");
  dispatch_16(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    auto go = [&](auto cfg_tag) {
      using C = decltype(cfg_tag);
      const int64_t tiles_m = (g.m + conv::BM - 1) / conv::BM;
      const unsigned grid = (unsigned)(tiles_m * (a.kout / C::BN));
      if (a.red_x)
        hipLaunchKernelGGL((conv::fprop_kernel<T, C, true>), dim3(grid), dim3(C::THREADS), C::LDS, s,
                           (const uint16_t*)a.in, (const uint16_t*)a.wt, (uint16_t*)a.out, g);
      else
        hipLaunchKernelGGL((conv::fprop_kernel<T, C>), dim3(grid), dim3(C::THREADS), C::LDS, s, (const uint16_t*)a.in,
                           (const uint16_t*)a.wt, (uint16_t*)a.out, g);
    };
    auto go2 = [&](auto cfg_tag) {
      using C = decltype(cfg_tag);
      const int64_t tiles_m = (g.m + C::BM - 1) / C::BM;
      const unsigned grid = (unsigned)(tiles_m * (a.kout / C::BN));
      if (a.red_x)
        hipLaunchKernelGGL((conv::fprop2_kernel<T, C, true>), dim3(grid), dim3(C::THREADS), C::LDS, s,
                           (const uint16_t*)a.in, (const uint16_t*)a.wt, (uint16_t*)a.out, g);
      else
        hipLaunchKernelGGL((conv::fprop2_kernel<T, C>), dim3(grid), dim3(C::THREADS), C::LDS, s,
                           (const uint16_t*)a.in, (const uint16_t*)a.wt, (uint16_t*)a.out, g);
    };
    auto go3 = [&](auto cfg_tag) {
      using C = decltype(cfg_tag);
      const int64_t tiles_m = (g.m + C::BM - 1) / C::BM, tiles_n = a.kout / C::BN;
      const int per_cu = std::max(1, (int)((160 * 1024) / C::LDS));
      int64_t P = std::max<int64_t>(1, (int64_t)cus * per_cu / tiles_n);
      P = std::min(P, tiles_m);
      conv::F3Sched sc{(int)P, (int)tiles_m};
      if (g.stats)
        hipLaunchKernelGGL((conv::fprop3_kernel<T, C, true>), dim3((unsigned)(P * tiles_n)), dim3(C::THREADS), C::LDS,
                           s, (const uint16_t*)a.in, (const uint16_t*)a.wt, (uint16_t*)a.out, g, sc);
      else
        hipLaunchKernelGGL((conv::fprop3_kernel<T, C, false>), dim3((unsigned)(P * tiles_n)), dim3(C::THREADS), C::LDS,
                           s, (const uint16_t*)a.in, (const uint16_t*)a.wt, (uint16_t*)a.out, g, sc);
    };
    switch (cfg) {
      case 0: go(FC0{}); break;
      case 1: go(FC1{}); break;
      case 2: go(FC2{}); break;
      case 3: go(FC3{}); break;
      case 4: go(FC4{}); break;
      case 5: go(FC5{}); break;
      case 6: go(FC6{}); break;
      case 7: go2(F7{}); break;
      case 8: go2(F8{}); break;
      case 9: go2(F9{}); break;
      case 10: go2(F10{}); break;
      case 11: go2(F11{}); break;
      case 12: go2(F12{}); break;
      case 13: go2(F13{}); break;
      case 14: go3(F14{}); break;
      case 15: go3(F15{}); break;
      case 16: go3(F16{}); break;
      case 17: go3(F17{}); break;
      case 18: go3(F18{}); break;
      case 19: go3(F19{}); break;
      default: go3(F20{}); break;
    }
  }, "conv_tap_fprop");
  check_launch("conv_tap_fprop");
}

bool conv_wgrad_supported(const ConvTapArgs& a) {
  if (!conv_tap_supported(a)) return false;
  return a.osh == 1 && a.osw == 1 && a.oph == 0 && a.opw == 0 && a.oht == a.oh && a.owt == a.ow;
}

static int g_wgrad_variant = [] {
  const char* e = std::getenv("APEX_AMD_WGRAD_VARIANT");
  return e ? std::atoi(e) : -1;
}();

void conv_force_wgrad_variant(int v) { g_wgrad_variant = v; }

// variant for this shape: forced (A/B) or the measured default — wgrad2 128 x 64 (variant 3),
// the best native tile at every ResNet-50 3x3 shape (profiles/wgrad3x3_variants_r04.jsonl; it
// beats MIOpen only at 28 x 28 x 128, where ops/conv.py tap_route routes it)
static int wgrad_variant(const ConvTapArgs& a) {
  if (g_wgrad_variant >= 0) return plan::conv_wgrad_variant_ok(a, g_wgrad_variant) ? g_wgrad_variant : 0;
  return plan::conv_wgrad_variant_ok(a, 3) ? 3 : 0;
}

// the halo-tile kernel (conv3x3_wgrad.hip) wherever it applies, unless a tap-kernel variant is forced
static bool use_halo_wgrad(const ConvTapArgs& a) {
  if (g_wgrad_variant >= 0 && g_wgrad_variant != kWgradHalo) return false;
  return conv_hwgrad_supported(a);
}

int64_t conv_wgrad_workspace_floats(const ConvTapArgs& a, int cus) {
  if (use_halo_wgrad(a)) return conv_hwgrad_workspace_floats(a, cus);
  const conv::WgPlan p = plan::conv_wgrad(a, cus, wgrad_variant(a));
  return (int64_t)p.splits * a.kout * a.ntaps * a.c;
}

void conv_wgrad(const ConvTapArgs& a, const void* dy, void* dw_out, int out_dtype, float* ws, int cus,
                hipStream_t s) {
  if (!conv_wgrad_supported(a) || !aligned16(dy) || !aligned16(dw_out) || !aligned16(ws))
    throw std::runtime_error("conv_wgrad: unsupported shape / dtype / alignment");
  if (use_halo_wgrad(a)) {
    conv_hwgrad(a, dy, dw_out, out_dtype, ws, cus, s);
    return;
  }
  const conv::Geo g = conv::make_geo(a);
  const int v = wgrad_variant(a);
  const conv::WgPlan p = plan::conv_wgrad(a, cus, v);
  const int dybytes = (int)std::min<int64_t>((int64_t)g.m * a.kout * 2, (1ll << 31) - 1);
  dispatch_16(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    auto go = [&](auto kern, int bm, int bn) {
      const size_t lds = (size_t)conv::STAGES * conv::WG_BK * (bm + bn) * 2;
      hipLaunchKernelGGL(kern, dim3(p.tiles, p.splits), dim3(conv::WG_THREADS), lds, s, (const uint16_t*)a.in,
                         (const uint16_t*)dy, ws, g, p.chunk);
    };
    auto go2 = [&](auto kern, int bm, int bn) {
      const size_t lds = (size_t)conv::STAGES * conv::WG_BK * (bm + bn) * 2;
      hipLaunchKernelGGL(kern, dim3(p.tiles, p.splits), dim3(conv::WG_THREADS), lds, s, (const uint16_t*)a.in,
                         (const uint16_t*)dy, ws, g, p.chunk, dybytes);
    };
    switch (v) {
      case 1: go2(conv::wgrad2_kernel<T, 64, 64, 2, 2>, 64, 64); break;
      case 2: go2(conv::wgrad2_kernel<T, 128, 128, 2, 2>, 128, 128); break;
      case 3: go2(conv::wgrad2_kernel<T, 128, 64, 2, 2>, 128, 64); break;
      case 4: go2(conv::wgrad2_kernel<T, 64, 128, 2, 2>, 64, 128); break;
      default:
        if (p.bm == 128) go(conv::wgrad_kernel<T, 128, 128>, 128, 128);
        else go(conv::wgrad_kernel<T, 64, 64>, 64, 64);
    }
  }, "conv_wgrad");
  const int64_t n = (int64_t)a.kout * a.ntaps * a.c;
  const int64_t grid = (n / 8 + 15) / 16;
  dispatch_float(out_dtype, [&](auto tag) {
    using TO = typename decltype(tag)::type;
    hipLaunchKernelGGL((conv::wgrad_reduce<TO>), dim3((unsigned)grid), dim3(256), 0, s, (const float*)ws, p.splits, n,
                       (TO*)dw_out);
  }, "conv_wgrad out");
  check_launch("conv_wgrad");
}

}  // namespace apex_amd
