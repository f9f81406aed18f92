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
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"

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
};

inline Geo make_geo(const ConvTapArgs& a) {
  Geo g;
  g.n = a.n; g.h = a.ih; g.w = a.iw; g.c = a.c; g.oh = a.oh; g.ow = a.ow; g.oht = a.oht; g.owt = a.owt;
  g.kout = a.kout; g.ish = a.ish; g.isw = a.isw; g.osh = a.osh; g.osw = a.osw; g.oph = a.oph; g.opw = a.opw;
  g.ntaps = a.ntaps;
  g.m = a.n * a.oh * a.ow;
  for (int t = 0; t < kConvMaxTaps; ++t) {
    g.dh[t] = t < a.ntaps ? a.dh[t] : 0;
    g.dw[t] = t < a.ntaps ? a.dw[t] : 0;
  }
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
constexpr int BM = 256, BK = 64, THREADS = 512;

template <int BN> struct Layout;
template <> struct Layout<256> { static constexpr int WM = 2, WN = 4; };
template <> struct Layout<128> { static constexpr int WM = 4, WN = 2; };
template <> struct Layout<64> { static constexpr int WM = 8, WN = 1; };

template <int BN>
constexpr size_t fprop_lds_bytes() {
  constexpr size_t ops = (size_t)2 * (BM * BK + BN * BK) * 2;
  constexpr size_t epi = (size_t)128 * (BN + 4) * 4;
  return ops > epi ? ops : epi;
}

// k-major fragment of a 32-row subtile at k-step kk from a swizzled [rows][64] image
__device__ __forceinline__ s16x8 frag_k(const uint16_t* tile, int rowbase, int kk, int lane) {
  const int row = rowbase + (lane & 31);
  const int c = (2 * kk + (lane >> 5)) ^ ((row >> 1) & 7);
  return *reinterpret_cast<const s16x8*>(tile + row * BK + 8 * c);
}

template <typename T, int BN>
__global__ void __launch_bounds__(THREADS, 1)
fprop_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y, Geo g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  constexpr int WM = Layout<BN>::WM, WN = Layout<BN>::WN;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
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

  // this lane's 4 A rows (fixed for the whole K loop): image base + input origin of the pixel
  int64_t abase[4];
  int aih[4], aiw[4], asrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (i * 8 + wave) + (lane >> 3);
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
    for (int i = 0; i < 4; ++i) {
      const int ih = aih[i] + dh, iw = aiw[i] + dw;
      const bool ok = (unsigned)ih < (unsigned)g.h && (unsigned)iw < (unsigned)g.w;
      const uint16_t* src = ok ? X + abase[i] + ((int64_t)ih * g.w + iw) * g.c + c0 + asrc[i] : g_zero + asrc[i];
      dma16(src, adst + (i * 8 + wave) * 512);
    }
    uint16_t* bdst = b_buf(buf);
    const int64_t k0 = (int64_t)t * g.c + c0;
#pragma unroll
    for (int i = 0; i < BN / 64; ++i) {
      const int j = i * 8 + wave;
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

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
    const uint16_t* at = a_buf(cur);
    const uint16_t* bt = b_buf(cur);
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      s16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag_k(at, wm * (BM / WM) + 32 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = frag_k(bt, wn * (BN / WN) + 32 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma<T>(af[i], bf[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: two 128-row halves staged as fp32 through LDS, 16-byte row stores ----
  constexpr int CST = BN + 4;
  constexpr int CPR = BN / 8;            // 8-column chunks per row
  constexpr int RP = THREADS / CPR;      // rows per pass
  float* cs = reinterpret_cast<float*>(lds);
  const int ch = tid % CPR, rsub = tid / CPR;
  const int gc = col0 + ch * 8;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int wr0 = wm * (BM / WM);
    if (wr0 / 128 == half) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rl = wr0 - 128 * half + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            cs[rl * CST + wn * (BN / WN) + 32 * j + (lane & 31)] = acc[i][j][r];
          }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 128 / RP; ++it) {
      const int rl = rsub + RP * it;
      const int m = row0 + half * 128 + rl;
      if (m < g.m) {
        const int nimg = m / ohw, rem = m - nimg * ohw;
        const int oy = rem / g.ow, ox = rem - oy * g.ow;
        const int64_t pix = ((int64_t)nimg * g.oht + oy * g.osh + g.oph) * g.owt + ox * g.osw + g.opw;
        float v[8];
        const float4 lo = *reinterpret_cast<const float4*>(cs + rl * CST + ch * 8);
        const float4 hi = *reinterpret_cast<const float4*>(cs + rl * CST + ch * 8 + 4);
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        Vec8<T>::store(reinterpret_cast<T*>(Y) + pix * g.kout + gc, v);
      }
    }
    __syncthreads();
  }
}

// =============================================================================================
// wgrad
// =============================================================================================
constexpr int WG_THREADS = 256, WG_BK = 64;

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
__global__ void __launch_bounds__(WG_THREADS, 2)
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
      const uint16_t* src = p < p_end ? DY + (int64_t)p * g.kout + k0 + 8 * c : g_zero + 8 * (c & 7);
      dma16(src, adst + piece * 512);
    }
    uint16_t* bdst = b_buf(buf);
#pragma unroll
    for (int i = 0; i < TB / 512 / 4; ++i) {
      const int piece = i * 4 + wave;
      const int row = piece * RB + lane / (BNW / 8);
      const int slot = lane % (BNW / 8);
      const int c = slot ^ (tr_swz<BNW>(row) << 2);
      const int p = pbase + row;
      const uint16_t* src = g_zero + 8 * (c & 7);
      if (p < p_end) {
        const int nimg = p / ohw, rem = p - nimg * ohw;
        const int oy = rem / g.ow, ox = rem - oy * g.ow;
        const int ih = oy * g.ish + dh, iw = ox * g.isw + dw;
        if ((unsigned)ih < (unsigned)g.h && (unsigned)iw < (unsigned)g.w)
          src = X + (((int64_t)nimg * g.h + ih) * g.w + iw) * g.c + c0 + 8 * c;
      }
      dma16(src, bdst + piece * 512);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
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

template <typename TO>
__global__ void __launch_bounds__(256) wgrad_reduce(const float* __restrict__ part, int splits, int64_t n,
                                                    TO* __restrict__ out) {
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += (int64_t)gridDim.x * 256 * 8) {
    float v[8], t8[8];
    Vec8<float>::load(v, part + i);
    for (int s = 1; s < splits; ++s) {
      Vec8<float>::load(t8, part + (int64_t)s * n + i);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += t8[k];
    }
    Vec8<TO>::store(out + i, v);
  }
}

struct WgPlan {
  int bm, bn, tiles, splits, chunk;
};

inline WgPlan wgrad_plan(const ConvTapArgs& a, int cus) {
  WgPlan p;
  const bool big = a.kout % 128 == 0 && a.c % 128 == 0;
  p.bm = big ? 128 : 64;
  p.bn = big ? 128 : 64;
  p.tiles = (a.kout / p.bm) * (a.ntaps * a.c / p.bn);
  const int64_t m = (int64_t)a.n * a.oh * a.ow;
  const int target = cus * 4;  // 2 resident workgroups per CU, two rounds
  int64_t s = (target + p.tiles - 1) / p.tiles;
  const int64_t max_s = (m + 16 * WG_BK - 1) / (16 * WG_BK);  // >= 16 K-steps per workgroup
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  int64_t chunk = (m + s - 1) / s;
  chunk = (chunk + WG_BK - 1) / WG_BK * WG_BK;
  p.chunk = (int)chunk;
  p.splits = (int)((m + chunk - 1) / chunk);
  return p;
}

}  // namespace conv

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

bool conv_tap_supported(const ConvTapArgs& a) {
  if (a.dtype != kBF16 && a.dtype != kF16) return false;
  if (a.c % 64 || a.kout % 64 || a.c <= 0 || a.kout <= 0) return false;
  if (a.ntaps < 1 || a.ntaps > kConvMaxTaps) return false;
  if (a.n <= 0 || a.oh <= 0 || a.ow <= 0) return false;
  if ((int64_t)a.n * a.oh * a.ow >= (1ll << 31) || (int64_t)a.n * a.ih * a.iw >= (1ll << 31)) return false;
  return aligned16(a.in) && aligned16(a.wt) && aligned16(a.out);
}

void conv_tap_fprop(const ConvTapArgs& a, int cus, hipStream_t s) {
  if (!conv_tap_supported(a)) throw std::runtime_error("conv_tap_fprop: unsupported shape / dtype / alignment");
  const conv::Geo g = conv::make_geo(a);
  const int64_t tiles_m = (g.m + conv::BM - 1) / conv::BM;
  int bn = 64;
  for (int cand : {256, 128}) {
    if (a.kout % cand == 0 && tiles_m * (a.kout / cand) >= cus) {
      bn = cand;
      break;
    }
  }
  const unsigned grid = (unsigned)(tiles_m * (a.kout / bn));
  dispatch_16(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    auto go = [&](auto kern, size_t lds) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(conv::THREADS), lds, s, (const uint16_t*)a.in, (const uint16_t*)a.wt,
                         (uint16_t*)a.out, g);
    };
    if (bn == 256) go(conv::fprop_kernel<T, 256>, conv::fprop_lds_bytes<256>());
    else if (bn == 128) go(conv::fprop_kernel<T, 128>, conv::fprop_lds_bytes<128>());
    else go(conv::fprop_kernel<T, 64>, conv::fprop_lds_bytes<64>());
  }, "conv_tap_fprop");
  check_launch("conv_tap_fprop");
}

bool conv_wgrad_supported(const ConvTapArgs& a) {
  if (!conv_tap_supported(a)) return false;
  return a.osh == 1 && a.osw == 1 && a.oph == 0 && a.opw == 0 && a.oht == a.oh && a.owt == a.ow;
}

int64_t conv_wgrad_workspace_floats(const ConvTapArgs& a, int cus) {
  const conv::WgPlan p = conv::wgrad_plan(a, cus);
  return (int64_t)p.splits * a.kout * a.ntaps * a.c;
}

void conv_wgrad(const ConvTapArgs& a, const void* dy, void* dw_out, int out_dtype, float* ws, int cus,
                hipStream_t s) {
  if (!conv_wgrad_supported(a) || !aligned16(dy) || !aligned16(dw_out) || !aligned16(ws))
    throw std::runtime_error("conv_wgrad: unsupported shape / dtype / alignment");
  const conv::Geo g = conv::make_geo(a);
  const conv::WgPlan p = conv::wgrad_plan(a, cus);
  dispatch_16(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    auto go = [&](auto kern, int bm, int bn) {
      const size_t lds = (size_t)2 * conv::WG_BK * (bm + bn) * 2;
      hipLaunchKernelGGL(kern, dim3(p.tiles, p.splits), dim3(conv::WG_THREADS), lds, s, (const uint16_t*)a.in,
                         (const uint16_t*)dy, ws, g, p.chunk);
    };
    if (p.bm == 128) go(conv::wgrad_kernel<T, 128, 128>, 128, 128);
    else go(conv::wgrad_kernel<T, 64, 64>, 64, 64);
  }, "conv_wgrad");
  const int64_t n = (int64_t)a.kout * a.ntaps * a.c;
  int64_t grid = (n / 8 + 255) / 256;
  if (grid > (int64_t)cus * 4) grid = (int64_t)cus * 4;
  dispatch_float(out_dtype, [&](auto tag) {
    using TO = typename decltype(tag)::type;
    hipLaunchKernelGGL((conv::wgrad_reduce<TO>), dim3((unsigned)grid), dim3(256), 0, s, (const float*)ws, p.splits, n,
                       (TO*)dw_out);
  }, "conv_wgrad out");
  check_launch("conv_wgrad");
}

}  // namespace apex_amd
