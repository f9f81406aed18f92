// ResNet stem for gfx950: 7x7/2 convolution (<= 4 input channels -> 64) + training batch norm +
// ReLU + 3x3/2 max pool, forward and backward, in five native kernels.
//
// Reference capability: the stem of the reference's ResNet-50 examples (torchvision conv1 /
// bn1 / relu / maxpool run as four library ops: examples/imagenet/main_amp.py), with the BN on
// apex's NHWC kernels (apex/contrib/csrc/groupbn).  Composition here (MI355X-first):
//
//  forward   pad_kernel    image [N, C<=4, H, W] (any strides) -> halo'd NHWC4 image
//                          XP [N][HP][WP][4] (zero halo of 3): the convolution then needs no
//                          bounds checks and every k-chunk is a 16-byte aligned load
//            fprop_kernel  implicit GEMM with K = 7 kernel rows x 32 (8 columns x 4 channels; the
//                          8th column carries zero weights): for an output pixel and kernel row r
//                          the 32 k-values are 64 CONTIGUOUS bytes of XP.  Swapped product
//                          Y^T = W . A^T: the weights are the MFMA A operand, resident in
//                          registers for the whole kernel (28 fragments); each lane's B fragment
//                          is one 16-byte load of its pixel's row chunk; 32 pixels x 64 channels
//                          per wave-tile = 28 MFMAs.  Channel rows are permuted so every lane holds
//                          16 consecutive channels of its pixel (two 16-byte stores); BN statistics
//                          (shift-centred sums) accumulate in registers and are folded once per
//                          workgroup (one partial row per workgroup).
//            pool_fwd      BN apply + ReLU + 3x3/2 max pool with the window separable: each lane
//                          walks a strip of pooled rows, keeping the horizontal max of the shared
//                          input row (6 loads per output instead of 9); 1-byte window indices.
//  backward  bwd_reduce    pool-backward gather + ReLU mask + BN backward sums in ONE pass over y
//                          (the full-resolution gradient is never written)
//            wgrad_kernel  dW = dX^T . im2col(XP) with dX = A g + B y + K recomputed from the
//                          pooled gradient, the window indices and y as the operand prologue; both
//                          operands staged pixel-major in LDS and fed with ds_read_b64_tr_b16;
//                          split over pixels, fp32 partials reduced in a fixed order.
// Against the library path (CK / MIOpen convolution on a channel-padded copy, BN statistics pass,
// apply+pool, pool backward writing the full-resolution gradient, BN reduction + dx passes, MIOpen
// weight gradient) this drops three full-resolution (N x 112 x 112 x 64) passes and moves both
// convolutions onto hand-written MFMA kernels.
#include "apex_amd/conv_api.h"
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/fastdiv.h"
#include "apex_amd/mfma.h"

#include <cstdlib>
#include <stdexcept>

namespace apex_amd {
namespace stem {
using namespace mfma;

constexpr int CO = 64;          // output channels
constexpr int KROW = 32;        // k per kernel row: 8 columns x 4 channels
constexpr int KT = 7 * KROW;    // 224
constexpr int NKS = KT / 16;    // 14 MFMA k-steps

// LDS-only barrier: this wave's LDS accesses complete, then a raw s_barrier.  __syncthreads()
// also drains every outstanding GLOBAL load (its workgroup fence waits vmcnt), which would
// serialize the register prefetch that is meant to stay in flight across the barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct Geo {
  int n, h, w, cin;
  int oh, ow, hp, wp, ph, pw;
  uint32_t m;  // n * oh * ow
};

inline Geo geo_of(int n, int h, int w, int cin) {
  Geo g;
  g.n = n;
  g.h = h;
  g.w = w;
  g.cin = cin;
  g.oh = (h - 1) / 2 + 1;
  g.ow = (w - 1) / 2 + 1;
  g.hp = 2 * (g.oh - 1) + 7;
  g.wp = 2 * (g.ow - 1) + 8;
  g.ph = (g.oh - 1) / 2 + 1;
  g.pw = (g.ow - 1) / 2 + 1;
  g.m = (uint32_t)((int64_t)n * g.oh * g.ow);
  return g;
}

// ---- image -> halo'd NHWC4 ---------------------------------------------------------------
// 4 padded pixels per thread per trip with every load issued before the first store: the
// per-pixel loads are 2-byte gathers, so bytes in flight per CU (not the store width) set the
// rate (one pixel per thread kept ~12 KB in flight per CU: 51 us for 185 MB).
constexpr int PAD_U = 4;
template <typename TI, typename T>
__global__ void __launch_bounds__(256) pad_kernel(const TI* __restrict__ x, int64_t sn, int64_t sc, int64_t sh,
                                                  int64_t sw, const Geo g, T* __restrict__ xp) {
  const uint32_t total = (uint32_t)g.n * g.hp * g.wp;
  const uint32_t gs = gridDim.x * 256u;
  for (uint32_t i0 = blockIdx.x * 256u + threadIdx.x; i0 < total; i0 += PAD_U * gs) {
    float v[PAD_U][4];
    bool in[PAD_U];
#pragma unroll
    for (int u = 0; u < PAD_U; ++u) {
      const uint32_t i = i0 + (uint32_t)u * gs;
      const uint32_t ic = i < total ? i : total - 1;
      const int j = (int)(ic % (uint32_t)g.wp);
      const uint32_t r = ic / (uint32_t)g.wp;
      const int ii = (int)(r % (uint32_t)g.hp), nn = (int)(r / (uint32_t)g.hp);
      const int ih = ii - 3, iw = j - 3;
      in[u] = ih >= 0 && ih < g.h && iw >= 0 && iw < g.w;
      const TI* src = x + nn * sn + min(max(ih, 0), g.h - 1) * sh + min(max(iw, 0), g.w - 1) * sw;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[u][c] = c < g.cin ? to_f(src[c * sc]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < PAD_U; ++u) {
      const uint32_t i = i0 + (uint32_t)u * gs;
      if (i >= total) break;
      uint16_t q[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) q[c] = in[u] ? from_f<T>(v[u][c]).x : (uint16_t)0;
      *reinterpret_cast<uint2*>(xp + (size_t)i * 4) =
          make_uint2(q[0] | ((uint32_t)q[1] << 16), q[2] | ((uint32_t)q[3] << 16));
    }
  }
}

// ---- weights [64, cin, 7, 7] (any strides) -> [64][224] with k = r * 32 + s * 4 + c -------
template <typename TW, typename T>
__global__ void __launch_bounds__(256) wpack_kernel(const TW* __restrict__ w, int cin, int64_t s0, int64_t s1,
                                                    int64_t s2, int64_t s3, T* __restrict__ wp) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= CO * KT) return;
  const int co = i / KT, k = i % KT, r = k / KROW, s = (k % KROW) / 4, c = k % 4;
  const float v = (s < 7 && c < cin) ? to_f(w[co * s0 + c * s1 + r * s2 + s * s3]) : 0.f;
  wp[i] = from_f<T>(v);
}

// ---- forward convolution + BN statistics ------------------------------------------------------
struct FpArgs {
  const uint16_t* xp;
  const uint16_t* wp;     // [64][224]
  const float* shift;     // [64] statistics shift (the running mean)
  uint16_t* y;            // [M][64]
  float* part;            // [2][G][64]
  Geo g;
  FastDiv div_ohw, div_ow;
  int tiles;              // ceil(M / 32)
};

// MFMA row m of channel tile t holds channel 32 t + perm(m): lane half h then owns channels
// 16 h .. 16 h + 15 of the tile in accumulator registers r = 0..15 (crow(r, h) -> 16 h + r)
__device__ __forceinline__ int chan_of_row(int m) { return 16 * ((m >> 2) & 1) + (m & 3) + 4 * (m >> 3); }

template <typename T>
__global__ void __launch_bounds__(256, 1) fprop_kernel(const FpArgs a) {
  __shared__ __attribute__((aligned(16))) float red[4 * 64 * 33];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, pl = lane & 31;
  // per-wave 4 KB output slab (32 pixels x 8 chunks of 16 B, chunk c of pixel x at c ^ (x & 7)) in
  // the statistics array, which is only used after the tile loop
  uint4* slab = reinterpret_cast<uint4*>(red) + wave * 256;
  const Geo& g = a.g;
  s16x8 wa[2][NKS];
  const int chm = chan_of_row(pl);
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      wa[t][ks] = *reinterpret_cast<const s16x8*>(a.wp + (32 * t + chm) * KT + 16 * ks + 8 * h);
  float sft[2][16], s1[2][16], s2[2][16];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sft[t][r] = a.shift ? a.shift[32 * t + 16 * h + r] : 0.f;
      s1[t][r] = s2[t][r] = 0.f;
    }
  const int nw = gridDim.x * 4, gw = blockIdx.x * 4 + wave;
  const int t0 = (int)((int64_t)gw * a.tiles / nw), t1 = (int)((int64_t)(gw + 1) * a.tiles / nw);
  const size_t rowstep = (size_t)g.wp * 4;

  auto src_of = [&](int tile, uint32_t& p) -> const uint16_t* {
    p = (uint32_t)tile * 32 + pl;
    const uint32_t pc = p < g.m ? p : g.m - 1;
    const uint32_t nn = fdiv(pc, a.div_ohw), rem = pc - nn * a.div_ohw.d;
    const uint32_t oh = fdiv(rem, a.div_ow), ow = rem - oh * a.div_ow.d;
    return a.xp + ((size_t)(nn * g.hp + 2 * oh) * g.wp + 2 * ow) * 4 + 8 * h;
  };
  auto load = [&](s16x8 (&b)[NKS], const uint16_t* src) {
#pragma unroll
    for (int r = 0; r < 7; ++r)
#pragma unroll
      for (int q = 0; q < 2; ++q) b[2 * r + q] = *reinterpret_cast<const s16x8*>(src + r * rowstep + 16 * q);
  };
  auto step = [&](const s16x8 (&b)[NKS], uint32_t p) {
    f32x16 acc[2] = {zero16(), zero16()};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      acc[0] = mma<T>(wa[0][ks], b[ks], acc[0]);
      acc[1] = mma<T>(wa[1][ks], b[ks], acc[1]);
    }
    const bool live = p < g.m;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      uint32_t wv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const T lo = from_f<T>(acc[t][2 * i]), hi = from_f<T>(acc[t][2 * i + 1]);
        wv[i] = (uint32_t)lo.x | ((uint32_t)hi.x << 16);
        if (live) {
          const float vl = to_f(lo) - sft[t][2 * i], vh = to_f(hi) - sft[t][2 * i + 1];
          s1[t][2 * i] += vl;
          s2[t][2 * i] = fmaf(vl, vl, s2[t][2 * i]);
          s1[t][2 * i + 1] += vh;
          s2[t][2 * i + 1] = fmaf(vh, vh, s2[t][2 * i + 1]);
        }
      }
      // a lane holds 2 x 16 B of its pixel's 128-B row: through the slab, so that each global
      // store below writes 8 whole rows (1 KB contiguous) instead of 16 B of 64 rows; the XOR
      // keeps the 8-lane ds_write_b128 groups (8 pixels, one chunk) on 8 distinct 16-B slots
      const int c0 = 4 * t + 2 * h, x7 = pl & 7;
      slab[pl * 8 + (c0 ^ x7)] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      slab[pl * 8 + ((c0 + 1) ^ x7)] = make_uint4(wv[4], wv[5], wv[6], wv[7]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own slab: no workgroup barrier
    const uint32_t pbase = p - (uint32_t)pl;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int L = lane + 64 * j, x = L >> 3, c = L & 7;
      const uint4 v = slab[x * 8 + (c ^ (x & 7))];
      if (pbase + (uint32_t)x < g.m) *reinterpret_cast<uint4*>(a.y + (size_t)(pbase + x) * CO + 8 * c) = v;
    }
    asm volatile("" ::: "memory");
  };

  // double-buffered: the next tile's 14 loads are in flight under this tile's 28 MFMAs
  s16x8 b0[NKS], b1[NKS];
  uint32_t p0 = 0, p1 = 0;
  // unconditional loads (past the end: a clamped tile, discarded) so the waits stay counted
  const int tl = t1 > t0 ? t1 - 1 : t0;
  load(b0, src_of(t0, p0));
  load(b1, src_of(min(t0 + 1, tl), p1));
  for (int tile = t0; tile < t1; tile += 2) {
    step(b0, p0);
    load(b0, src_of(min(tile + 2, tl), p0));
    if (tile + 1 < t1) step(b1, p1);
    load(b1, src_of(min(tile + 3, tl), p1));
  }

  // fold the statistics: per-lane sums -> LDS -> one row per workgroup (fixed order)
  const int ch = threadIdx.x & 63, which = threadIdx.x >> 6;  // which: 0 = s1, 1 = s2 (threads < 128)
  __syncthreads();  // every wave is done with its output slab
  for (int pass = 0; pass < 2; ++pass) {
    float* row = red + (wave * 64 + lane) * 33;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) row[16 * t + r] = pass == 0 ? s1[t][r] : s2[t][r];
    __syncthreads();
    if (which == pass) {
      const int t = ch >> 5, hh = (ch >> 4) & 1, r = ch & 15;
      float acc = 0.f;
      for (int w = 0; w < 4; ++w)
        for (int l = 0; l < 32; ++l) acc += red[(w * 64 + 32 * hh + l) * 33 + 16 * t + r];
      a.part[((size_t)pass * gridDim.x + blockIdx.x) * CO + ch] = acc;
    }
    __syncthreads();
  }
}

// ---- BN apply + ReLU + 3x3/2 max pool (pad 1) -------------------------------------------------
// pooled rows per lane (2 PR + 1 input rows x 3 columns, all loads issued first; adjacent pooled
// rows share an input row): APEX_AMD_STEM_PR = 2 (default) | 4 — 4 measured 144.7 vs 128 us in the
// step (profiles/r05/ab_stem_pr_r05x.txt): the taller strip holds 27 loads per lane in flight

struct PoolArgs {
  const uint16_t* y;   // [N][OH][OW][64]
  const float* coef;   // [2][64] scale | shift
  uint16_t* p;         // [N][PH][PW][64]
  uint8_t* idx;        // [N][PH][PW][64] window index kh * 3 + kw
  Geo g;
  int strips;
};

// horizontal best (value, column) of one loaded input row: the value the unfused apply pass
// would store, so argmax ties resolve identically; strict > keeps the first maximum
template <typename T>
__device__ __forceinline__ void hbest(const uint4 (&raw)[3], const bool (&ok)[3], const float (&sc)[8],
                                      const float (&sh)[8], float (&hv)[8], int (&hk)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    hv[e] = -INFINITY;
    hk[e] = 0;
  }
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    if (!ok[b]) continue;
    float v[8];
    Vec8<T>::load(v, reinterpret_cast<const T*>(&raw[b]));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float o = to_f(from_f<T>(fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f)));
      if (o > hv[e]) {
        hv[e] = o;
        hk[e] = b;
      }
    }
  }
}

template <typename T, int PR>
__global__ void __launch_bounds__(256) pool_fwd_kernel(const PoolArgs a) {
  const Geo& g = a.g;
  const uint32_t total = (uint32_t)g.n * a.strips * g.pw * 8;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const int c8 = (int)(i & 7);
    uint32_t r = i >> 3;
    const int pw = (int)(r % (uint32_t)g.pw);
    r /= (uint32_t)g.pw;
    const int strip = (int)(r % (uint32_t)a.strips), nn = (int)(r / (uint32_t)a.strips);
    const int ph0 = strip * PR;
    // input rows 2 ph0 - 1 .. 2 ph0 + 3, columns 2 pw - 1 .. 2 pw + 1
    uint4 raw[2 * PR + 1][3];
    bool ok[2 * PR + 1][3];
#pragma unroll
    for (int rr = 0; rr < 2 * PR + 1; ++rr) {
      const int yr = 2 * ph0 - 1 + rr;
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const int col = 2 * pw - 1 + b;
        ok[rr][b] = yr >= 0 && yr < g.oh && col >= 0 && col < g.ow;
        // clamped address, unconditional load (no branch around loads: counted vmcnt waits)
        const int yc = min(max(yr, 0), g.oh - 1), cc = min(max(col, 0), g.ow - 1);
        raw[rr][b] = *reinterpret_cast<const uint4*>(a.y + ((size_t)(nn * g.oh + yc) * g.ow + cc) * CO + c8 * 8);
      }
    }
    float sc[8], sh[8];
    Vec8<float>::load(sc, a.coef + c8 * 8);
    Vec8<float>::load(sh, a.coef + CO + c8 * 8);
    float cv[8];
    int ck[8];
    hbest<T>(raw[0], ok[0], sc, sh, cv, ck);
#pragma unroll
    for (int j = 0; j < PR; ++j) {
      const int ph = ph0 + j;
      if (ph >= g.ph) break;
      float v1[8], v2[8];
      int k1[8], k2[8];
      hbest<T>(raw[2 * j + 1], ok[2 * j + 1], sc, sh, v1, k1);
      hbest<T>(raw[2 * j + 2], ok[2 * j + 2], sc, sh, v2, k2);
      float best[8];
      uint32_t bi[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        // row-major first maximum: rows in order, strict > (same as the window scan)
        best[e] = cv[e];
        bi[e] = (uint32_t)ck[e];
        if (v1[e] > best[e]) {
          best[e] = v1[e];
          bi[e] = 3u + (uint32_t)k1[e];
        }
        if (v2[e] > best[e]) {
          best[e] = v2[e];
          bi[e] = 6u + (uint32_t)k2[e];
        }
        cv[e] = v2[e];
        ck[e] = k2[e];
      }
      const size_t o = ((size_t)(nn * g.ph + ph) * g.pw + pw) * CO + c8 * 8;
      Vec8<T>::store(reinterpret_cast<T*>(a.p + o), best);
      *reinterpret_cast<uint2*>(a.idx + o) = make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                                                        bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
    }
  }
}

// ---- backward: pool gather + ReLU mask (+ BN backward) ----------------------------------------
struct BwdArgs {
  const uint16_t* dp;     // [N][PH][PW][64] pooled gradient
  const uint8_t* idx;     // [N][PH][PW][64]
  const uint16_t* y;      // [M][64] convolution output (BN input)
  const float* coef;      // [2][64] forward scale | shift (ReLU mask recompute)
  const float* mean;      // [64] batch mean
  const float* cb;        // [3][64] dx = A g + B y + K
  const uint16_t* xp;     // halo'd image
  float* part;            // bwd_reduce: [2][G][64]
  float* ws;              // wgrad: [G][64][224]
  Geo g;
  FastDiv div_ohw, div_ow;
  FastDiv div_q, div_qw;  // wgrad: quads per image, quads per row
  uint32_t nq;            // wgrad: quads in the batch
  uint32_t chunk;         // wgrad: quads per workgroup (multiple of WQ)
  uint32_t xbytes;        // wgrad: halo'd image bytes (im2col buffer-load bound)
};

template <typename T>
__global__ void __launch_bounds__(256) bwd_reduce_kernel(const BwdArgs a) {
  __shared__ float red[2][32][CO + 1];
  const int tid = threadIdx.x, c8 = tid & 7;
  float sc[8], sh[8], mu[8], a1[8], a2[8];
  Vec8<float>::load(sc, a.coef + c8 * 8);
  Vec8<float>::load(sh, a.coef + CO + c8 * 8);
  Vec8<float>::load(mu, a.mean + c8 * 8);
#pragma unroll
  for (int e = 0; e < 8; ++e) a1[e] = a2[e] = 0.f;
  // one item = a 2 x 2 quad of conv-output pixels (rows 2 qh, 2 qh + 1; columns 2 qw, 2 qw + 1) x 8
  // channels: every pool window containing one of them is among (qh | qh + 1) x (qw | qw + 1), so
  // the quad loads those 4 windows once instead of 4 per pixel.  A pixel at padded row
  // hh = 2 qh + 1 + dy sits at window row hh - 2 ph = 1 + dy - 2 sh of slot row sh (in the window only
  // for sh = 0 or dy = 1); columns alike.  Per pixel the matching windows are summed in the same
  // (ph, pw) order a per-pixel gather would use.
  const uint32_t qh_n = (uint32_t)(a.g.oh + 1) >> 1, qw_n = (uint32_t)(a.g.ow + 1) >> 1;
  const uint32_t total = (uint32_t)a.g.n * qh_n * qw_n * 8u, stride = gridDim.x * 256u;
  for (uint32_t i = blockIdx.x * 256u + tid; i < total; i += stride) {
    const uint32_t q = i >> 3, nn = q / (qh_n * qw_n), rem = q - nn * (qh_n * qw_n);
    const int qh = (int)(rem / qw_n), qw = (int)(rem - (uint32_t)qh * qw_n);
    uint2 ix[4];
    uint4 gv[4], yv[4];
    bool wok[4], pok[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ph = qh + (s >> 1), pw = qw + (s & 1);
      wok[s] = ph < a.g.ph && pw < a.g.pw;
      const size_t o = ((size_t)(nn * a.g.ph + min(ph, a.g.ph - 1)) * a.g.pw + min(pw, a.g.pw - 1)) * CO + c8 * 8;
      ix[s] = *reinterpret_cast<const uint2*>(a.idx + o);
      gv[s] = *reinterpret_cast<const uint4*>(a.dp + o);
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int yh = 2 * qh + (d >> 1), yw = 2 * qw + (d & 1);
      pok[d] = yh < a.g.oh && yw < a.g.ow;
      const size_t pix = ((size_t)nn * a.g.oh + min(yh, a.g.oh - 1)) * a.g.ow + min(yw, a.g.ow - 1);
      yv[d] = *reinterpret_cast<const uint4*>(a.y + pix * CO + c8 * 8);
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (!pok[d]) continue;
      const int dy = d >> 1, dx = d & 1;
      float v[8], gs[8];
      Vec8<T>::load(v, reinterpret_cast<const T*>(&yv[d]));
#pragma unroll
      for (int e = 0; e < 8; ++e) gs[e] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int sr = s >> 1, sc2 = s & 1;
        if ((sr && !dy) || (sc2 && !dx)) continue;  // compile-time: the window misses the pixel
        const uint32_t kk = wok[s] ? (uint32_t)((1 + dy - 2 * sr) * 3 + (1 + dx - 2 * sc2)) : 255u;
        const uint32_t w[2] = {ix[s].x, ix[s].y};
        const uint32_t gw[4] = {gv[s].x, gv[s].y, gv[s].z, gv[s].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t k = (w[e >> 2] >> (8 * (e & 3))) & 0xffu;
          const float g = to_f(T{(uint16_t)((gw[e >> 1] >> (16 * (e & 1))) & 0xffffu)});
          gs[e] += k == kk ? g : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gm = fmaf(v[e], sc[e], sh[e]) > 0.f ? gs[e] : 0.f;
        a1[e] += gm;
        a2[e] = fmaf(gm, v[e] - mu[e], a2[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][tid >> 3][c8 * 8 + e] = a1[e];
    red[1][tid >> 3][c8 * 8 + e] = a2[e];
  }
  __syncthreads();
  if (tid < 2 * CO) {
    const int which = tid >> 6, ch = tid & 63;
    float acc = 0.f;
    for (int r = 0; r < 32; ++r) acc += red[which][r][ch];
    a.part[((size_t)which * gridDim.x + blockIdx.x) * CO + ch] = acc;
  }
}

// ---- backward: weight gradient with the BN-backward prologue ---------------------------------
constexpr int WPX = 128;            // pixels per step (the GEMM k dimension)
constexpr int WQ = WPX / 4;         // 2 x 2 pixel quads per step
constexpr int DSTR = CO + 32;       // dX image row stride (elements): rows 192 B apart in bank space
constexpr int IL_EL = 7 * WPX * KROW;  // im2col image [kernel row][pixel][32] (elements)
static_assert((WPX * DSTR + 2 * IL_EL) * 2 + 5 * CO * 4 <= 160 * 1024, "stem wgrad LDS");

__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, uint16_t* lds_dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff,
                                           (int)soff, 0, 0);
}

// A step is 32 quads of conv-output pixels (2 x 2, as in bwd_reduce_kernel) = 128 pixels: pixel row
// 4 q + d of the step is pixel d (row-major in the quad) of quad q, in the dX image and in the
// im2col image alike (the GEMM k order is free).
//  * dX: one (quad, 4 channels) item per lane loads the quad's 4 pool windows and 4 BN inputs once
//    (2 loads per pixel instead of 5 for a per-pixel gather) into registers, two steps ahead (two
//    register sets); the item is committed (pool gather, ReLU mask, dX = A g + B y + K) to the
//    single dX stage after the previous step's MFMAs.
//  * im2col: kernel row r of a pixel is 64 contiguous bytes of the halo'd NHWC4 image, so it goes
//    global -> LDS by buffer_load ... lds (lane-linear 16 B: wave w stages pixels 16 w .. 16 w + 15,
//    4 lanes each, all 7 rows; [r][pixel][32] rows are 64 B apart, conflict-free for the
//    transposed fragment reads) into a 2-stage ring, with no registers in flight.
// The im2col DMA of step s + 1 is issued after step s's commit barrier and lands under its MFMAs.
// Waves 0-6 run the MFMAs (k-tile u = wave = kernel row u, both 32-channel tiles).
// MODE (diagnostics, APEX_AMD_STEM_WG_MODE; 0 in production): bit 0 skips the pooled-gradient
// gather loads, bit 1 the MFMAs, bit 2 the im2col loads
template <typename T, int MODE>
__global__ void __launch_bounds__(512, 1) wgrad_kernel(const BwdArgs a) {
  // three distinct LDS objects: the compiler's alias analysis then sees that the MFMA reads of one
  // im2col stage do not depend on the DMA in flight into the other, and does not wait for it
  __shared__ __attribute__((aligned(16))) uint16_t dl[WPX * DSTR];
  __shared__ __attribute__((aligned(16))) uint16_t il0[IL_EL];
  __shared__ __attribute__((aligned(16))) uint16_t il1[IL_EL];
  __shared__ __attribute__((aligned(16))) float cf[5 * CO];  // forward scale | shift, backward A | B | K
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, pl = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Geo& g = a.g;
  const uint32_t q_begin = blockIdx.x * a.chunk;
  const uint32_t q_end = min(q_begin + a.chunk, a.nq);
  const int steps = q_begin < q_end ? (int)((q_end - q_begin + WQ - 1) / WQ) : 0;
  for (int i = tid; i < 5 * CO; i += 512) cf[i] = i < 2 * CO ? a.coef[i] : a.cb[i - 2 * CO];
  const int c4 = tid & 15, ql = tid >> 4;  // dX item: quad ql of the step, channels 4 c4 ..
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.xp, 0, __builtin_amdgcn_readfirstlane(a.xbytes), 0x00020000);
  const uint32_t rowbytes = __builtin_amdgcn_readfirstlane((uint32_t)g.wp * 8);

  auto quad_of = [&](uint32_t q, uint32_t& nn, int& qh, int& qw) {
    nn = fdiv(q, a.div_q);
    const uint32_t rem = q - nn * a.div_q.d;
    const uint32_t t = fdiv(rem, a.div_qw);
    qh = (int)t;
    qw = (int)(rem - t * a.div_qw.d);
  };

  // the pooled-gradient gather of a step, raw, in registers (two sets: issued two steps ahead)
  struct GRegs {
    uint32_t ix[4];
    uint2 gv[4], yv[4];
    uint32_t okm;  // bits 0-3: window s exists; bits 4-7: pixel d exists; bit 8: quad live
  };
  constexpr int NG = (MODE & 1) ? 4 : 12;  // gather loads per lane per step
  auto issue_dma = [&](int st, uint16_t* ilst) {
    if constexpr (!(MODE & 4)) {
      const uint32_t base = q_begin + (uint32_t)st * WQ;
      // im2col: pixel 16 wave + (lane >> 2) of the step, 16-B chunk lane & 3, kernel rows 0..6
      const int px = 16 * wave + (lane >> 2);
      uint32_t nn;
      int qh, qw;
      quad_of(min(base + (uint32_t)(px >> 2), q_end - 1), nn, qh, qw);
      const int oh = min(2 * qh + ((px >> 1) & 1), g.oh - 1), ow = min(2 * qw + (px & 1), g.ow - 1);
      const uint32_t voff = ((nn * (uint32_t)g.hp + 2u * (uint32_t)oh) * (uint32_t)g.wp + 2u * (uint32_t)ow) * 8u +
                            16u * (uint32_t)(lane & 3);
      uint16_t* dst = ilst + 16 * wave * KROW;
#pragma unroll
      for (int r = 0; r < 7; ++r) bdma16(xr, voff, (uint32_t)r * rowbytes, dst + r * WPX * KROW);
    }
  };
  auto issue_gather = [&](int st, GRegs& G) {
    const uint32_t base = q_begin + (uint32_t)st * WQ;
    const uint32_t q = min(base + (uint32_t)ql, q_end - 1);
    uint32_t nn;
    int qh, qw;
    quad_of(q, nn, qh, qw);
    uint32_t okm = base + (uint32_t)ql < q_end ? 256u : 0u;
    // every slot loads (clamped addresses): no branch around a load, counted vmcnt waits
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ph = qh + (s >> 1), pw = qw + (s & 1);
      okm |= (ph < g.ph && pw < g.pw) ? 1u << s : 0u;
      const size_t o = ((size_t)(nn * g.ph + min(ph, g.ph - 1)) * g.pw + min(pw, g.pw - 1)) * CO + c4 * 4;
      if constexpr (MODE & 1) {
        G.ix[s] = 0;
        G.gv[s] = make_uint2(0, 0);
      } else {
        G.ix[s] = *reinterpret_cast<const uint32_t*>(a.idx + o);
        G.gv[s] = *reinterpret_cast<const uint2*>(a.dp + o);
      }
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int yh = 2 * qh + (d >> 1), yw = 2 * qw + (d & 1);
      okm |= (yh < g.oh && yw < g.ow) ? 16u << d : 0u;
      const size_t pix = ((size_t)nn * g.oh + min(yh, g.oh - 1)) * g.ow + min(yw, g.ow - 1);
      G.yv[d] = *reinterpret_cast<const uint2*>(a.y + pix * CO + c4 * 4);
    }
    G.okm = okm;
  };
  auto commit = [&](const GRegs& G) {
    float sc[4], sh[4], A[4], B[4], K[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sc[e] = cf[c4 * 4 + e];
      sh[e] = cf[CO + c4 * 4 + e];
      A[e] = cf[2 * CO + c4 * 4 + e];
      B[e] = cf[3 * CO + c4 * 4 + e];
      K[e] = cf[4 * CO + c4 * 4 + e];
    }
    const uint32_t okm = G.okm;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int dy = d >> 1, dxc = d & 1;
      const float lv = (okm & 256u) && (okm & (16u << d)) ? 1.f : 0.f;
      const uint32_t yw2[2] = {G.yv[d].x, G.yv[d].y};
      float gs[4] = {0.f, 0.f, 0.f, 0.f}, dx[4];
      // the windows holding pixel d, summed in the (ph, pw) order a per-pixel gather uses
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int sr = s >> 1, sc2 = s & 1;
        if ((sr && !dy) || (sc2 && !dxc)) continue;  // compile-time: the window misses the pixel
        const uint32_t kk = (okm >> s) & 1u ? (uint32_t)((1 + dy - 2 * sr) * 3 + (1 + dxc - 2 * sc2)) : 255u;
        const uint32_t gw[2] = {G.gv[s].x, G.gv[s].y};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t k = (G.ix[s] >> (8 * e)) & 0xffu;
          const float gg = to_f(T{(uint16_t)((gw[e >> 1] >> (16 * (e & 1))) & 0xffffu)});
          gs[e] += k == kk ? gg : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = to_f(T{(uint16_t)((yw2[e >> 1] >> (16 * (e & 1))) & 0xffffu)});
        const float gm = fmaf(v, sc[e], sh[e]) > 0.f ? gs[e] : 0.f;
        // dX rounded to the storage type, as the unfused path's dx tensor; a dead pixel's operands
        // are a clamped live pixel's (finite), so the mask multiply zeroes it without the
        // per-element branch a select turns into
        dx[e] = fmaf(A[e], gm, fmaf(B[e], v, K[e])) * lv;
      }
      *reinterpret_cast<uint2*>(dl + (4 * ql + d) * DSTR + c4 * 4) =
          make_uint2((uint32_t)from_f<T>(dx[0]).x | ((uint32_t)from_f<T>(dx[1]).x << 16),
                     (uint32_t)from_f<T>(dx[2]).x | ((uint32_t)from_f<T>(dx[3]).x << 16));
    }
  };

  f32x16 acc[2] = {zero16(), zero16()};
  GRegs g0, g1;
  // Issue order: gather(0), DMA(0), gather(1); then in step s: DMA(s + 1), gather(s + 2), issued
  // unconditionally (past the last step: the last step's again, discarded), so on every path the
  // loads younger than DMA(s) when step s commits are gather(s + 1)'s NG: vmcnt(NG) retires DMA(s)
  // (and gather(s), which the commit used), and the compiler's own counted waits stay exact.
  auto step = [&](int st, uint16_t* cur, uint16_t* nxt, GRegs& G) {
    commit(G);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NG) : "memory");
    lds_barrier();
    issue_dma(min(st + 1, steps - 1), nxt);      // lands under this step's MFMAs
    issue_gather(min(st + 2, steps - 1), G);     // two steps ahead (G was just committed)
    if (wave < 7 && !(MODE & 2)) {
      const uint16_t* ib = cur + wave * WPX * KROW;
#pragma unroll
      for (int ks = 0; ks < WPX / 16; ++ks) {
        const int klo = 16 * ks + 8 * h;
        const s16x8 a0 = frag_tr<DSTR>(dl, 0, klo, klo + 4, lane);
        const s16x8 a1 = frag_tr<DSTR>(dl, 32, klo, klo + 4, lane);
        const s16x8 bf = frag_tr<KROW>(ib, 0, klo, klo + 4, lane);
        acc[0] = mma<T>(a0, bf, acc[0]);
        acc[1] = mma<T>(a1, bf, acc[1]);
      }
    }
    lds_barrier();
  };
  __syncthreads();  // cf
  if (steps > 0) {
    issue_gather(0, g0);
    issue_dma(0, il0);
    issue_gather(min(1, steps - 1), g1);
    // pairs (the im2col stage and the gather register set of every access are compile-time; no
    // branch around a step inside the loop, so the back edge always carries the same loads)
    int st = 0;
    for (; st + 1 < steps; st += 2) {
      step(st, il0, il1, g0);
      step(st + 1, il1, il0, g1);
    }
    if (st < steps) step(st, il0, il1, g0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the discarded tail loads
  }
  if (wave < 7) {
    float* ws = a.ws + (size_t)blockIdx.x * CO * KT;
    const int col = 32 * wave + pl;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) ws[(size_t)(32 * t + crow(r, h)) * KT + col] = acc[t][r];
  }
}

// dW[co][c][r][s] (strided, weight dtype) = sum over the G partials of k = r * 32 + s * 4 + c.
// A block owns 64 consecutive elements of the flat [64][224] partial; its 4 thread groups take
// every 4th partial (coalesced 256-byte rows, 64 loads per thread in flight instead of one thread
// walking all G partials), then one LDS fold in group order (fixed order: deterministic).
template <typename TW>
__global__ void __launch_bounds__(256) wgrad_reduce(const float* __restrict__ ws, int G, int cin, int64_t s0,
                                                    int64_t s1, int64_t s2, int64_t s3, TW* __restrict__ dw) {
  __shared__ float red[4][64];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63), grp = threadIdx.x >> 6;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int j = grp;
  for (; j + 12 < G; j += 16)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] += ws[(size_t)(j + 4 * u) * CO * KT + e];
  for (; j < G; j += 4) acc[0] += ws[(size_t)j * CO * KT + e];
  red[grp][threadIdx.x & 63] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (grp != 0) return;
  const float v = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
  const int co = e / KT, k = e % KT, r = k / KROW, sx = (k % KROW) / 4, c = k % 4;
  if (sx < 7 && c < cin) dw[co * s0 + c * s1 + r * s2 + sx * s3] = from_f<TW>(v);
}

inline void check_geo(const Geo& g) {
  if (g.n <= 0 || g.h <= 0 || g.w <= 0 || g.cin < 1 || g.cin > 4)
    throw std::runtime_error("stem: needs a non-empty image with 1-4 channels");
  if ((int64_t)g.n * g.hp * g.wp * 4 >= (1ll << 31) || (int64_t)g.m * CO >= (1ll << 31))
    throw std::runtime_error("stem: tensors past 2^31 elements (32-bit indexing)");
}

}  // namespace stem

void stem_geometry(int n, int h, int w, int* oh, int* ow, int* hp, int* wp, int* ph, int* pw) {
  const stem::Geo g = stem::geo_of(n, h, w, 1);
  *oh = g.oh;
  *ow = g.ow;
  *hp = g.hp;
  *wp = g.wp;
  *ph = g.ph;
  *pw = g.pw;
}

int stem_fprop_rows(int cus) { return cus; }
int stem_reduce_rows(int cus) { return cus * 4; }
int stem_wgrad_parts(int cus) { return cus; }

void stem_pad(const void* x, int x_t, int n, int cin, int h, int w, const int64_t* strides, void* xp, int t,
              int cus, hipStream_t s) {
  const stem::Geo g = stem::geo_of(n, h, w, cin);
  stem::check_geo(g);
  const int64_t total = (int64_t)n * g.hp * g.wp;
  int64_t grid = (total + 255) / 256;
  if (grid > (int64_t)cus * 16) grid = (int64_t)cus * 16;
  dispatch_float(x_t, [&](auto ti) {
    using TI = typename decltype(ti)::type;
    dispatch_16(t, [&](auto to) {
      using T = typename decltype(to)::type;
      hipLaunchKernelGGL((stem::pad_kernel<TI, T>), dim3((unsigned)grid), dim3(256), 0, s, (const TI*)x, strides[0],
                         strides[1], strides[2], strides[3], g, (T*)xp);
    }, "stem pad (out)");
  }, "stem pad (in)");
  check_launch("stem_pad");
}

void stem_wpack(const void* w, int w_t, int cin, const int64_t* strides, void* wp, int t, hipStream_t s) {
  if (cin < 1 || cin > 4) throw std::runtime_error("stem: 1-4 input channels");
  dispatch_float(w_t, [&](auto tw) {
    using TW = typename decltype(tw)::type;
    dispatch_16(t, [&](auto to) {
      using T = typename decltype(to)::type;
      hipLaunchKernelGGL((stem::wpack_kernel<TW, T>), dim3((stem::CO * stem::KT + 255) / 256), dim3(256), 0, s,
                         (const TW*)w, cin, strides[0], strides[1], strides[2], strides[3], (T*)wp);
    }, "stem wpack (out)");
  }, "stem wpack (in)");
  check_launch("stem_wpack");
}

void stem_fprop(const void* xp, const void* wp, const float* shift, void* y, float* part, int n, int h, int w,
                int t, int cus, hipStream_t s) {
  stem::FpArgs a;
  a.g = stem::geo_of(n, h, w, 4);
  stem::check_geo(a.g);
  a.xp = (const uint16_t*)xp;
  a.wp = (const uint16_t*)wp;
  a.shift = shift;
  a.y = (uint16_t*)y;
  a.part = part;
  a.div_ohw = make_fastdiv((uint32_t)(a.g.oh * a.g.ow));
  a.div_ow = make_fastdiv((uint32_t)a.g.ow);
  a.tiles = (int)((a.g.m + 31) / 32);
  dispatch_16(t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    hipLaunchKernelGGL((stem::fprop_kernel<T>), dim3(stem_fprop_rows(cus)), dim3(256), 0, s, a);
  }, "stem fprop");
  check_launch("stem_fprop");
}

void stem_pool_fwd(const void* y, const float* coef, void* p, uint8_t* idx, int n, int h, int w, int t, int cus,
                   hipStream_t s) {
  stem::PoolArgs a;
  a.g = stem::geo_of(n, h, w, 4);
  stem::check_geo(a.g);
  a.y = (const uint16_t*)y;
  a.coef = coef;
  a.p = (uint16_t*)p;
  a.idx = idx;
  static const int pr = [] {
    const char* e = std::getenv("APEX_AMD_STEM_PR");
    return e && std::atoi(e) == 4 ? 4 : 2;
  }();
  a.strips = (a.g.ph + pr - 1) / pr;
  const int64_t total = (int64_t)n * a.strips * a.g.pw * 8;
  int64_t grid = (total + 255) / 256;
  if (grid > (int64_t)cus * 16) grid = (int64_t)cus * 16;
  dispatch_16(t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (pr == 2) hipLaunchKernelGGL((stem::pool_fwd_kernel<T, 2>), dim3((unsigned)grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((stem::pool_fwd_kernel<T, 4>), dim3((unsigned)grid), dim3(256), 0, s, a);
  }, "stem pool fwd");
  check_launch("stem_pool_fwd");
}

static stem::BwdArgs bwd_args(const void* dp, const uint8_t* idx, const void* y, const float* coef, int n, int h,
                              int w) {
  stem::BwdArgs a{};
  a.g = stem::geo_of(n, h, w, 4);
  stem::check_geo(a.g);
  a.dp = (const uint16_t*)dp;
  a.idx = idx;
  a.y = (const uint16_t*)y;
  a.coef = coef;
  a.div_ohw = make_fastdiv((uint32_t)(a.g.oh * a.g.ow));
  a.div_ow = make_fastdiv((uint32_t)a.g.ow);
  return a;
}

void stem_bwd_reduce(const void* dp, const uint8_t* idx, const void* y, const float* coef, const float* mean,
                     float* part, int n, int h, int w, int t, int cus, hipStream_t s) {
  stem::BwdArgs a = bwd_args(dp, idx, y, coef, n, h, w);
  a.mean = mean;
  a.part = part;
  dispatch_16(t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    hipLaunchKernelGGL((stem::bwd_reduce_kernel<T>), dim3(stem_reduce_rows(cus)), dim3(256), 0, s, a);
  }, "stem bwd reduce");
  check_launch("stem_bwd_reduce");
}

void stem_wgrad(const void* dp, const uint8_t* idx, const void* y, const float* coef, const float* cb,
                const void* xp, float* ws, void* dw, int dw_t, int cin, const int64_t* dw_strides, int n, int h, int w,
                int t, int cus, hipStream_t s) {
  stem::BwdArgs a = bwd_args(dp, idx, y, coef, n, h, w);
  a.cb = cb;
  a.xp = (const uint16_t*)xp;
  a.xbytes = (uint32_t)((int64_t)n * a.g.hp * a.g.wp * 8);
  a.ws = ws;
  const int G = stem_wgrad_parts(cus);
  const uint32_t qh_n = (uint32_t)(a.g.oh + 1) / 2, qw_n = (uint32_t)(a.g.ow + 1) / 2;
  a.nq = (uint32_t)a.g.n * qh_n * qw_n;
  a.div_q = make_fastdiv(qh_n * qw_n);
  a.div_qw = make_fastdiv(qw_n);
  a.chunk = (uint32_t)(((int64_t)a.nq + G - 1) / G);
  a.chunk = (a.chunk + stem::WQ - 1) / stem::WQ * stem::WQ;

  if (cin < 1 || cin > 4) throw std::runtime_error("stem wgrad: 1-4 input channels");
  dispatch_16(t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    static const int mode = [] {
      const char* e = std::getenv("APEX_AMD_STEM_WG_MODE");
      return e ? std::atoi(e) : 0;
    }();
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(G), dim3(512), 0, s, a); };
    switch (mode) {
      case 1: go(stem::wgrad_kernel<T, 1>); break;
      case 2: go(stem::wgrad_kernel<T, 2>); break;
      case 4: go(stem::wgrad_kernel<T, 4>); break;
      case 7: go(stem::wgrad_kernel<T, 7>); break;
      default: go(stem::wgrad_kernel<T, 0>); break;
    }
  }, "stem wgrad");
  dispatch_float(dw_t, [&](auto tag) {
    using TW = typename decltype(tag)::type;
    hipLaunchKernelGGL((stem::wgrad_reduce<TW>), dim3(stem::CO * stem::KT / 64), dim3(256), 0, s, ws, G, cin,
                       dw_strides[0], dw_strides[1], dw_strides[2], dw_strides[3], (TW*)dw);
  }, "stem wgrad reduce");
  check_launch("stem_wgrad");
}

}  // namespace apex_amd
