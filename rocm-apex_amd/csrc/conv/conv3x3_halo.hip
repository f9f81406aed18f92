// Halo-tile 3x3 (pad 1, stride 1) convolution for C, K multiples of 64 / 128, NHWC bf16 / fp16,
// for gfx950 — the forward of ResNet stages 2-4 and, with the flipped weight, their data gradient.
//
// Why: the tap GEMM of conv_igemm.hip (fprop2) gathers its A tile (256 pixels x 64 channels) from
// global memory ONCE PER TAP; at 128 output channels per workgroup that is ~78 B of L2 traffic per
// CU cycle at full MFMA rate — more than the L2 delivers, so it runs at 23-27 % of the MFMA peak
// (profiles/pmc_resnet_kernels_r04al.md, 86-94 us for a 59-GFLOP 28x28x128 conv).  Here:
//   * a workgroup (8 waves: 2 channel groups x 4 pixel groups) owns 128 output channels and walks
//     a range of pixel TILES: R consecutive output rows of the batch (flattened n*h row space,
//     R*w <= 256; a tile may cross an image boundary: its halo is taken in the row space where
//     every image carries its zero padding rows, so the boundary needs no special case);
//   * per 64-channel block the tile's input HALO (<= 448 slots of 128 B, zero outside the images)
//     is staged into LDS once by buffer_load ... lds and read by all 9 taps at shifted slots; the
//     next block's halo streams into the second halo buffer under the current block's 9 taps;
//   * per tap the weight slice [128 channels][64] streams through a 3-deep LDS ring (counted vmcnt,
//     raw barrier: the loads stay in flight across barriers);
//   * MFMA with the WEIGHT as the A operand: the accumulators hold [channel][pixel], so each lane
//     owns one pixel and 4 consecutive channels per register group — the epilogue stores 8-byte
//     channel runs straight from registers (buffer stores: pixels past the tile are dropped by
//     the range check, so every wave issues the same number of stores and the counted vmcnt of
//     the next tile stays exact);
//   * optional prologue: relu(x * scale[c] + shift[c]) applied to the staged halo in LDS (each wave
//     converts its own DMA pieces once they land, padding slots stay exact zeros) — the producing
//     batch norm + ReLU of a ResNet bottleneck, so that activation is never written to memory;
//   * optional BN-statistics epilogue of the output (sum / sum of squares about a shift), one
//     partial row per workgroup.
// Reference capability: the fused NHWC convolutions of apex/contrib/bottleneck
// (apex/contrib/csrc/bottleneck/bottleneck.cpp:1104 bottleneck_forward: scale-bias-ReLU-conv).
#include "apex_amd/conv_api.h"
#include "apex_amd/conv_halo.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/fastdiv.h"
#include "apex_amd/mfma.h"

#include <algorithm>
#include <stdexcept>

namespace apex_amd {
namespace hfp {
using namespace mfma;

constexpr int NT = 512;                 // 8 waves
constexpr int NPP = 256;                // output pixels per tile
constexpr int KB = 128;                 // output channels per workgroup
constexpr int BK = 64;                  // input channels per block (one K-step = one tap of it)
constexpr int HSL = 448;                // halo slots per block image (128 B each)
constexpr int HIW = HSL / 8 / 8;        // halo DMA instructions per wave (7)
constexpr int WIW = KB * BK * 2 / 1024 / 8;  // weight DMA instructions per wave per K-step (2)
constexpr int SB = 3;                   // weight ring stages
constexpr int HALO_EL = HSL * BK;
constexpr int WT_EL = KB * BK;
constexpr size_t LDS = (size_t)(2 * HALO_EL + SB * WT_EL) * 2;
static_assert(LDS <= 163840, "LDS budget");
static_assert(HSL % 64 == 0, "halo DMA instructions split evenly over 8 waves");

struct Args {
  const uint16_t* x;     // [n][h][w][c]
  const uint16_t* w;     // [k][9][c]
  uint16_t* y;           // [n][h][w][k]
  const float* pcoef;    // nullable [2][c]: prologue scale | shift
  float* stats;          // nullable [2][P][k]
  const float* shift;    // nullable [k]
  int n, h, wd, c, k;
  int R, HC;             // tile rows, halo slot columns
  int rows_total, ntiles, P;
  FastDiv div_h, div_hp, div_w, div_hc;
  int xbytes, wbytes, ybytes;
};

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint16_t* lds_dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff, 0, 0,
                                           0);
}

// padded-row index of flattened output row r: image img = r / h sits in rows img*(h+2) .. +h+1,
// its first and last being the zero padding
__device__ __forceinline__ int padded_row(const Args& p, int r) {
  const int img = (int)fdiv((uint32_t)r, p.div_h);
  return img * (p.h + 2) + (r - img * p.h) + 1;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename T, bool PRO, bool STATS>
__global__ void __launch_bounds__(NT, 1) fprop_kernel(const Args p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* halo = lds;                     // 2 x HALO_EL
  uint16_t* wring = lds + 2 * HALO_EL;      // SB x WT_EL
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, lh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wave >> 2, pg = wave & 3;  // channel group (64), pixel group (64)
  const int nkb = p.k / KB;
  const int g = xcd_remap(blockIdx.x, p.P * nkb);
  // consecutive workgroups (one XCD) take the same pixel range for the k-blocks: halo re-reads
  // hit that XCD's L2
  const int kb = g % nkb, pidx = g / nkb;
  const int t_begin = (int)((int64_t)pidx * p.ntiles / p.P), t_end = (int)((int64_t)(pidx + 1) * p.ntiles / p.P);
  const int ntile = t_end - t_begin;
  const int ncb = p.c / BK;
  const int nsteps = ntile * 9 * ncb, ncbg = ntile * ncb;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, __builtin_amdgcn_readfirstlane(p.xbytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, __builtin_amdgcn_readfirstlane(p.wbytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.y, 0, __builtin_amdgcn_readfirstlane(p.ybytes), 0x00020000);
  const int hpad = p.h + 2;

  // ---- weight DMA: rows kb*128 + r, this lane's 16-B chunk (source-swizzled) ----
  uint32_t woff[WIW];
#pragma unroll
  for (int i = 0; i < WIW; ++i) {
    const int r = 8 * (i * 8 + wave) + (lane >> 3);
    const int sc = (lane & 7) ^ ((r >> 1) & 7);
    woff[i] = (uint32_t)(((kb * KB + r) * 9 * p.c + 8 * sc) * 2);
  }
  auto issue_w = [&](int q) {
    const int cbg = q / 9, t = q - cbg * 9;
    const int cb = cbg % ncb;
    const uint32_t k0 = (uint32_t)((t * p.c + cb * BK) * 2);
    uint16_t* dst = wring + (q % SB) * WT_EL;
#pragma unroll
    for (int i = 0; i < WIW; ++i) bdma16(wr, woff[i] + k0, dst + (i * 8 + wave) * 512);
  };

  // ---- halo DMA: this lane's slot of each of its HIW pieces (tile-invariant part) ----
  // packed per piece: halo row (bits 0-9), column (10-19), source chunk (20-22)
  uint32_t hpk[HIW];
#pragma unroll
  for (int i = 0; i < HIW; ++i) {
    const int s = 8 * (i * 8 + wave) + (lane >> 3);
    const int hr = (int)fdiv((uint32_t)s, p.div_hc);
    hpk[i] = (uint32_t)hr | ((uint32_t)(s - hr * p.HC) << 10) | ((uint32_t)((lane & 7) ^ ((s >> 1) & 7)) << 20);
  }
  auto hrow = [&](int i) { return (int)(hpk[i] & 1023u); };
  auto hcol = [&](int i) { return (int)((hpk[i] >> 10) & 1023u); };
  auto hsc = [&](int i) { return (int)(hpk[i] >> 20); };
  uint32_t pend_mask = 0;  // validity of this lane's pieces of the last issued halo (prologue)
  auto issue_halo = [&](int cbg) {
    const int tile = t_begin + cbg / ncb, cb = cbg % ncb;
    const int plo = padded_row(p, tile * p.R) - 1;
    uint16_t* dst = halo + (cbg & 1) * HALO_EL;
    uint32_t mk = 0;
#pragma unroll
    for (int i = 0; i < HIW; ++i) {
      const int pr = plo + hrow(i);
      const int img = (int)fdiv((uint32_t)pr, p.div_hp);
      const int yy = pr - img * hpad - 1, ix = hcol(i) - 1;
      const bool ok = img < p.n && (unsigned)yy < (unsigned)p.h && (unsigned)ix < (unsigned)p.wd;
      const uint32_t off = (uint32_t)((((img * p.h + yy) * p.wd + ix) * p.c + cb * BK + 8 * hsc(i)) * 2);
      bdma16(xr, ok ? off : 0x80000000u, dst + (i * 8 + wave) * 512);
      mk |= ok ? (1u << i) : 0u;
    }
    pend_mask = mk;
  };
  // prologue: this wave's landed pieces of halo buffer (cbg & 1) -> relu(x * s + b) in place
  auto transform = [&](int cbg) {
    const int cb = cbg % ncb;
    uint16_t* buf = halo + (cbg & 1) * HALO_EL;
    // a rolled loop (the chunk is recomputed from the piece index): unrolled, the compiler keeps
    // every piece's coefficient and data registers live at once
#pragma unroll 1
    for (int i = 0; i < HIW; ++i) {
      if (!((pend_mask >> i) & 1u)) continue;
      const int sl = 8 * (i * 8 + wave) + (lane >> 3);
      const int c0 = cb * BK + 8 * ((lane & 7) ^ ((sl >> 1) & 7));
      uint16_t* q = buf + (i * 8 + wave) * 512 + lane * 8;
      float sc[8], sh[8], v[8];
      Vec8<float>::load(sc, p.pcoef + c0);
      Vec8<float>::load(sh, p.pcoef + p.c + c0);
      Vec8<T>::load(v, reinterpret_cast<const T*>(q));
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f);
      Vec8<T>::store(reinterpret_cast<T*>(q), v);
    }
  };

  // ---- fragment addresses ----
  // A (weights, rows = output channels cg*64 + 32 i + lr): chunk (2 kk + lh) ^ ((row >> 1) & 7)
  int abase[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = cg * 64 + 32 * i + lr;
    abase[i] = row * BK + ((lh ^ ((row >> 1) & 7)) << 3);
  }
  // B (halo, one pixel per lane per subtile j): slot of the pixel's centre tap, per tile
  int pslot[2];
  auto tile_slots = [&](int tile) {
    const int plo = padded_row(p, tile * p.R) - 1;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int jp = pg * 64 + 32 * j + lr;
      const int rr = (int)fdiv((uint32_t)jp, p.div_w), x = jp - rr * p.wd;
      const int r = min(tile * p.R + min(rr, p.R - 1), p.rows_total - 1);
      pslot[j] = (padded_row(p, r) - plo) * p.HC + x + 1;
    }
  };

  // ---- statistics state: after each tile's reduce-scatter over the 32 pixels of a half-wave,
  // lane lr owns ONE channel (subtile lr & 1, register lr >> 1 of the wave's accumulators), so
  // the running sums are 2 registers per lane (+ its shift) instead of 64 + 32 ----
  const int stat_ch = kb * KB + cg * 64 + 32 * (lr & 1) + crow(lr >> 1, lh);
  const float stat_shift = (STATS && p.shift) ? p.shift[stat_ch] : 0.f;
  float S1 = 0.f, S2 = 0.f;  // sums of (y - shift) and (y - shift)^2 of stat_ch over this WG's pixels

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  // ---- prologue: halo of block 0, weights of steps 0 and 1 ----
  if (nsteps > 0) {
    issue_halo(0);
    issue_w(0);
    if (nsteps > 1) issue_w(1);
    if constexpr (PRO) {
      if (nsteps > 1) wait_vm<2 * WIW>();
      else wait_vm<WIW>();
      transform(0);
    }
    tile_slots(t_begin);
  }

  // H(s): halo DMA instructions this wave issued at step s (after that step's weight DMA);
  // E(s): output stores it issued at step s (a tile's last step: 16 buffer stores, every lane,
  // always issued — pixels past the tile are dropped by the range check, not by a branch)
  constexpr int ES = 16;
  auto hcount = [&](int s) { return (s >= 0 && s % 9 == 0 && s / 9 + 1 < ncbg) ? HIW : 0; };
  auto ecount = [&](int s) { return (s >= 0 && s % 9 == 8 && (s / 9) % ncb == ncb - 1) ? ES : 0; };
#pragma unroll 1
  for (int q = 0; q < nsteps; ++q) {
    const int cbg = q / 9, t = q - cbg * 9;
    // weights of step q landed: the vector-memory instructions issued after them are step q+1's
    // weights and the halos / epilogue stores of steps q-2 and q-1
    const int younger = (q + 1 < nsteps ? WIW : 0) + hcount(q - 2) + hcount(q - 1) + ecount(q - 2) + ecount(q - 1);
    switch (younger) {
      case WIW: wait_vm<WIW>(); break;
      case HIW: wait_vm<HIW>(); break;
      case WIW + HIW: wait_vm<WIW + HIW>(); break;
      case ES: wait_vm<ES>(); break;
      case WIW + ES: wait_vm<WIW + ES>(); break;
      case HIW + ES: wait_vm<HIW + ES>(); break;
      case WIW + HIW + ES: wait_vm<WIW + HIW + ES>(); break;
      default: wait_vm<0>(); break;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (q + 2 < nsteps) issue_w(q + 2);
    if (t == 0 && cbg + 1 < ncbg) issue_halo(cbg + 1);

    const uint16_t* hb = halo + (cbg & 1) * HALO_EL;
    const uint16_t* wb = wring + (q % SB) * WT_EL;
    const int toff = (t / 3 - 1) * p.HC + (t % 3 - 1);
    int bb[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int s = pslot[j] + toff;
      bb[j] = s * BK + ((lh ^ ((s >> 1) & 7)) << 3);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      s16x8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = *reinterpret_cast<const s16x8*>(wb + (abase[i] ^ (kk << 4)));
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = *reinterpret_cast<const s16x8*>(hb + (bb[j] ^ (kk << 4)));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma<T>(af[i], bf[j], acc[i][j]);
    }

    if constexpr (PRO) {
      // the next block's halo (issued at t = 0) gets its prologue here, published by the next
      // barrier; the weight DMAs issued at t = 1..4 may still be in flight
      if (t == 4 && cbg + 1 < ncbg) {
        __builtin_amdgcn_sched_barrier(0);  // keep the prologue's loads out of the MFMA block
        const int nw = (q - 1 + 2 < nsteps) + (q - 2 + 2 < nsteps) + (q - 3 + 2 < nsteps) + (q + 2 < nsteps);
        if (nw == 4) wait_vm<4 * WIW>();
        else if (nw == 3) wait_vm<3 * WIW>();
        else if (nw == 2) wait_vm<2 * WIW>();
        else if (nw == 1) wait_vm<WIW>();
        else wait_vm<0>();
        transform(cbg + 1);
      }
    }

    if (t == 8 && cbg % ncb == ncb - 1) {
      // ---- tile epilogue from registers: pixel lr of subtile j, channels in runs of 4 ----
      const int tile = t_begin + cbg / ncb;
      int nval = 0;
      bool okj[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int jp = pg * 64 + 32 * j + lr;
        const int rr = (int)fdiv((uint32_t)jp, p.div_w), x = jp - rr * p.wd;
        const int r = tile * p.R + rr;
        const bool ok = rr < p.R && r < p.rows_total;
        okj[j] = ok;
        if constexpr (STATS) nval += __popcll(__ballot(ok) & (lh ? 0xffffffff00000000ull : 0xffffffffull));
        const int64_t pix = (int64_t)r * p.wd + x;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            const int ch = kb * KB + cg * 64 + 32 * i + 8 * gq + 4 * lh;
            const T a0 = from_f<T>(acc[i][j][4 * gq + 0]), a1 = from_f<T>(acc[i][j][4 * gq + 1]);
            const T a2 = from_f<T>(acc[i][j][4 * gq + 2]), a3 = from_f<T>(acc[i][j][4 * gq + 3]);
            const uint32_t lo = (uint32_t)a0.x | ((uint32_t)a1.x << 16);
            const uint32_t hi = (uint32_t)a2.x | ((uint32_t)a3.x << 16);
            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
            const uint32_t voff = ok ? (uint32_t)((pix * p.k + ch) * 2) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{lo, hi}, yr, voff, 0, 0);
          }
      }
      if constexpr (STATS) {
        // per subtile i: this lane's sums over its 2 pixels (the stored, rounded values), then a
        // reduce-scatter over the 32 lanes of each half — at the stage of mask m a lane keeps the
        // half of its values selected by its lane bit and adds the partner's copy of that half —
        // leaving register r = lr >> 1 in the lane pair (lr, lr ^ 1); lane lr keeps subtile lr & 1
        const float nf = (float)nval;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          float x1[16], x2[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float a = 0.f, b2 = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const float v = okj[j] ? to_f(from_f<T>(acc[i][j][r])) : 0.f;
              a += v;
              b2 = fmaf(v, v, b2);
            }
            x1[r] = a;
            x2[r] = b2;
          }
#pragma unroll
          for (int m = 16, K = 8; m >= 2; m >>= 1, K >>= 1) {
            const bool b = (lr & m) != 0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
              const float s1 = b ? x1[k] : x1[k + K], s2 = b ? x2[k] : x2[k + K];
              const float r1 = __shfl_xor(s1, m, 64), r2 = __shfl_xor(s2, m, 64);
              x1[k] = (b ? x1[k + K] : x1[k]) + r1;
              x2[k] = (b ? x2[k + K] : x2[k]) + r2;
            }
          }
          const float t1 = x1[0] + __shfl_xor(x1[0], 1, 64), t2 = x2[0] + __shfl_xor(x2[0], 1, 64);
          // about the shift: Σ(y-s) = Σy - n s, Σ(y-s)^2 = Σy^2 - 2 s Σy + n s^2
          if ((lr & 1) == i) {
            S1 += t1 - nf * stat_shift;
            S2 += t2 - 2.f * stat_shift * t1 + nf * stat_shift * stat_shift;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = zero16();
      if (cbg + 1 < ncbg) tile_slots(tile + 1);
    }
  }

  if constexpr (!STATS) return;
  // ---- statistics: every lane holds one channel's sums; fold the 4 pixel-group waves ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);  // [2][4 pixel groups][KB]
  const int cl = stat_ch - kb * KB;
  red[(0 * 4 + pg) * KB + cl] = S1;
  red[(1 * 4 + pg) * KB + cl] = S2;
  __syncthreads();
  if (tid < 2 * KB) {
    const int which = tid / KB, c = tid % KB;
    float v = 0.f;
#pragma unroll
    for (int w4 = 0; w4 < 4; ++w4) v += red[(which * 4 + w4) * KB + c];
    p.stats[((int64_t)which * p.P + pidx) * p.k + kb * KB + c] = v;
  }
}

struct Plan {
  bool ok;
  int R, HC, ntiles, P;
};

inline Plan make_plan(const ConvTapArgs& a, int cus) {
  Plan pl{false, 0, 0, 0, 0};
  const int h = a.oh, w = a.ow;
  if (w < 1 || h < 1 || w > NPP) return pl;
  const int HC = w + 2;
  // the most rows per tile whose pixels fit and whose halo (R + 2 rows, plus 2 per image boundary
  // crossed) fits the slot budget
  for (int r = NPP / w; r >= 1; --r) {
    const int crossings = (r + h - 1) / h;  // image boundaries a tile of r rows may cross, at most
    if ((r + 2 + 2 * crossings) * HC <= HSL) {
      pl.R = r;
      break;
    }
  }
  if (pl.R == 0) return pl;
  pl.HC = HC;
  const int64_t rows = (int64_t)a.n * h;
  pl.ntiles = (int)((rows + pl.R - 1) / pl.R);
  const int nkb = a.kout / KB;
  pl.P = std::max(1, std::min(cus / nkb, pl.ntiles));
  pl.ok = true;
  return pl;
}

}  // namespace hfp

bool conv_hfp_supported(const ConvTapArgs& a) {
  if (a.dtype != kBF16 && a.dtype != kF16) return false;
  if (a.ntaps != 9 || a.c % 64 || a.kout % 128 || a.c <= 0 || a.kout <= 0 || a.n <= 0) return false;
  if (a.ish != 1 || a.isw != 1 || a.osh != 1 || a.osw != 1 || a.oph != 0 || a.opw != 0) return false;
  if (a.oh != a.ih || a.ow != a.iw || a.oht != a.oh || a.owt != a.ow) return false;
  if (a.scale || a.bias || a.residual || a.mask || a.relu) return false;
  for (int t = 0; t < 9; ++t)
    if (a.dh[t] != t / 3 - 1 || a.dw[t] != t % 3 - 1) return false;
  const int64_t xb = (int64_t)a.n * a.ih * a.iw * a.c * 2, yb = (int64_t)a.n * a.oh * a.ow * a.kout * 2;
  const int64_t wb = (int64_t)a.kout * 9 * a.c * 2;
  if (xb >= (1ll << 31) - (1ll << 24) || yb >= (1ll << 31) || wb >= (1ll << 31)) return false;
  if (((uintptr_t)a.in & 15) || ((uintptr_t)a.out & 15) || ((uintptr_t)a.wt & 15)) return false;
  return hfp::make_plan(a, 256).ok;
}

// Default route only for small images (h * w <= 64: 7 x 7 at ResNet-50 stage 4, where the tap GEMM's
// M tiles are mostly ragged: fwd 98 vs 109 us, dgrad 87 vs 123 us at 7x7x512 bs 256); at 14 x 14 /
// 28 x 28 the tap GEMM is as fast or faster (76 vs 73 / 102 vs 97 us dgrad; profiles/r05/
// halo_fprop_ab_r05d.jsonl).  APEX_AMD_CONV_HFP=1: that small-image route (off by default, see
// below), =all: wherever supported, unset / 0: never.
static int g_hfp_mode = -1;  // conv_hfp_set_mode: -1 = the environment's choice
void conv_hfp_set_mode(int mode) { g_hfp_mode = mode; }

bool conv_hfp_default(const ConvTapArgs& a) {
  static const int env_mode = [] {
    const char* e = std::getenv("APEX_AMD_CONV_HFP");
    if (e && e[0] == '1') return 1;
    if (e && e[0] == 'a') return 2;
    // off by default since round 6: the tap kernel (fprop2 128 x 128) now runs the 7x7x512
    // forward faster than this kernel in the whole step (same-box A/B 12,477-12,487 vs
    // 12,457-12,460 img/s, profiles/r06/ab_ds_hfp_r06c.txt; its dgrad twin runs 71 us vs 102)
    return 0;
  }();
  const int mode = g_hfp_mode >= 0 ? g_hfp_mode : env_mode;
  if (mode == 0 || !conv_hfp_supported(a)) return false;
  return mode == 2 || (int64_t)a.oh * a.ow <= 64;
}

int conv_hfp_stats_rows(const ConvTapArgs& a, int cus) { return hfp::make_plan(a, cus).P; }

void conv_hfp(const ConvTapArgs& a, const float* pcoef, int cus, hipStream_t s) {
  if (!conv_hfp_supported(a)) throw std::runtime_error("conv_hfp: unsupported shape / epilogue");
  const hfp::Plan pl = hfp::make_plan(a, cus);
  hfp::Args p;
  p.x = static_cast<const uint16_t*>(a.in);
  p.w = static_cast<const uint16_t*>(a.wt);
  p.y = static_cast<uint16_t*>(a.out);
  p.pcoef = pcoef;
  p.stats = a.stats;
  p.shift = a.stats_shift;
  p.n = a.n;
  p.h = a.ih;
  p.wd = a.iw;
  p.c = a.c;
  p.k = a.kout;
  p.R = pl.R;
  p.HC = pl.HC;
  p.rows_total = a.n * a.oh;
  p.ntiles = pl.ntiles;
  p.P = pl.P;
  p.div_h = make_fastdiv((uint32_t)a.ih);
  p.div_hp = make_fastdiv((uint32_t)(a.ih + 2));
  p.div_w = make_fastdiv((uint32_t)a.iw);
  p.div_hc = make_fastdiv((uint32_t)pl.HC);
  p.xbytes = (int)((int64_t)a.n * a.ih * a.iw * a.c * 2);
  p.wbytes = (int)((int64_t)a.kout * 9 * a.c * 2);
  p.ybytes = (int)((int64_t)a.n * a.oh * a.ow * a.kout * 2);
  const unsigned grid = (unsigned)(pl.P * (a.kout / hfp::KB));
  dispatch_16(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    auto go = [&](auto kern) {
      static thread_local const void* done[8] = {};
      const void* fp = reinterpret_cast<const void*>(kern);
      bool seen = false;
      for (const void*& d : done) {
        if (d == fp) {
          seen = true;
          break;
        }
        if (!d) {
          (void)hipFuncSetAttribute(fp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hfp::LDS);
          d = fp;
          seen = true;
          break;
        }
      }
      if (!seen) (void)hipFuncSetAttribute(fp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hfp::LDS);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(hfp::NT), hfp::LDS, s, p);
    };
    const bool st = a.stats != nullptr;
    if (pcoef) {
      if (st) go(hfp::fprop_kernel<T, true, true>);
      else go(hfp::fprop_kernel<T, true, false>);
    } else {
      if (st) go(hfp::fprop_kernel<T, false, true>);
      else go(hfp::fprop_kernel<T, false, false>);
    }
  }, "conv_hfp");
  check_launch("conv_hfp");
}

}  // namespace apex_amd
