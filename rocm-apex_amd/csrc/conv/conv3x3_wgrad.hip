// Halo-tile 3x3 (pad 1, stride 1) weight gradient for gfx950: dW[k][tap][c] = sum over output
// pixels p of dY[p][k] * X[p shifted by tap][c], NHWC bf16 / fp16, fp32 accumulation.
//
// Why not the per-tap split-M kernel (conv_igemm.hip wgrad2_kernel) or MIOpen's igemm_wrw: both
// stage the shifted input ONCE PER TAP (9 gathers of the same rows per pixel tile) and re-stage
// dY for every tap's column block, so at ResNet-50 shapes they run at 15-20 % of the MFMA peak
// (profiles/resnet50_node_r04z.md: igemm_wrw 117-154 us per 59-GFLOP conv).  Here:
//   * a workgroup owns an output block of KB (64 / 128) output channels x ALL 9 taps x 64 input
//     channels, and walks a contiguous range of pixel TILES: R output rows of one image (or G
//     whole small images), at most 112 pixels (7 reduction slices of 16);
//   * per tile the dY rows [112][KB] and the input HALO [(R + 2) x HC slots][64] (zero outside the
//     image, HC >= w + 2 columns) are staged into LDS ONCE by buffer_load ... lds (out-of-range
//     offsets fill zeros: padding, ragged tails, images past the batch), through a 3-stage ring
//     with counted vmcnt and a raw barrier (cdna_hip_programming.md "Pipelining across barriers");
//   * every tap reads its shifted window straight out of the halo: for a 16-pixel slice each lane
//     holds the halo slot of its two pixel rows (tile-invariant, computed once), the tap's column
//     shift is one of three precomputed addresses and its row shift an instruction-immediate
//     offset (HC % 4 == 0 keeps the bank swizzle invariant under row shifts);
//   * one dY fragment feeds 9 MFMAs (one per tap), so per 32x32x16 MFMA a wave reads ~1.1 (TK 1)
//     or ~0.6 (TK 2) fragments from LDS, both operands through ds_read_b64_tr_b16 (pixel-major
//     images, the reduction dim is their row).
// Each workgroup writes its fp32 partial block ([split][k][9][c]); a fixed-order pass sums the
// splits (deterministic, no float atomics).
// Reference capability: the weight-gradient graphs of apex/contrib/bottleneck
// (apex/contrib/csrc/bottleneck/bottleneck.cpp:2236 bottleneck_backward_wgrad2), which run on
// cuDNN there and not at all on ROCm.
#include "apex_amd/conv_api.h"
#include "apex_amd/conv_halo.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/mfma.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace apex_amd {
namespace hwg {
using namespace mfma;

constexpr int NS = 7;           // 16-pixel reduction slices per tile
constexpr int NPP = NS * 16;    // tile pixel capacity

struct Args {
  const uint16_t* x;   // [n][ih][iw][c]
  const uint16_t* dy;  // [n][h][w][k]
  float* ws;           // [splits][k][9][c]
  const float* xcoef;  // nullable [2][c]: x' = relu(x * xcoef[c] + xcoef[c + C]) (the producing BN + ReLU)
  int h, w, c, k;      // output grid, channels
  int ih, iw;          // input grid (= h, w at stride 1; 2h, 2w at stride 2)
  int he;              // stride 2: halo slots of the even-column plane (w + 1; odd plane follows)
  int R, HR, HC, hs;   // tile rows, halo rows / columns per image block, halo slots (G * HR * HC)
  int np;              // real pixels per tile (G * R * w)
  int tpi;             // tiles per image (h / R); 1 for whole-image tiles
  int ntiles, splits, nblk_c;
  int xbytes, dybytes;
};

// NW waves: 4 (one per SIMD: 64 output channels, a 3-stage ring) or 8 (two per SIMD sharing each
// halo tile: 128 output channels, so a staged halo feeds twice the MFMAs; 2-stage ring to fit the
// LDS; APEX_AMD_HWG_NW=8)
// ST 2 (stride-2 convs): the halo of R output rows is 2R + 1 input rows, its columns split into an
// even plane (input columns -1, 1, 3, ...) and an odd plane (0, 2, ...), so the three column taps of
// consecutive output pixels read consecutive slots as at stride 1; ~4x the halo per pixel, so a
// 2-stage ring (no prologue form)
template <int TK, int HSL, int HC_, int NW_ = 4, int ST = 1, int NS_ = NS>
struct Cfg {
  static constexpr int NW = NW_, NT = NW * 64;
  static constexpr int S = (NW == 8 || ST == 2) ? 2 : 3;  // LDS ring stages
  static constexpr int HC = HC_;                       // halo columns (slots per halo row)
  static constexpr int KB = 32 * (NW / 2) * TK;        // output channels per workgroup
  // dY image rows (DMA count % NW == 0); the stride-2 8-wave form stages just its slices' rows
  static constexpr int DYR = (ST == 2 && NW == 8) ? NS_ * 16 : ((TK == 1 || NW == 8) ? 128 : 112);
  static constexpr int DYI = DYR * KB * 2 / 1024;      // dY DMA instructions per tile
  static constexpr int HI = HSL / 8;                   // halo DMA instructions per tile (8 slots each)
  static constexpr int DYW = DYI / NW, HW = HI / NW;   // per wave
  static constexpr int PER = DYW + HW;
  static constexpr int DY_EL = DYR * KB;               // dY image (elements)
  static constexpr int STAGE_EL = DY_EL + HSL * 64;    // one ring stage (elements)
  static constexpr size_t LDS = (size_t)S * STAGE_EL * 2;
  static_assert(DYI % NW == 0 && HI % NW == 0, "DMA instructions must split evenly over the waves");
  static_assert(DYR >= NS_ * 16, "dY image holds the tile");
  static_assert(LDS <= 160 * 1024, "ring exceeds the 160 KiB LDS");
};

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint16_t* lds_dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff, 0, 0,
                                           0);
}

// 16-byte chunk swizzle of a pixel-major image row r (W elements per row) read by
// ds_read_b64_tr_b16: the 4 consecutive rows a 16-lane group reads land in 4 different 64-byte
// quarters of the bank row
template <int W>
__device__ __forceinline__ int swz(int r) {
  return W == 64 ? ((r >> 1) & 1) : (r & 3);
}

template <int W>
__device__ __forceinline__ int img_addr(int row, int col) {
  const int ck = col >> 3, off = col & 7;
  return row * W + ((ck ^ (swz<W>(row) << 2)) << 3) + off;
}

__device__ __forceinline__ s16x8 frag2(const uint16_t* lo, const uint16_t* hi) {
  const s16x4 a = tr_read(lo), b = tr_read(hi);
  return s16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <typename T, int TK, int HSL, int HC, bool PRO, int NW = 4, int ST = 1, int NSL = NS>
__global__ void __launch_bounds__(NW * 64, 1) wgrad_kernel(const Args p) {
  using C = Cfg<TK, HSL, HC, NW, ST, NSL>;
  static_assert(ST == 1 || !PRO, "stride 2: no prologue form");
  constexpr int KB = C::KB, S = C::S;
  static_assert(!(PRO && S < 3), "the BN prologue rewrites the next tile's halo under the current MFMAs: 3 stages");
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, lh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = wave >> 1, ct = wave & 1;  // kout tiles kg*TK .. +TK-1, c tile ct (32 channels)
  const int nblk = (p.k / KB) * p.nblk_c;
  const int wg = xcd_remap(blockIdx.x, nblk * p.splits);
  // consecutive workgroups (one XCD) share a pixel range: dY / halo re-reads hit that XCD's L2
  const int split = wg / nblk, blk = wg - split * nblk;
  const int k0 = (blk / p.nblk_c) * KB, c0 = (blk % p.nblk_c) * 64;
  const int t_begin = (int)((int64_t)split * p.ntiles / p.splits);
  const int t_end = (int)((int64_t)(split + 1) * p.ntiles / p.splits);
  const int nt = t_end - t_begin;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, __builtin_amdgcn_readfirstlane(p.xbytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t dr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, 0, __builtin_amdgcn_readfirstlane(p.dybytes), 0x00020000);

  // ---- DMA constants of this lane (tile-invariant) ----
  int dyrow[C::DYW];
  uint32_t dyrel[C::DYW];
#pragma unroll
  for (int i = 0; i < C::DYW; ++i) {
    const int j = i * NW + wave;
    int row, sc;
    if constexpr (KB == 64) {
      row = 8 * j + (lane >> 3);
      sc = (lane & 7) ^ (swz<64>(row) << 2);
    } else {
      row = 4 * j + (lane >> 4);
      sc = (lane & 15) ^ (swz<128>(row) << 2);
    }
    dyrow[i] = row;
    dyrel[i] = (uint32_t)((row * p.k + k0 + 8 * sc) * 2);
  }
  int hrel[C::HW];
  uint32_t hfl[C::HW];  // bit 0: column in range, bit 1: top halo row, bit 2: bottom halo row
  const int hblk = p.HR * HC;
#pragma unroll
  for (int i = 0; i < C::HW; ++i) {
    const int j = i * NW + wave;
    const int slot = 8 * j + (lane >> 3);
    const int sc = (lane & 7) ^ (swz<64>(slot) << 2);
    const int gi = slot / hblk, rem = slot - gi * hblk;
    const int hy = rem / HC, hj = rem - hy * HC;
    const int hx = ST == 1 ? hj : (hj < p.he ? 2 * hj : 2 * (hj - p.he) + 1);
    const bool ok = slot < p.hs && hx >= 1 && hx <= p.iw;
    hrel[i] = (((gi * p.ih + hy - 1) * p.iw) + hx - 1) * p.c * 2 + (c0 + 8 * sc) * 2;
    // (stride 2: the last halo row, input row 2 (y0 + R) - 1, is inside the image)
    hfl[i] = (ok ? 1u : 0u) | (hy == 0 ? 2u : 0u) | (ST == 1 && hy == p.HR - 1 ? 4u : 0u);
  }
  // PRO (the producing BN + ReLU, x' = relu(x * xcoef[c] + xcoef[C + c])): every lane rewrites the
  // 16-byte halo chunks IT loaded once their DMA has landed (no barrier needed before that; the
  // stage's publishing barrier follows), interleaved with the previous tile's MFMA slices.
  // Chunks the DMA zero-filled (padding, ragged tails, images past the batch) stay zero.  A
  // lane's chunks hold channel group (lane & 7) or (lane & 7) ^ 4 (the slot's swizzle bit).
  float xs[PRO ? 2 : 1][8], xb[PRO ? 2 : 1][8];
  uint32_t hsw = 0;
  if constexpr (PRO) {
#pragma unroll
    for (int gsel = 0; gsel < 2; ++gsel) {
      const int ch = c0 + 8 * ((lane & 7) ^ (4 * gsel));
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xs[gsel][e] = p.xcoef[ch + e];
        xb[gsel][e] = p.xcoef[p.c + ch + e];
      }
    }
#pragma unroll
    for (int i = 0; i < C::HW; ++i)
      if (swz<64>(8 * (i * NW + wave) + (lane >> 3))) hsw |= 1u << i;
  }

  auto issue = [&](int t, int stage) -> uint32_t {
    const int px0 = t * p.np;
    const int y0 = (t % p.tpi) * p.R;
    const uint32_t kill = (y0 == 0 ? 2u : 0u) | (y0 + p.R == p.h ? 4u : 0u);
    uint16_t* base = lds + stage * C::STAGE_EL;
    const uint32_t dyo = (uint32_t)px0 * (uint32_t)p.k * 2u;
#pragma unroll
    for (int i = 0; i < C::DYW; ++i) {
      const uint32_t voff = dyrow[i] < p.np ? dyo + dyrel[i] : 0x80000000u;
      bdma16(dr, voff, base + (i * NW + wave) * 512);
    }
    const int xo = px0 * (ST * ST) * p.c * 2;  // the tile's input origin (ih = ST h, iw = ST w)
    uint32_t vm = 0;  // bit i: halo chunk i of this lane holds image data (PRO rewrites it)
#pragma unroll
    for (int i = 0; i < C::HW; ++i) {
      const bool valid = (hfl[i] & 1u) && !(hfl[i] & kill);
      vm |= valid ? 1u << i : 0u;
      const uint32_t voff = valid ? (uint32_t)(xo + hrel[i]) : 0x80000000u;
      bdma16(xr, voff, base + C::DY_EL + (i * NW + wave) * 512);
    }
    return vm;
  };
  auto xform = [&](int stage, uint32_t vm, int i) {
    if constexpr (PRO) {
      if (!((vm >> i) & 1u)) return;
      uint16_t* q = lds + stage * C::STAGE_EL + C::DY_EL + (i * NW + wave) * 512 + lane * 8;
      const int gsel = (hsw >> i) & 1u;
      float v[8];
      Vec8<T>::load(v, reinterpret_cast<const T*>(q));
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(fmaf(v[e], gsel ? xs[1][e] : xs[0][e], gsel ? xb[1][e] : xb[0][e]), 0.f);
      Vec8<T>::store(reinterpret_cast<T*>(q), v);
    }
  };

  // ---- fragment addresses (elements from a stage base; tile-invariant) ----
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  int aaddr[TK][2];
#pragma unroll
  for (int i = 0; i < TK; ++i) {
    const int col = 32 * (kg * TK + i) + 16 * (g & 1) + 4 * pp;
    const int r0 = 8 * (g >> 1) + q;
    aaddr[i][0] = img_addr<KB>(r0, col);
    aaddr[i][1] = img_addr<KB>(r0 + 4, col);
  }
  // halo: per slice, lo / hi pixel row, tap column shift dw = -1, 0, 1 at tap row dh = -1 (dh = 0
  // and 1 add HC and 2 HC slots: an instruction-immediate offset, HC being a compile-time size)
  int baddr[NSL][2][3];
  {
    const int col = 32 * ct + 16 * (g & 1) + 4 * pp;
    const int rw = p.R * p.w;
#pragma unroll
    for (int s = 0; s < NSL; ++s)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {
        const int px = 16 * s + 8 * (g >> 1) + q + 4 * hl;
        // slots of tap row 0, column taps 0 / 1 / 2 (pixel rows past the tile: any real slots,
        // their dY rows are zero)
        int sl0 = 0, sl1 = 1, sl2 = 2;
        if (px < p.np) {
          const int gi = px / rw, rem = px - gi * rw;
          const int y = rem / p.w, x = rem - y * p.w;
          const int rb = (gi * p.HR + ST * y) * HC;
          sl0 = rb + x;
          sl1 = ST == 1 ? rb + x + 1 : rb + p.he + x;
          sl2 = rb + x + (ST == 1 ? 2 : 1);
        }
        baddr[s][hl][0] = C::DY_EL + img_addr<64>(sl0, col);
        baddr[s][hl][1] = C::DY_EL + img_addr<64>(sl1, col);
        baddr[s][hl][2] = C::DY_EL + img_addr<64>(sl2, col);
      }
  }

  f32x16 acc[TK][9];
#pragma unroll
  for (int i = 0; i < TK; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = zero16();

  uint32_t vq0 = 0, vq1 = 0, vq2 = 0;  // halo valid masks of tiles it, it + 1, it + 2
#pragma unroll
  for (int st = 0; st < S - 1; ++st)
    if (st < nt) {
      const uint32_t m = issue(t_begin + st, st);
      if (st == 0) vq0 = m;
      else vq1 = m;
    }
  if constexpr (PRO) {
    if (nt > 0) {  // tile 0's own chunks (tile 1's DMA may stay in flight)
      if (nt > 1 && S > 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < C::HW; ++i) xform(0, vq0, i);
    }
  }

  for (int it = 0; it < nt; ++it) {
    // this wave's DMA of tile it has landed (younger tiles may still be in flight); the barrier
    // publishes every wave's pieces and retires every wave's reads of the stage refilled next
    const int ahead = min(nt - 1 - it, S - 2);
    if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + S - 1 < nt) vq2 = issue(t_begin + it + S - 1, (it + S - 1) % S);
    const uint16_t* sb = lds + (it % S) * C::STAGE_EL;
    const bool xnext = PRO && it + 1 < nt;  // PRO: rewrite tile it + 1's chunks under these MFMAs
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      s16x8 af[TK], bf[9];
#pragma unroll
      for (int i = 0; i < TK; ++i)
        af[i] = frag2(sb + aaddr[i][0] + s * 16 * KB, sb + aaddr[i][1] + s * 16 * KB);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int dh = t / 3, dw = t % 3;
        bf[t] = frag2(sb + baddr[s][0][dw] + dh * HC * 64, sb + baddr[s][1][dw] + dh * HC * 64);
      }
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < TK; ++i) acc[i][t] = mma<T>(af[i], bf[t], acc[i][t]);
      if constexpr (PRO) {
        if (xnext) {
          if (s == 0) {  // tile it + 1's DMA landed (tile it + 2's may stay in flight)
            if (S > 2 && it + 2 < nt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::PER) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
#pragma unroll
          for (int i = s * C::HW / NSL; i < (s + 1) * C::HW / NSL; ++i) xform((it + 1) % S, vq1, i);
        }
      }
    }
    vq0 = vq1;
    vq1 = vq2;
    vq2 = 0;
  }

  // ---- fp32 partial block: lane holds c = c0 + 32 ct + lr, k rows crow(r, lh) ----
  float* dst = p.ws + (int64_t)split * p.k * 9 * p.c;
#pragma unroll
  for (int i = 0; i < TK; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kr = k0 + 32 * (kg * TK + i) + crow(r, lh);
        dst[((int64_t)kr * 9 + t) * p.c + c0 + 32 * ct + lr] = acc[i][t][r];
      }
}

// fixed-order sum of the split partials (16 thread groups per block each take every 16th split,
// then one LDS fold in group order)
template <typename TO>
__global__ void __launch_bounds__(256) reduce_kernel(const float* __restrict__ part, int splits, int64_t n,
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
      for (int e = 0; e < 8; ++e) a[e] += t8[e];
    }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[grp][v * 8 + e] = a[e];
  __syncthreads();
  if (grp != 0 || i >= n) return;
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = 0.f;
  for (int g2 = 0; g2 < 16; ++g2)
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] += red[g2][v * 8 + e];
  Vec8<TO>::store(out + i, a);
}

// ---- launch plan ----
// Instantiated (TK, halo slots, halo columns) tuples, in order of preference: 128-channel blocks
// where the ring still holds 3 stages (28 x 28 / 14 x 14 at ResNet-50 widths), else 64.
struct Inst {
  int tk, hsl, hc;
};
// (TK 2 — 18 accumulator tiles, 288 registers per lane — does not fit beside the operands without
// spilling on hipcc 7.2, so every block is 64 output channels for now)
constexpr Inst kInst[] = {{1, 224, 12}, {1, 256, 16}, {1, 256, 32}, {1, 256, 60}};

struct Plan {
  bool ok;
  int tk, hsl, R, G, HR, HC, hs, np, tpi, ntiles, splits, nblk_c, nw, st, ns, he;
};

// stride-2 instances (4 waves, 64 output channels, 2-stage ring): (halo slots, halo columns,
// 16-pixel slices) — 7 x 7 / 14 x 14 outputs (two whole images / 7 rows per tile, 98 pixels of
// 112) and 28 x 28 (2 rows, 56 pixels of 64); halo slots % 32 == 0 (the DMA split over 4 waves)
// 8-wave forms (128 output channels share each staged halo: half the halo bytes per MFMA, the
// stride-2 kernel's limit) where the 2-stage ring fits: 28 x 28 (2 rows), 14 x 14 (2 rows) and
// 7 x 7 (one image)
struct Inst2 {
  int hsl, hc, ns, nw;
};
constexpr Inst2 kInst2[] = {{480, 16, 7, 4}, {480, 32, 7, 4}, {320, 60, 4, 4}, {320, 60, 4, 8}, {256, 16, 4, 8},
                            {192, 32, 2, 8}};

// 8-wave workgroups (128 output channels per staged halo: two waves per SIMD, half the halo
// staging per MFMA) wherever kout % 128 == 0 and no prologue: 92 -> 80 us at 7x7 / 14x14, 82.5 ->
// 74.5 us at 28x28 in the step (profiles/r06/resnet50_step_timeline_r06m.md), whole step +0.15 %
// same box (profiles/r06/ab_hwg_nw8_r06l.txt).  APEX_AMD_HWG_NW=4 restores the 4-wave kernel.
inline int env_nw() {
  static const int v = [] {
    const char* e = std::getenv("APEX_AMD_HWG_NW");
    return e && std::atoi(e) == 4 ? 4 : 8;
  }();
  return v;
}

// tile geometry for halo width hc and slot budget hsl: rows of one image (the largest divisor of
// h whose pixels and halo fit) or, for small images, as many whole images as fit
inline bool tile_geo(int h, int w, int hc, int hsl, int& R, int& G) {
  if (w + 2 > hc) return false;
  R = 0;
  G = 1;
  if (h * w <= NPP / 2) {
    if ((h + 2) * hc > hsl) return false;
    R = h;
    G = std::max(1, std::min(NPP / (h * w), hsl / ((h + 2) * hc)));
    return true;
  }
  for (int r = h; r >= 1; --r)
    if (h % r == 0 && r * w <= NPP && (r + 2) * hc <= hsl) {
      R = r;
      return true;
    }
  return false;
}

// stride 2: R output rows (a divisor of h) or G whole images per tile, 2R + 1 halo rows, columns
// w + 1 (even plane) + w (odd plane) <= hc
inline bool tile_geo2(int h, int w, Inst2 in, int& R, int& G) {
  if (2 * w + 1 > in.hc) return false;
  const int npp = in.ns * 16;
  R = 0;
  G = 1;
  if (h * w <= npp / 2) {
    if ((2 * h + 1) * in.hc > in.hsl) return false;
    R = h;
    G = std::max(1, std::min(npp / (h * w), in.hsl / ((2 * h + 1) * in.hc)));
    return true;
  }
  for (int r = h; r >= 1; --r)
    if (h % r == 0 && r * w <= npp && (2 * r + 1) * in.hc <= in.hsl) {
      R = r;
      return true;
    }
  return false;
}

inline Plan make_plan(const ConvTapArgs& a, int cus, bool pro = false) {
  Plan pl{};
  pl.ok = false;
  const int h = a.oh, w = a.ow;
  if (w < 1 || h < 1) return pl;
  pl.st = a.ish;
  pl.ns = NS;
  pl.he = 0;
  if (pl.st == 2) {
    if (pro) return pl;
    pl.tk = 1;
    const bool nw8 = a.kout % 128 == 0 && env_nw() == 8;
    double best = -1.0;
    for (Inst2 in : kInst2) {
      int R, G;
      if ((in.nw == 8 && !nw8) || !tile_geo2(h, w, in, R, G)) continue;
      // pixel-slot efficiency, 8-wave forms weighted 1.3x (half the halo traffic per MFMA)
      const double eff = (double)(G * R * w) / (in.ns * 16) * (in.nw == 8 ? 1.3 : 1.0);
      if (eff > best + 1e-9) {
        best = eff;
        pl.nw = in.nw;
        pl.hsl = in.hsl;
        pl.HC = in.hc;
        pl.ns = in.ns;
        pl.R = R;
        pl.G = G;
      }
    }
    if (best < 0) return pl;
    pl.HR = 2 * pl.R + 1;
    pl.he = w + 1;
  } else {
    pl.nw = (!pro && a.kout % 128 == 0) ? env_nw() : 4;
    double best = -1.0;
    for (Inst in : kInst) {
      if (in.tk == 2 && a.kout % 128) continue;
      if (pl.nw == 8) in.hsl = 256;  // (the 8-wave DMA split needs halo pieces % 8)
      int R, G;
      if (!tile_geo(h, w, in.hc, in.hsl, R, G)) continue;
      // pixel-slot efficiency, with a 10 % bonus for the 128-channel block (half the halo re-reads)
      const double eff = (double)(G * R * w) / NPP * (in.tk == 2 ? 1.1 : 1.0);
      if (eff > best + 1e-9) {
        best = eff;
        pl.tk = in.tk;
        pl.hsl = in.hsl;
        pl.HC = in.hc;
        pl.R = R;
        pl.G = G;
      }
    }
    if (best < 0) return pl;
    pl.HR = pl.R + 2;
  }
  pl.hs = pl.G * pl.HR * pl.HC;
  pl.np = pl.G * pl.R * w;
  pl.tpi = pl.G > 1 ? 1 : h / pl.R;
  pl.ntiles = pl.G > 1 ? (a.n + pl.G - 1) / pl.G : a.n * pl.tpi;
  pl.nblk_c = a.c / 64;
  const int nblk = (a.kout / (32 * (pl.nw / 2) * pl.tk)) * pl.nblk_c;
  int sp = std::max(1, cus / nblk);
  sp = std::min(sp, pl.ntiles);
  pl.splits = sp;
  pl.ok = true;
  return pl;
}

}  // namespace hwg

bool conv_hwgrad_supported(const ConvTapArgs& a) {
  if (a.dtype != kBF16 && a.dtype != kF16) return false;
  if (a.ntaps != 9 || a.c % 64 || a.kout % 64 || a.c <= 0 || a.kout <= 0 || a.n <= 0) return false;
  // stride 1 (same-size output) or stride 2 of an even-sized input (ih = 2 oh, iw = 2 ow)
  if (a.ish != a.isw || (a.ish != 1 && a.ish != 2)) return false;
  if (a.osh != 1 || a.osw != 1 || a.oph != 0 || a.opw != 0) return false;
  if (a.ih != a.ish * a.oh || a.iw != a.isw * a.ow || a.oht != a.oh || a.owt != a.ow) return false;
  for (int t = 0; t < 9; ++t)
    if (a.dh[t] != t / 3 - 1 || a.dw[t] != t % 3 - 1) return false;
  const int64_t xb = (int64_t)a.n * a.ih * a.iw * a.c * 2, db = (int64_t)a.n * a.oh * a.ow * a.kout * 2;
  // buffer ranges, and the per-tile byte origins in 32 bits with a tile of headroom
  if (xb + (int64_t)hwg::NPP * 8 * a.ish * a.isw * a.c * 2 >= (1ll << 31) || db + (int64_t)hwg::NPP * a.kout * 2 >= (1ll << 31))
    return false;
  if (((uintptr_t)a.in & 15) || ((uintptr_t)a.out & 15)) return false;
  return hwg::make_plan(a, 256).ok;
}

int64_t conv_hwgrad_workspace_floats(const ConvTapArgs& a, int cus) {
  // (the prologue form always plans 4 waves; the plain form may plan 8 with fewer splits: size for
  // the larger of the two so one workspace serves either)
  const hwg::Plan pl = hwg::make_plan(a, cus);
  const hwg::Plan p4 = hwg::make_plan(a, cus, true);
  if (p4.splits > pl.splits) return (int64_t)p4.splits * a.kout * 9 * a.c;
  return (int64_t)pl.splits * a.kout * 9 * a.c;
}

void conv_hwgrad(const ConvTapArgs& a, const void* dy, void* dw_out, int out_dtype, float* ws, int cus,
                 hipStream_t s) {
  conv_hwgrad_pro(a, dy, dw_out, out_dtype, ws, cus, s, nullptr);
}

void conv_hwgrad_pro(const ConvTapArgs& a, const void* dy, void* dw_out, int out_dtype, float* ws, int cus,
                     hipStream_t s, const float* xcoef) {
  if (!conv_hwgrad_supported(a) || ((uintptr_t)dy & 15) || ((uintptr_t)dw_out & 15) || ((uintptr_t)ws & 15))
    throw std::runtime_error("conv_hwgrad: unsupported shape / dtype / alignment");
  const hwg::Plan pl = hwg::make_plan(a, cus, xcoef != nullptr);
  hwg::Args p;
  p.x = static_cast<const uint16_t*>(a.in);
  p.dy = static_cast<const uint16_t*>(dy);
  p.ws = ws;
  p.xcoef = xcoef;
  p.h = a.oh;
  p.w = a.ow;
  p.ih = a.ih;
  p.iw = a.iw;
  p.he = pl.he;
  p.c = a.c;
  p.k = a.kout;
  p.R = pl.R;
  p.HR = pl.HR;
  p.HC = pl.HC;
  p.hs = pl.hs;
  p.np = pl.np;
  p.tpi = pl.tpi;
  p.ntiles = pl.ntiles;
  p.splits = pl.splits;
  p.nblk_c = pl.nblk_c;
  p.xbytes = (int)((int64_t)a.n * a.ih * a.iw * a.c * 2);
  p.dybytes = (int)((int64_t)a.n * a.oh * a.ow * a.kout * 2);
  const int nblk = (a.kout / (32 * (pl.nw / 2) * pl.tk)) * pl.nblk_c;
  const unsigned grid = (unsigned)(nblk * pl.splits);
  dispatch_16(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    auto go = [&](auto kern, size_t lds) {
      // the LDS opt-in once per kernel instance (a per-launch attribute call is host time on
      // every step of an eager training loop)
      static thread_local const void* done[16] = {};
      const void* fp = reinterpret_cast<const void*>(kern);
      bool seen = false;
      for (const void*& d : done) {
        if (d == fp) {
          seen = true;
          break;
        }
        if (!d) {
          (void)hipFuncSetAttribute(fp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
          d = fp;
          seen = true;
          break;
        }
      }
      if (!seen) (void)hipFuncSetAttribute(fp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(pl.nw * 64), lds, s, p);
    };
#define HWG_CASE2(HSL_, HC_, NS_, NW_)                                                              \
  if (pl.st == 2 && pl.nw == NW_ && pl.hsl == HSL_ && pl.HC == HC_ && pl.ns == NS_) {                  \
    go(hwg::wgrad_kernel<T, 1, HSL_, HC_, false, NW_, 2, NS_>, hwg::Cfg<1, HSL_, HC_, NW_, 2, NS_>::LDS);  \
    return;                                                                                         \
  }
    HWG_CASE2(480, 16, 7, 4) HWG_CASE2(480, 32, 7, 4) HWG_CASE2(320, 60, 4, 4) HWG_CASE2(320, 60, 4, 8)
    HWG_CASE2(256, 16, 4, 8) HWG_CASE2(192, 32, 2, 8)
#undef HWG_CASE2
#define HWG_CASE(TK_, HSL_, HC_)                                                                    \
  if (pl.st == 1 && pl.nw == 4 && pl.tk == TK_ && pl.hsl == HSL_ && pl.HC == HC_) {                               \
    if (xcoef) go(hwg::wgrad_kernel<T, TK_, HSL_, HC_, true>, hwg::Cfg<TK_, HSL_, HC_>::LDS);           \
    else go(hwg::wgrad_kernel<T, TK_, HSL_, HC_, false>, hwg::Cfg<TK_, HSL_, HC_>::LDS);                \
    return;                                                                                         \
  }                                                                                                 \
  if (pl.st == 1 && pl.nw == 8 && !xcoef && pl.tk == TK_ && pl.hsl == 256 && pl.HC == HC_) {                        \
    go(hwg::wgrad_kernel<T, TK_, 256, HC_, false, 8>, hwg::Cfg<TK_, 256, HC_, 8>::LDS);                \
    return;                                                                                         \
  }
    HWG_CASE(1, 224, 12) HWG_CASE(1, 256, 16) HWG_CASE(1, 256, 32) HWG_CASE(1, 256, 60)
#undef HWG_CASE
    throw std::runtime_error("conv_hwgrad: no kernel for the plan");
  }, "conv_hwgrad");
  const int64_t n = (int64_t)a.kout * 9 * a.c;
  const int64_t blocks = (n / 8 + 15) / 16;
  dispatch_float(out_dtype, [&](auto tag) {
    using TO = typename decltype(tag)::type;
    hipLaunchKernelGGL((hwg::reduce_kernel<TO>), dim3((unsigned)blocks), dim3(256), 0, s, (const float*)ws, pl.splits,
                       n, (TO*)dw_out);
  }, "conv_hwgrad out");
  check_launch("conv_hwgrad");
}

}  // namespace apex_amd
