// Memory-bound 1x1 convolutions of the ResNet bottleneck as NHWC GEMMs with the batch norm
// fused in: Y[M, N] = pro(A[M, K]) . W^T, where
//   * pro = the PRODUCING batch norm's apply + ReLU on the operand load (relu(a * s[k] + t[k])),
//     so the normalized activation is never written;
//   * the epilogue emits per-output-channel sum / sum-of-squares partials (about a per-channel
//     shift) from the fp32 accumulators for the CONSUMING batch norm, so its statistics pass never
//     re-reads Y.
// Reference capability: the scale-bias-ReLU-conv-with-BN-statistics graphs of the fused
// bottleneck (apex/contrib/csrc/bottleneck/bottleneck.cpp:1104-1287) and groupbn's separate
// stats / apply kernels (apex/contrib/csrc/groupbn/nhwc_batch_norm_kernel.h) — here one gfx950
// kernel per convolution.
//
// Why a dedicated kernel: at ResNet-50 bs 256 every 1x1 conv of stages 1-2 is ~26 GFLOP over
// 0.25-0.5 GB of activations — 10 us of MFMA against 40-80 us of HBM.  The roofline is the
// activation stream, so the design is built around reading A exactly once:
//   * one wave owns 32 output rows x all NC columns of a tile (NC <= 256: CN = NC / 32
//     v_mfma_f32_32x32x16 accumulator blocks), so A fragments are wave-private and go straight
//     from HBM into registers (16-byte loads, the MFMA A-operand map) — no LDS round trip;
//   * the weight tile [NC][K] (<= 133 KB) is loaded ONCE per persistent workgroup into LDS
//     (rows padded by 16 B: the 32 rows a B-fragment read touches hit distinct 16-B slots);
//   * A fragments are double-buffered in registers one K-chunk (<= 128 deep) ahead, across tiles;
//   * epilogue: bf16 round, staged through a wave-private LDS slab 64 columns at a time and
//     written as 16-byte row vectors; the statistics are per-lane running sums in registers
//     (the C layout puts one column on each lane), reduced once at the end of the kernel.
// dgrad (dX = dY . W) is the same kernel with the weight read transposed into the LDS image.
#include "apex_amd/conv_api.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/fastdiv.h"
#include "apex_amd/mfma.h"

#include <cstdlib>
#include <stdexcept>

namespace apex_amd {
namespace c1bn {
using namespace mfma;

struct Args {
  const uint16_t* a;    // [M][K]
  const uint16_t* w;    // !WT: [ncols][K]  WT: [K][ncols]
  uint16_t* y;          // [M][ncols]
  int64_t m;
  int ncols;            // total output columns (blockIdx.y selects NC of them)
  int ntiles;           // ceil(M / 128)
  const float* pcoef;   // PRO: [2][K] scale | shift of the producing batch norm (then ReLU)
  const float* shift;   // STATS: per-output-channel shift [ncols] (nullable = 0)
  float* part;          // STATS: [2][gridDim.x][ncols] partial sums (S1 slab, then S2 slab)
  const uint16_t* res;  // nullable [M][ncols]: y += res before the store (a residual gradient)
  // rs_w2 > 0: res is the gradient of a stride-2 subsample of this output instead, [N][rs_h2][rs_w2]
  // [ncols] over output rows (n, y, x) of an [N][H][W] image (rs_hw = H W, rs_w = W): only the
  // rows with even y and x get res[n][y / 2][x / 2] (the strided 1x1 downsample's data gradient)
  FastDiv rs_hw, rs_w;
  int rs_h2, rs_w2;
  // PRO == kProBnAddRelu with pc_split: pcoef is the output BN's [scale | shift] [2][K] and pc_res
  // the residual (downsample) BN's [2][K], null = identity; the [4][K] rows are assembled on the
  // LDS load (no separate concatenation launch on the host side)
  const float* pc_res;
  int pc_split;
  const uint16_t* py;   // PRO == kProBnBwd: second operand tensor [M][K] (the BN's input)
  uint16_t* aout;       // PRO == kProBnBwd / kProBnAddRelu, nullable: the transformed operand written out [M][K]
  uint8_t* bout;        // PRO == kProBnAddRelu, nullable: its ReLU bits [M * K / 8] (bit j of byte i = element 8 i + j)
  // RED (dgrad form): the output is the gradient of a ReLU'd batch-norm output (the block
  // below's) — masked with that BN's forward ReLU bits, and its backward reduction
  // sum(g), sum(g * (x - mean)) accumulated per column into part [2][G][ncols]
  const uint8_t* rbits;  // [M * ncols / 8]; null: the mask is recomputed as rx * rcoef[c] + rcoef[C + c] > 0
  const float* rcoef;    // the BN's forward apply coefficients [2][ncols] (recomputed-mask mode)
  const uint16_t* rx;    // the BN's input [M][ncols]
  const float* rmean;    // the BN's batch mean [ncols]
  // RED, nullable: a SECOND batch norm fed by the same (masked) gradient — the downsample BN of
  // the block below, whose output is summed with bn3's before the shared ReLU.  Its reduction
  // sum(g * (x2 - mean2)) is accumulated too and part becomes [4][G][ncols]:
  // [sum g | sum g (x - mean) | sum g | sum g (x2 - mean2)] (two contiguous [2][G] slabs)
  const uint16_t* rx2;
  const float* rmean2;
};

// operand prologues
constexpr int kProNone = 0;
constexpr int kProBnRelu = 1;  // a' = relu(a * c[k] + c[K + k])            (BN apply + ReLU)
constexpr int kProBnBwd = 2;   // a' = c[k] * a + c[K + k] * y + c[2K + k]  (BN backward dx from the
                               //       masked gradient a and the BN input y: bwd_apply fused)
constexpr int kProBnAddRelu = 3;  // a' = relu(fma(a, c[k], c[2K + k]) + fma(y, c[K + k], c[3K + k])): the
                                  //   block below's output BN + residual / downsample BN (y) + ReLU with
                                  //   the apply passes' exact arithmetic, so its apply pass is gone; a'
                                  //   and its ReLU bits are written out for the block's other uses
constexpr int kProBnBwdMask = 4;  // a' = c[k] * (y * c[3K + k] + c[4K + k] > 0 ? a : 0) + c[K + k] * y + c[2K + k]:
                                  //   kProBnBwd with the BN's forward ReLU mask recomputed from y (the
                                  //   unmasked gradient in: the reduction pass writes nothing), the
                                  //   standalone bwd_apply's exact arithmetic
// per-k coefficient rows of a prologue
constexpr int pro_rows(int pro) {
  return pro == kProBnRelu ? 2 : pro == kProBnBwd ? 3 : pro == kProBnAddRelu ? 4 : pro == kProBnBwdMask ? 5 : 0;
}
constexpr bool pro_two(int pro) {  // a second operand
  return pro == kProBnBwd || pro == kProBnAddRelu || pro == kProBnBwdMask;
}

constexpr int kSS = 64 + 8;  // staging row stride (elements): rows h and h+4 land 16 banks apart

constexpr int lds_bytes_nw(int nc, int kr, int pro, bool red, int nw) {
  return nc * (kr + 8) * 2 + nw * 32 * kSS * 2 + pro_rows(pro) * kr * 4 +
         (red ? nw * 3 * nc * 4 : 0);
}

// waves per workgroup: 4 (two workgroups per CU) while the weight image is small; 8 sharing one
// image when a 4-wave workgroup would hold the CU's LDS alone anyway (8 waves either way — a
// 4-wave CU streams at half the rate, profiles/resnet50_node_r03a.md)
constexpr int pick_nw(int nc, int kr, int pro, bool red) {
  return lds_bytes_nw(nc, kr, pro, red, 4) <= 80 * 1024 ? 4
         : lds_bytes_nw(nc, kr, pro, red, 8) <= 160 * 1024 ? 8 : 4;
}

// the weight image leaves ONE 4-wave workgroup per CU: the register file of a whole SIMD per wave
constexpr bool one_wg_per_cu(int nc, int kr, int pro, bool red) {
  return pick_nw(nc, kr, pro, red) == 4 && lds_bytes_nw(nc, kr, pro, red, 4) > 80 * 1024;
}

// RED2: the second (downsample) BN's reduction in the RED epilogue — compile-time, since the
// runtime form cost every single-BN dgrad ~6 % (stage 3: 110.6 -> 117.6 us, r06a vs r06z)
template <typename T, int NC, int KR, bool WT, int PRO, bool STATS, bool RED, int NW, int DEPTH, bool RED2 = false>
__global__ void __launch_bounds__(NW * 64, (NW == 8 || one_wg_per_cu(NC, KR, PRO, RED)) ? 1 : 2) fused1x1(Args p) {
  constexpr int kWaves = NW, kRowsB = NW * 32, NT = NW * 64;
  constexpr int BS = KR + 8;                 // B image row stride (elements)
  constexpr int CN = NC / 32;                // accumulator blocks per wave
  // k depth per register chunk: 128, 64 at 256 columns (128 accumulator registers); the two-
  // tensor BN-backward prologue halves it again (it holds a second operand's fragments)
  constexpr int KCH0 = NC >= 256 ? 64 : 128;
  constexpr int KCH1 = pro_two(PRO) ? KCH0 / 2 : KCH0;
  constexpr int KCH = KR < KCH1 ? KR : KCH1;
  constexpr int KC = KCH / 16;               // k-steps per chunk
  constexpr int NCH = KR / KCH;              // chunks per tile
  static_assert(NC % 64 == 0 && KR % 64 == 0, "tile shape");
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* bimg = lds;                       // [NC][BS]
  uint16_t* stg = lds + NC * BS;              // [kWaves][32][kSS]
  float* pc = reinterpret_cast<float*>(stg + kWaves * 32 * kSS);  // [2 or 3][KR]
  float* rsum = pc + pro_rows(PRO) * KR;  // RED: [kWaves][3][NC]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, lr = lane & 31, lh = lane >> 5;
  const int col0 = blockIdx.y * NC;

  // ---- weight tile -> LDS, once per workgroup ----
  if constexpr (!WT) {
    for (int i = tid; i < NC * KR / 8; i += NT) {
      const int n = i / (KR / 8), k8 = (i % (KR / 8)) * 8;
      *reinterpret_cast<uint4*>(bimg + n * BS + k8) =
          *reinterpret_cast<const uint4*>(p.w + (int64_t)(col0 + n) * KR + k8);
    }
  } else {
    // transposed image: consecutive threads take consecutive k, so the 2-byte LDS stores of a
    // wave land on consecutive addresses (the n-major order put all 64 lanes on two banks:
    // 32-way conflicts, the 29-55 % conflict cycles of the dgrad forms in
    // profiles/pmc_resnet_kernels_r04.md); the 16-byte global reads stride by rows instead (a
    // one-time read of a small, L2-resident weight)
    for (int i = tid; i < NC * KR / 8; i += NT) {
      const int k = i % KR, n8 = (i / KR) * 8;
      const uint4 v = *reinterpret_cast<const uint4*>(p.w + (int64_t)k * p.ncols + col0 + n8);
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bimg[(n8 + 2 * j) * BS + k] = (uint16_t)(w4[j] & 0xffffu);
        bimg[(n8 + 2 * j + 1) * BS + k] = (uint16_t)(w4[j] >> 16);
      }
    }
  }
  // coefficient rows: 16-byte loads (4 consecutive k of one row; KR % 4 == 0, rows start 16-byte
  // aligned when the tensors are), all of a thread's loads issued before its LDS stores
  const bool pc_vec = ((reinterpret_cast<uintptr_t>(p.pcoef) | reinterpret_cast<uintptr_t>(p.pc_res)) & 15) == 0;
  if constexpr (PRO == kProBnAddRelu) {
    if (p.pc_split) {
      if (pc_vec) {
        constexpr int N4 = KR;  // 4 rows x KR / 4 vectors
#pragma unroll 4
        for (int i = tid; i < N4; i += NT) {
          const int row = i / (KR / 4), kk = (i - row * (KR / 4)) * 4;
          float4 v;
          if (row == 0 || row == 2) v = *reinterpret_cast<const float4*>(p.pcoef + (row >> 1) * KR + kk);
          else if (p.pc_res) v = *reinterpret_cast<const float4*>(p.pc_res + (row >> 1) * KR + kk);
          else v = row == 1 ? make_float4(1.f, 1.f, 1.f, 1.f) : make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4*>(pc + row * KR + kk) = v;
        }
      } else {
        for (int i = tid; i < 4 * KR; i += NT) {
          const int row = i / KR, kk = i - row * KR;
          float v;
          if (row == 0 || row == 2) v = p.pcoef[(row >> 1) * KR + kk];
          else if (p.pc_res) v = p.pc_res[(row >> 1) * KR + kk];
          else v = row == 1 ? 1.f : 0.f;
          pc[i] = v;
        }
      }
    } else if (pc_vec) {
#pragma unroll 4
      for (int i = tid; i < KR; i += NT)
        reinterpret_cast<float4*>(pc)[i] = reinterpret_cast<const float4*>(p.pcoef)[i];
    } else {
      for (int i = tid; i < 4 * KR; i += NT) pc[i] = p.pcoef[i];
    }
  } else if constexpr (PRO != kProNone) {
    if (pc_vec) {
#pragma unroll 4
      for (int i = tid; i < pro_rows(PRO) * KR / 4; i += NT)
        reinterpret_cast<float4*>(pc)[i] = reinterpret_cast<const float4*>(p.pcoef)[i];
    } else {
      for (int i = tid; i < pro_rows(PRO) * KR; i += NT) pc[i] = p.pcoef[i];
    }
  }
  float sh[CN], s1[CN], s2[CN];
#pragma unroll
  for (int cb = 0; cb < CN; ++cb) {
    sh[cb] = (STATS && p.shift) ? p.shift[col0 + 32 * cb + lr] : 0.f;
    s1[cb] = s2[cb] = 0.f;
  }
  if constexpr (RED)
    for (int i = tid; i < kWaves * 3 * NC; i += NT) rsum[i] = 0.f;
  __syncthreads();

  f32x16 acc[CN];
#pragma unroll
  for (int cb = 0; cb < CN; ++cb) acc[cb] = zero16();

  constexpr int KY = pro_two(PRO) ? KC : 1;
  struct Frags {
    s16x8 a[KC];
    s16x8 y[KY];
  };
  auto load = [&](Frags& f, int t, int ch) {
    int64_t row = (int64_t)t * kRowsB + wid * 32 + lr;
    if (row >= p.m) row = p.m - 1;  // tail rows: valid memory, masked in the epilogue
    const int64_t off = row * KR + ch * KCH + 8 * lh;
#pragma unroll
    for (int s = 0; s < KC; ++s) f.a[s] = *reinterpret_cast<const s16x8*>(p.a + off + 16 * s);
    if constexpr (pro_two(PRO)) {
#pragma unroll
      for (int s = 0; s < KC; ++s) f.y[s] = *reinterpret_cast<const s16x8*>(p.py + off + 16 * s);
    }
  };

  auto compute = [&](const Frags& f, int t, int ch) {
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      s16x8 a = f.a[s];
      if constexpr (pro_two(PRO)) {
        const int kb = ch * KCH + 16 * s + 8 * lh;
        constexpr int NQ = pro_rows(PRO);
        float c[NQ][8];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const float4 u0 = *reinterpret_cast<const float4*>(pc + q * KR + kb);
          const float4 u1 = *reinterpret_cast<const float4*>(pc + q * KR + kb + 4);
          c[q][0] = u0.x; c[q][1] = u0.y; c[q][2] = u0.z; c[q][3] = u0.w;
          c[q][4] = u1.x; c[q][5] = u1.y; c[q][6] = u1.z; c[q][7] = u1.w;
        }
        unsigned mb = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v;
          if constexpr (PRO == kProBnAddRelu) {
            v = fmaf(to_f(T{(uint16_t)a[j]}), c[0][j], c[2][j]) + fmaf(to_f(T{(uint16_t)f.y[s][j]}), c[1][j], c[3][j]);
            v = fmaxf(v, 0.f);
            mb |= (v > 0.f ? 1u : 0u) << j;
          } else if constexpr (PRO == kProBnBwdMask) {
            const float yv = to_f(T{(uint16_t)f.y[s][j]});
            const float g = fmaf(yv, c[3][j], c[4][j]) > 0.f ? to_f(T{(uint16_t)a[j]}) : 0.f;
            v = fmaf(c[0][j], g, fmaf(c[1][j], yv, c[2][j]));
          } else {
            v = fmaf(c[0][j], to_f(T{(uint16_t)a[j]}), fmaf(c[1][j], to_f(T{(uint16_t)f.y[s][j]}), c[2][j]));
          }
          a[j] = (short)from_f<T>(v).x;
        }
        // BN dx (kProBnBwd: for the weight gradient) / the block output (kProBnAddRelu: the
        // residual and weight-gradient operand of this block): staged in the wave's slab and
        // written out as whole-row runs after the chunk (below) — a fragment puts one row on
        // each lane, so direct stores would touch 32 partial cache lines per instruction
        (void)mb;
        if (p.aout && blockIdx.y == 0)
          *reinterpret_cast<s16x8*>(stg + wid * 32 * kSS + lr * kSS + 16 * s + 8 * lh) = a;
      }
      if constexpr (PRO == kProBnRelu) {
        const int kb = ch * KCH + 16 * s + 8 * lh;
        const float4 c0 = *reinterpret_cast<const float4*>(pc + kb);
        const float4 c1 = *reinterpret_cast<const float4*>(pc + kb + 4);
        const float4 d0 = *reinterpret_cast<const float4*>(pc + KR + kb);
        const float4 d1 = *reinterpret_cast<const float4*>(pc + KR + kb + 4);
        const float sc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float sf[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = fmaxf(fmaf(to_f(T{(uint16_t)a[j]}), sc[j], sf[j]), 0.f);
          a[j] = (short)from_f<T>(v).x;
        }
      }
#pragma unroll
      for (int cb = 0; cb < CN; ++cb) {
        const s16x8 b = *reinterpret_cast<const s16x8*>(bimg + (32 * cb + lr) * BS + ch * KCH + 16 * s + 8 * lh);
        acc[cb] = mma<T>(a, b, acc[cb]);
      }
    }
    if constexpr (pro_two(PRO)) {
      // the chunk's transformed operand [32 rows][KCH] from the slab: KCH / 8 lanes per row, each
      // 16 B (and, for the add + ReLU prologue, its 8 ReLU bits: one byte)
      if (p.aout && blockIdx.y == 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint16_t* sl = stg + wid * 32 * kSS;
        constexpr int LPR = KCH / 8;
        const int64_t row0 = (int64_t)t * kRowsB + wid * 32;
#pragma unroll
        for (int i = 0; i < 32 * LPR / 64; ++i) {
          const int qid = lane + 64 * i, rr = qid / LPR, c8 = (qid % LPR) * 8;
          const s16x8 v = *reinterpret_cast<const s16x8*>(sl + rr * kSS + c8);
          if (row0 + rr < p.m) {
            const int64_t off = (row0 + rr) * KR + ch * KCH + c8;
            *reinterpret_cast<s16x8*>(p.aout + off) = v;
            if constexpr (PRO == kProBnAddRelu) {
              if (p.bout) {
                unsigned mb = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) mb |= (v[j] > 0 ? 1u : 0u) << j;  // relu output: > 0 <=> bits > 0
                p.bout[off >> 3] = (uint8_t)mb;
              }
            }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
  };

  auto epilogue = [&](int t) {
    const int64_t row0 = (int64_t)t * kRowsB + wid * 32;
    if constexpr (STATS) {
#pragma unroll
      for (int cb = 0; cb < CN; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (row0 + crow(r, lh) < p.m) {
            const float d = acc[cb][r] - sh[cb];
            s1[cb] += d;
            s2[cb] = fmaf(d, d, s2[cb]);
          }
        }
    }
    uint16_t* st = stg + wid * 32 * kSS;
#pragma unroll
    for (int g = 0; g < CN / 2; ++g) {
      // this group's residual / reduction operands first: their HBM latency runs under the
      // LDS staging below instead of after it (the compiler barrier keeps loads from being
      // hoisted across the staging otherwise)
      const bool has_res = WT && p.res != nullptr;  // residual add: a dgrad-form option
      uint4 rv[4], xq[4], xq2[4];
      unsigned mbv[4];
      constexpr bool red2 = RED && RED2;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qid = lane + 64 * i, rr = qid >> 3, c8 = (qid & 7) * 8;
        const int64_t off = (row0 + rr) * p.ncols + col0 + 64 * g + c8;
        const bool ok = row0 + rr < p.m;
        rv[i] = make_uint4(0, 0, 0, 0);
        if (has_res && ok) {
          int64_t roff = off;
          bool rok = true;
          if (p.rs_w2 > 0) {  // kernel-argument-uniform branch
            const uint32_t R = (uint32_t)(row0 + rr);
            const uint32_t img = fdiv(R, p.rs_hw), rem = R - img * p.rs_hw.d;
            const uint32_t yy = fdiv(rem, p.rs_w), xx = rem - yy * p.rs_w.d;
            rok = ((yy | xx) & 1u) == 0;
            roff = (((int64_t)img * p.rs_h2 + (yy >> 1)) * p.rs_w2 + (xx >> 1)) * p.ncols + col0 + 64 * g + c8;
          }
          if (rok) rv[i] = *reinterpret_cast<const uint4*>(p.res + roff);
        }
        if constexpr (RED) {
          xq[i] = ok ? *reinterpret_cast<const uint4*>(p.rx + off) : make_uint4(0, 0, 0, 0);
          if constexpr (red2) xq2[i] = ok ? *reinterpret_cast<const uint4*>(p.rx2 + off) : make_uint4(0, 0, 0, 0);
          mbv[i] = (ok && p.rbits) ? p.rbits[off >> 3] : 0u;
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) st[crow(r, lh) * kSS + 32 * q + lr] = from_f<T>(acc[2 * g + q][r]).x;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      float rs[8], rq[8], rq2[8], mu[8], mu2[8], rsc[8], rsh[8];
      if constexpr (RED) {
#pragma unroll
        for (int j = 0; j < 8; ++j) rs[j] = rq[j] = rq2[j] = 0.f;
        const int cc = col0 + 64 * g + (lane & 7) * 8;
        Vec8<float>::load(mu, p.rmean + cc);
        if constexpr (red2) Vec8<float>::load(mu2, p.rmean2 + cc);
        if (!p.rbits) {  // wave-uniform: the mask of a plain BN + ReLU, recomputed from its input
          Vec8<float>::load(rsc, p.rcoef + cc);
          Vec8<float>::load(rsh, p.rcoef + p.ncols + cc);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qid = lane + 64 * i, rr = qid >> 3, c8 = (qid & 7) * 8;
        uint4 v = *reinterpret_cast<const uint4*>(st + rr * kSS + c8);
        const int64_t off = (row0 + rr) * p.ncols + col0 + 64 * g + c8;
        if (row0 + rr < p.m) {
          if (RED || has_res) {  // wave-uniform branch
            float a[8];
            Vec8<T>::load(a, reinterpret_cast<const T*>(&v));
            if (has_res) {
              float b[8];
              Vec8<T>::load(b, reinterpret_cast<const T*>(&rv[i]));
#pragma unroll
              for (int j = 0; j < 8; ++j) a[j] += b[j];
            }
            if constexpr (RED) {
              float xv[8];
              Vec8<T>::load(xv, reinterpret_cast<const T*>(&xq[i]));
              unsigned mb = mbv[i];
              if (!p.rbits) {
                mb = 0u;
#pragma unroll
                for (int j = 0; j < 8; ++j) mb |= (fmaf(xv[j], rsc[j], rsh[j]) > 0.f ? 1u : 0u) << j;
              }
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                // the stored (rounded) gradient is what the rest of the backward sees
                const float gq = ((mb >> j) & 1u) ? to_f(from_f<T>(a[j])) : 0.f;
                a[j] = gq;
                rs[j] += gq;
                rq[j] = fmaf(gq, xv[j] - mu[j], rq[j]);
              }
              if constexpr (red2) {
                float xv2[8];
                Vec8<T>::load(xv2, reinterpret_cast<const T*>(&xq2[i]));
#pragma unroll
                for (int j = 0; j < 8; ++j) rq2[j] = fmaf(a[j], xv2[j] - mu2[j], rq2[j]);
              }
            }
            Vec8<T>::store(reinterpret_cast<T*>(&v), a);
          }
          *reinterpret_cast<uint4*>(p.y + off) = v;
        }
      }
      if constexpr (RED) {
        // lanes l, l ^ 8, ..., l ^ 56 hold the same 8 columns: a reduce-scatter over lane bits
        // 5, 4, 3 (4 + 2 + 1 exchanges per sum instead of 3 x 8) leaves lane l the total of
        // column 4 b5 + 2 b4 + b3 of its 8; the 64 lanes then own 64 distinct columns and add
        // them into this wave's LDS accumulators (wave-private: no atomics)
#pragma unroll
        for (int st = 0; st < 3; ++st) {
          const int msk = 32 >> st, half = 4 >> st;
          const bool up = (lane & msk) != 0;
#pragma unroll
          for (int j = 0; j < half; ++j) {
            const float ss = up ? rs[j] : rs[j + half];
            const float sq = up ? rq[j] : rq[j + half];
            const float gs = __shfl_xor(ss, msk, 64);
            const float gq = __shfl_xor(sq, msk, 64);
            rs[j] = (up ? rs[j + half] : rs[j]) + gs;
            rq[j] = (up ? rq[j + half] : rq[j]) + gq;
            if constexpr (red2) {
              const float sq2 = up ? rq2[j] : rq2[j + half];
              const float gq2 = __shfl_xor(sq2, msk, 64);
              rq2[j] = (up ? rq2[j + half] : rq2[j]) + gq2;
            }
          }
        }
        const int jc = ((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1);
        float* r0p = rsum + (wid * 3) * NC + 64 * g + (lane & 7) * 8 + jc;
        r0p[0] += rs[0];
        r0p[NC] += rq[0];
        if constexpr (red2) r0p[2 * NC] += rq2[0];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int cb = 0; cb < CN; ++cb) acc[cb] = zero16();
  };

  // flat (tile, chunk) stream with DEPTH - 1 chunks' loads in flight under the current chunk's
  // math: a ring of DEPTH register sets (2: the next chunk only; 3: two ahead — one chunk's math
  // is shorter than the HBM latency under full load, so a single chunk in flight leaves every
  // wave waiting at the top of each chunk).  The prefetch is unconditional (past the end: the last
  // tile again, discarded): a branch around the loads makes the compiler's vmcnt waits
  // conservative.
  const int tlast = p.ntiles - 1;
  auto adv = [&](int& tt, int& cc) {
    if (++cc == NCH) {
      cc = 0;
      tt += gridDim.x;
    }
  };
  int t = blockIdx.x, ch = 0;
  if constexpr (DEPTH == 2) {
    Frags fa, fb;
    load(fa, min(t, tlast), 0);
    while (t < p.ntiles) {
      {
        int nt = t, nch = ch;
        adv(nt, nch);
        load(fb, min(nt, tlast), nch);
        compute(fa, t, ch);
        if (ch == NCH - 1) epilogue(t);
        t = nt;
        ch = nch;
      }
      if (t >= p.ntiles) break;
      {
        int nt = t, nch = ch;
        adv(nt, nch);
        load(fa, min(nt, tlast), nch);
        compute(fb, t, ch);
        if (ch == NCH - 1) epilogue(t);
        t = nt;
        ch = nch;
      }
    }
  } else if constexpr (DEPTH >= 4) {
    // deeper ring for the one-workgroup-per-CU shapes (a 4-wave CU needs more bytes in flight
    // per wave).  Named register sets rotated by an explicit unrolled body: an array of them
    // indexed by the rotation (even with constant indices after the unroll) was left in scratch
    // at DEPTH 4 (592 B per lane, profiles/r06/scratch_census_r06s.md)
    static_assert(DEPTH <= 5, "ring depth");
    Frags f0, f1, f2, f3, f4;  // f4: DEPTH 5 only
    int tn = t, cn = ch;
    auto pre = [&](Frags& f) {
      load(f, min(tn, tlast), cn);
      adv(tn, cn);
    };
    pre(f0);
    pre(f1);
    pre(f2);
    if constexpr (DEPTH == 5) pre(f3);
    bool done = false;
    auto step = [&](Frags& nxt, const Frags& cur) {
      if (done) return;
      pre(nxt);
      compute(cur, t, ch);
      if (ch == NCH - 1) epilogue(t);
      adv(t, ch);
      done = t >= p.ntiles;
    };
    while (!done) {
      if constexpr (DEPTH == 4) {
        step(f3, f0);
        step(f0, f1);
        step(f1, f2);
        step(f2, f3);
      } else {
        step(f4, f0);
        step(f0, f1);
        step(f1, f2);
        step(f2, f3);
        step(f3, f4);
      }
    }
  } else {
    Frags f0, f1, f2;
    int t1 = t, c1 = ch;
    adv(t1, c1);
    int t2 = t1, c2 = c1;
    adv(t2, c2);
    load(f0, min(t, tlast), ch);
    load(f1, min(t1, tlast), c1);
    // one ring step: prefetch position 2 into `nxt`, run position 0 from `cur`, shift positions
    auto step = [&](Frags& nxt, const Frags& cur) {
      load(nxt, min(t2, tlast), c2);
      compute(cur, t, ch);
      if (ch == NCH - 1) epilogue(t);
      t = t1;
      ch = c1;
      t1 = t2;
      c1 = c2;
      adv(t2, c2);
    };
    while (t < p.ntiles) {
      step(f2, f0);
      if (t >= p.ntiles) break;
      step(f0, f1);
      if (t >= p.ntiles) break;
      step(f1, f2);
    }
  }

  if constexpr (RED) {
    __syncthreads();
    // rows 0, 1 (and with the second BN: 2 = a copy of row 0, 3 = its g (x2 - mean2) sums)
    const int nrows = p.rx2 ? 4 : 2;
    for (int i = tid; i < nrows * NC; i += NT) {
      const int which = i / NC, n = i % NC;
      const int src = which == 2 ? 0 : which == 3 ? 2 : which;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) v += rsum[(w * 3 + src) * NC + n];
      p.part[((int64_t)which * gridDim.x + blockIdx.x) * p.ncols + col0 + n] = v;
    }
  }
  if constexpr (STATS) {
    float* red = reinterpret_cast<float*>(stg);  // [kWaves][2][NC] (8 KB at NC = 256 <= staging slab)
#pragma unroll
    for (int cb = 0; cb < CN; ++cb) {
      s1[cb] += __shfl_xor(s1[cb], 32, 64);
      s2[cb] += __shfl_xor(s2[cb], 32, 64);
    }
    __syncthreads();
    if (lh == 0) {
#pragma unroll
      for (int cb = 0; cb < CN; ++cb) {
        red[(wid * 2 + 0) * NC + 32 * cb + lr] = s1[cb];
        red[(wid * 2 + 1) * NC + 32 * cb + lr] = s2[cb];
      }
    }
    __syncthreads();
    for (int i = tid; i < 2 * NC; i += NT) {
      const int which = i / NC, n = i % NC;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) v += red[(w * 2 + which) * NC + n];
      p.part[((int64_t)which * gridDim.x + blockIdx.x) * p.ncols + col0 + n] = v;
    }
  }
}

// finalize kernels: 8 channels x kFinG row groups per block (the partial rows of a 3x3 conv's
// 256-row tiles number ~3k at ResNet stage 1: 128 groups keep ~25 independent loads per thread)
constexpr int kFinG = 128;

// ---- statistics finalize: fixed-order sum of the per-workgroup partials -> batch mean /
// inv_std, the running-stat EMA and the apply coefficients coef = [scale | shift] ----
// ``shift`` (the statistics' centring shift) is usually the running mean itself, so shift, rmean
// and rvar are NOT restrict: shift[ch] is read into a register before rmean[ch] is written.
__global__ void __launch_bounds__(8 * kFinG) stats_finalize(const float* __restrict__ part, int g, int c, float n,
                                                      const float* shift, const float* __restrict__ w,
                                                      const float* __restrict__ b, float eps, float momentum,
                                                      float* rmean, float* rvar,
                                                      float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                                      float* __restrict__ coef) {
  // 8 channels x 32 partial-row groups per block (the finalize is latency-bound)
  __shared__ float red[2][kFinG][9];
  const int lc = threadIdx.x & 7, grp = threadIdx.x >> 3, ch = blockIdx.x * 8 + lc;
  float a = 0.f, q = 0.f;
  if (ch < c)
    for (int j = grp; j < g; j += kFinG) {
      a += part[(int64_t)j * c + ch];
      q += part[(int64_t)(g + j) * c + ch];
    }
  red[0][grp][lc] = a;
  red[1][grp][lc] = q;
  __syncthreads();
  if (grp != 0 || ch >= c) return;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll 8
  for (int i = 0; i < kFinG; ++i) {
    s1 += red[0][i][lc];
    s2 += red[1][i][lc];
  }
  const float sft = shift ? shift[ch] : 0.f;
  const float dm = s1 / n;
  const float var_b = fmaxf(s2 / n - dm * dm, 0.f);
  const float mm = sft + dm;
  const float istd = rsqrtf(var_b + eps);
  save_mean[ch] = mm;
  save_invstd[ch] = istd;
  const float sc = istd * (w ? w[ch] : 1.f);
  coef[ch] = sc;
  coef[c + ch] = (b ? b[ch] : 0.f) - mm * sc;
  if (rmean) rmean[ch] = (1.f - momentum) * rmean[ch] + momentum * mm;
  if (rvar) rvar[ch] = (1.f - momentum) * rvar[ch] + momentum * (n > 1.f ? var_b * n / (n - 1.f) : var_b);
}

// backward reduction finalize (the RED partials): grad_w, grad_b and the dx coefficients
// coef_bwd = [A | B | K] with dx = A * g + B * x + K (the BN backward of a training-mode norm)
// ---- group (cross-rank) statistics from the epilogue partials: the Welford payload
// [mean(C) | M2(C) | count] of this rank, M2 = sum of squared deviations from the local mean,
// for the group exchange + merge of csrc/groupbn (bn_nhwc_stats_merge) ----
__global__ void __launch_bounds__(8 * kFinG) part_payload(const float* __restrict__ part, int g, int c, float n,
                                                    const float* shift, float* __restrict__ payload) {
  __shared__ float red[2][kFinG][9];
  const int lc = threadIdx.x & 7, grp = threadIdx.x >> 3, ch = blockIdx.x * 8 + lc;
  float a = 0.f, q = 0.f;
  if (ch < c)
    for (int j = grp; j < g; j += kFinG) {
      a += part[(int64_t)j * c + ch];
      q += part[(int64_t)(g + j) * c + ch];
    }
  red[0][grp][lc] = a;
  red[1][grp][lc] = q;
  __syncthreads();
  if (grp != 0 || ch >= c) return;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll 8
  for (int i = 0; i < kFinG; ++i) {
    s1 += red[0][i][lc];
    s2 += red[1][i][lc];
  }
  const float dm = s1 / n;
  payload[ch] = (shift ? shift[ch] : 0.f) + dm;
  payload[c + ch] = fmaxf(s2 - s1 * dm, 0.f);
  if (ch == 0) payload[2 * c] = n;
}

__global__ void __launch_bounds__(8 * kFinG) bwd_finalize(const float* __restrict__ part, int g, int c, float inv_n,
                                                    const float* __restrict__ mean, const float* __restrict__ istd,
                                                    const float* __restrict__ w, float* __restrict__ gw,
                                                    float* __restrict__ gb, float* __restrict__ coef) {
  __shared__ float red[2][kFinG][9];
  const int lc = threadIdx.x & 7, grp = threadIdx.x >> 3, ch = blockIdx.x * 8 + lc;
  float a = 0.f, q = 0.f;
  if (ch < c)
    for (int j = grp; j < g; j += kFinG) {
      a += part[(int64_t)j * c + ch];
      q += part[(int64_t)(g + j) * c + ch];
    }
  red[0][grp][lc] = a;
  red[1][grp][lc] = q;
  __syncthreads();
  if (grp != 0 || ch >= c) return;
  float sdy = 0.f, sdyx = 0.f;
#pragma unroll 8
  for (int i = 0; i < kFinG; ++i) {
    sdy += red[0][i][lc];
    sdyx += red[1][i][lc];
  }
  const float is = istd[ch];
  if (gw) gw[ch] = sdyx * is;
  if (gb) gb[ch] = sdy;
  const float A = is * (w ? w[ch] : 1.f);
  const float B = -A * is * is * (sdyx * inv_n);
  coef[ch] = A;
  coef[c + ch] = B;
  coef[2 * c + ch] = -A * (sdy * inv_n) - B * mean[ch];
}

// prefetch ring depth (APEX_AMD_C1BN_DEPTH=2..5 overrides, for A/B): 3 where the third register
// set fits beside the accumulators without spills (<= 128 columns but 128 x 128), else 2; the
// shapes whose weight image leaves ONE 4-wave workgroup per CU (128 columns x k 512) take a
// deeper ring (APEX_AMD_C1BN_DEPTH1, default 4): 4 waves carry the CU's whole HBM stream
static int g_c1bn_depth = [] {
  const char* e = std::getenv("APEX_AMD_C1BN_DEPTH");
  return e ? std::atoi(e) : 0;
}();
static int g_c1bn_depth1 = [] {
  const char* e = std::getenv("APEX_AMD_C1BN_DEPTH1");
  return e ? std::atoi(e) : 4;
}();
constexpr int default_depth(int nc, int kr) { return nc <= 128 && !(nc == 128 && kr == 128) ? 3 : 2; }


template <typename T, int NC, int KR, bool WT, int PRO, bool STATS, bool RED, int DEPTH, bool RED2 = false>
void launch_d(const Args& a0, int cus, hipStream_t s) {
  constexpr int NW = pick_nw(NC, KR, PRO, RED);
  constexpr int lds = lds_bytes_nw(NC, KR, PRO, RED, NW);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&fused1x1<T, NC, KR, WT, PRO, STATS, RED, NW, DEPTH, RED2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  Args a = a0;
  a.ntiles = (int)((a.m + NW * 32 - 1) / (NW * 32));
  const int per_cu = (160 * 1024) / lds >= 2 ? 2 : 1;
  // one resident round over the whole grid (column groups included): every workgroup loads the
  // weight image once and then streams ~ntiles / gx tiles
  const int gy = a.ncols / NC;
  int gx = (cus * per_cu + gy - 1) / gy;
  if (gx > a.ntiles) gx = a.ntiles;
  hipLaunchKernelGGL((fused1x1<T, NC, KR, WT, PRO, STATS, RED, NW, DEPTH, RED2>), dim3(gx, a.ncols / NC), dim3(NW * 64),
                     lds, s, a);
}

template <typename T, int NC, int KR, bool WT, int PRO, bool STATS, bool RED = false, bool RED2 = false>
void launch_t(const Args& a, int cus, hipStream_t s) {
  if constexpr (one_wg_per_cu(NC, KR, PRO, RED)) {
    int d = g_c1bn_depth >= 2 && g_c1bn_depth <= 5 ? g_c1bn_depth : g_c1bn_depth1;
    // the BN-backward prologue + reduction form at depth 5 (its round-5 depth-4 ring sat in scratch;
    // the named ring of round 6 removed that for every form, and depth 4 stays the measured best for
    // the others: profiles/r06/ab_c1bn_depth_r06ae.txt)
    if ((PRO == kProBnBwd || PRO == kProBnBwdMask) && RED && d == 4) d = 5;
    if (d == 5) return launch_d<T, NC, KR, WT, PRO, STATS, RED, 5, RED2>(a, cus, s);
    if (d == 4) return launch_d<T, NC, KR, WT, PRO, STATS, RED, 4, RED2>(a, cus, s);
    if (d == 2) return launch_d<T, NC, KR, WT, PRO, STATS, RED, 2, RED2>(a, cus, s);
    return launch_d<T, NC, KR, WT, PRO, STATS, RED, 3, RED2>(a, cus, s);
  }
  const int d = g_c1bn_depth == 2 || g_c1bn_depth == 3 ? g_c1bn_depth : default_depth(NC, KR);
  if (d == 3) launch_d<T, NC, KR, WT, PRO, STATS, RED, 3, RED2>(a, cus, s);
  else launch_d<T, NC, KR, WT, PRO, STATS, RED, 2, RED2>(a, cus, s);
}

inline int grid_x(int64_t m, int nc, int kr, int pro, int cus, int ncols, bool red = false) {
  const int nw = pick_nw(nc, kr, pro, red);
  const int lds = lds_bytes_nw(nc, kr, pro, red, nw);
  const int per_cu = (160 * 1024) / lds >= 2 ? 2 : 1;
  const int ntiles = (int)((m + nw * 32 - 1) / (nw * 32));
  const int gy = ncols / nc;
  const int gx = (cus * per_cu + gy - 1) / gy;
  return gx < ntiles ? gx : ntiles;
}

// column tile: the widest of 256 / 128 / 64 that divides ncols (256 needs the 128 accumulator
// registers of 8 blocks; the register file holds it at 2 waves / SIMD; at k = 512 its weight
// image would not fit the LDS)
// The deepest reduction that still takes the 256- / 128-column tile (APEX_AMD_C1BN_NC256_MAXK,
// APEX_AMD_C1BN_NC128_MAXK: A/B knobs).  At k = 256 the 256-column weight image (135 KB) leaves
// one 4-wave workgroup per CU, which streams at about half the rate of 8 waves: 128 columns there
// re-read the operand from L2 twice as often but run 2 workgroups per CU — +1.6 % on the whole
// ResNet-50 step (12,109-12,168 -> 12,323-12,336 img/s same box, profiles/r05/ab_c1bn_nc_r05o.txt).
inline int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
// 256-column tiles only on request (APEX_AMD_C1BN_NC256_MAXK / _RED_MAXK = <max k>): beside the
// backward-reduction epilogue their 128 accumulator registers spilled (80-120 B / lane) and
// 128-column tiles measured +0.8 % on the step (profiles/r06/ab_c1bn_nc256_r06u.txt); keeping 256
// for the other forms at k <= 64 measured -0.4 % (profiles/r06/ab_tap_prefetch_nc256_r06ab.txt)
inline int col_tile(int ncols, int kr, bool red) {
  static const int max256 = env_int("APEX_AMD_C1BN_NC256_MAXK", 0);
  static const int max256_red = env_int("APEX_AMD_C1BN_NC256_RED_MAXK", 0);
  static const int max128 = env_int("APEX_AMD_C1BN_NC128_MAXK", 512);
  if (ncols % 256 == 0 && kr <= 256 && kr <= (red ? max256_red : max256)) return 256;
  return ncols % 128 == 0 && kr <= max128 ? 128 : 64;
}

// the column tile, narrowed while the workgroup's LDS (weight image + staging + prologue rows +
// reduction sums) would not fit: the recomputed-mask BN-backward prologue's 5 rows at k 512
inline int col_tile_fit(int ncols, int kr, int pro, bool red) {
  int nc = col_tile(ncols, kr, red);
  while (nc > 64 && lds_bytes_nw(nc, kr, pro, red, pick_nw(nc, kr, pro, red)) > 160 * 1024) nc /= 2;
  if (lds_bytes_nw(nc, kr, pro, red, pick_nw(nc, kr, pro, red)) > 160 * 1024)
    throw std::runtime_error("conv1x1_bn: no column tile fits the LDS for this reduction depth / prologue");
  return nc;
}

template <typename T, bool WT, int PRO, bool STATS, bool RED = false, bool RED2 = false>
void dispatch_shape(const Args& a, int nc, int kr, int cus, hipStream_t s) {
#define C1BN_CASE(NC_, KR_)                                 \
  if (nc == NC_ && kr == KR_) {                             \
    launch_t<T, NC_, KR_, WT, PRO, STATS, RED, RED2>(a, cus, s);  \
    return;                                                 \
  }
  C1BN_CASE(64, 64) C1BN_CASE(64, 128) C1BN_CASE(64, 256) C1BN_CASE(64, 512)
  C1BN_CASE(128, 64) C1BN_CASE(128, 128) C1BN_CASE(128, 256) C1BN_CASE(128, 512)
  C1BN_CASE(256, 64) C1BN_CASE(256, 128) C1BN_CASE(256, 256)
#undef C1BN_CASE
  throw std::runtime_error("conv1x1_bn: unsupported (columns, reduction) tile");
}

}  // namespace c1bn

bool conv1x1_bn_supported(int64_t m, int k, int ncols) {
  if (m <= 0 || ncols % 64 != 0 || ncols <= 0) return false;
  if (!(k == 64 || k == 128 || k == 256 || k == 512)) return false;
  return true;
}

namespace c1bn {
// res_h, res_w > 0: the residual is the stride-2 subsample gradient of an [N][res_h][res_w] output
inline void set_res_geometry(Args& a, int64_t m, int res_h, int res_w) {
  if (res_h <= 0 || res_w <= 0) return;
  if (m % ((int64_t)res_h * res_w) != 0 || m >= (1ll << 31))
    throw std::runtime_error("conv1x1_bn: subsampled residual needs M = N * res_h * res_w < 2^31");
  a.rs_hw = make_fastdiv((uint32_t)(res_h * res_w));
  a.rs_w = make_fastdiv((uint32_t)res_w);
  a.rs_h2 = (res_h + 1) / 2;
  a.rs_w2 = (res_w + 1) / 2;
}
}  // namespace c1bn

int conv1x1_bn_partials(int64_t m, int k, int ncols, bool pro, int cus, bool pro_addrelu) {
  const int pk = pro_addrelu ? c1bn::kProBnAddRelu : pro ? c1bn::kProBnRelu : c1bn::kProNone;
  return c1bn::grid_x(m, c1bn::col_tile_fit(ncols, k, pk, false), k, pk, cus, ncols);
}

void conv1x1_bn(const void* a, const void* w, void* y, int64_t m, int k, int ncols, bool w_kmajor_out, int dtype,
                const float* pcoef, const float* shift, float* part, int cus, hipStream_t s, const void* res,
                const void* py, void* aout, bool pro_relu, uint8_t* bout, int res_h, int res_w, bool pc_split,
                const float* pc_res, bool pro_mask) {
  if (!conv1x1_bn_supported(m, k, ncols)) throw std::runtime_error("conv1x1_bn: unsupported shape");
  c1bn::Args args{};
  args.pc_split = pc_split ? 1 : 0;
  args.pc_res = pc_res;
  if (pc_split && !(py && pro_relu)) throw std::runtime_error("conv1x1_bn: split coefficients are an add + ReLU option");
  c1bn::set_res_geometry(args, m, res_h, res_w);
  args.a = static_cast<const uint16_t*>(a);
  args.w = static_cast<const uint16_t*>(w);
  args.y = static_cast<uint16_t*>(y);
  args.m = m;
  args.ncols = ncols;
  args.ntiles = 0;  // set per wave count by launch_t
  args.pcoef = pcoef;
  args.shift = shift;
  args.part = part;
  args.res = static_cast<const uint16_t*>(res);
  args.py = static_cast<const uint16_t*>(py);
  args.aout = static_cast<uint16_t*>(aout);
  args.bout = bout;
  const bool wt = w_kmajor_out;
  const bool stats = part != nullptr;
  // py given: the two-operand prologue (pcoef = [3][k]) — BN backward, or with pro_relu the block
  // below's output BN + residual + ReLU; else pcoef = the BN apply + ReLU [2][k]
  const int pro = pcoef == nullptr ? c1bn::kProNone
                  : py            ? (pro_relu ? c1bn::kProBnAddRelu : pro_mask ? c1bn::kProBnBwdMask : c1bn::kProBnBwd)
                                  : c1bn::kProBnRelu;
  if (pro_mask && pro != c1bn::kProBnBwdMask) throw std::runtime_error("conv1x1_bn: pro_mask needs py and pcoef");
  const int nc = c1bn::col_tile_fit(ncols, k, pro, false);
  if (aout && !c1bn::pro_two(pro)) throw std::runtime_error("conv1x1_bn: aout needs a two-operand prologue");
  if (bout && pro != c1bn::kProBnAddRelu) throw std::runtime_error("conv1x1_bn: bout needs the add + ReLU prologue");
  auto go = [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (wt) {
      if (stats || pro == c1bn::kProBnRelu)
        throw std::runtime_error("conv1x1_bn: the transposed-weight (dgrad) form takes the BN-backward prologue only");
      if (pro == c1bn::kProBnAddRelu) throw std::runtime_error("conv1x1_bn: the add + ReLU prologue is a forward option");
      if (pro == c1bn::kProBnBwd) c1bn::dispatch_shape<T, true, c1bn::kProBnBwd, false>(args, nc, k, cus, s);
      else if (pro == c1bn::kProBnBwdMask) c1bn::dispatch_shape<T, true, c1bn::kProBnBwdMask, false>(args, nc, k, cus, s);
      else c1bn::dispatch_shape<T, true, c1bn::kProNone, false>(args, nc, k, cus, s);
    } else {
      if (pro == c1bn::kProBnBwd || pro == c1bn::kProBnBwdMask)
        throw std::runtime_error("conv1x1_bn: BN-backward prologue is a dgrad-form option");
      if (pro == c1bn::kProBnAddRelu) {
        if (stats) c1bn::dispatch_shape<T, false, c1bn::kProBnAddRelu, true>(args, nc, k, cus, s);
        else c1bn::dispatch_shape<T, false, c1bn::kProBnAddRelu, false>(args, nc, k, cus, s);
        return;
      }
      if (pro == c1bn::kProBnRelu) {
        if (stats) c1bn::dispatch_shape<T, false, c1bn::kProBnRelu, true>(args, nc, k, cus, s);
        else c1bn::dispatch_shape<T, false, c1bn::kProBnRelu, false>(args, nc, k, cus, s);
      } else {
        if (stats) c1bn::dispatch_shape<T, false, c1bn::kProNone, true>(args, nc, k, cus, s);
        else c1bn::dispatch_shape<T, false, c1bn::kProNone, false>(args, nc, k, cus, s);
      }
    }
  };
  dispatch_16(dtype, go, "conv1x1_bn");
  check_launch("conv1x1_bn");
}

int conv1x1_dgrad_bnred_partials(int64_t m, int k, int ncols, int cus, bool pro, bool pro_mask) {
  const int pk = pro ? (pro_mask ? c1bn::kProBnBwdMask : c1bn::kProBnBwd) : c1bn::kProNone;
  return c1bn::grid_x(m, c1bn::col_tile_fit(ncols, k, pk, true), k, pk, cus, ncols, true);
}

void conv1x1_dgrad_bnred(const void* g, const void* w, void* out, int64_t m, int k, int ncols, int dtype,
                         const void* res, const uint8_t* bits, const void* x, const float* mean, float* part, int cus,
                         hipStream_t s, const float* rcoef, const void* py, const float* pcoef, void* aout, int res_h,
                         int res_w, bool pro_mask, const void* x2, const float* mean2) {
  if (!conv1x1_bn_supported(m, k, ncols)) throw std::runtime_error("conv1x1_dgrad_bnred: unsupported shape");
  if ((!bits && !rcoef) || !x || !mean || !part)
    throw std::runtime_error("conv1x1_dgrad_bnred: a mask source (bits or coef), x, mean and part are required");
  if ((py == nullptr) != (pcoef == nullptr)) throw std::runtime_error("conv1x1_dgrad_bnred: prologue needs py and pcoef");
  c1bn::Args args{};
  args.a = static_cast<const uint16_t*>(g);
  args.w = static_cast<const uint16_t*>(w);
  args.y = static_cast<uint16_t*>(out);
  args.m = m;
  args.ncols = ncols;
  args.part = part;
  args.res = static_cast<const uint16_t*>(res);
  c1bn::set_res_geometry(args, m, res_h, res_w);
  args.rbits = bits;
  args.rcoef = rcoef;
  args.rx = static_cast<const uint16_t*>(x);
  args.rmean = mean;
  if ((x2 == nullptr) != (mean2 == nullptr)) throw std::runtime_error("conv1x1_dgrad_bnred: x2 and mean2 go together");
  args.rx2 = static_cast<const uint16_t*>(x2);
  args.rmean2 = mean2;
  args.pcoef = pcoef;
  args.py = static_cast<const uint16_t*>(py);
  args.aout = static_cast<uint16_t*>(aout);
  const int nc = c1bn::col_tile_fit(ncols, k, py ? (pro_mask ? c1bn::kProBnBwdMask : c1bn::kProBnBwd) : c1bn::kProNone,
                                    true);
  dispatch_16(dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (py && pro_mask && x2) c1bn::dispatch_shape<T, true, c1bn::kProBnBwdMask, false, true, true>(args, nc, k, cus, s);
    else if (py && pro_mask) c1bn::dispatch_shape<T, true, c1bn::kProBnBwdMask, false, true>(args, nc, k, cus, s);
    else if (py && x2) c1bn::dispatch_shape<T, true, c1bn::kProBnBwd, false, true, true>(args, nc, k, cus, s);
    else if (py) c1bn::dispatch_shape<T, true, c1bn::kProBnBwd, false, true>(args, nc, k, cus, s);
    else if (x2) c1bn::dispatch_shape<T, true, c1bn::kProNone, false, true, true>(args, nc, k, cus, s);
    else c1bn::dispatch_shape<T, true, c1bn::kProNone, false, true>(args, nc, k, cus, s);
  }, "conv1x1_dgrad_bnred");
  check_launch("conv1x1_dgrad_bnred");
}

void conv1x1_bn_finalize(const float* part, int g, int c, float n, const float* shift, const float* w, const float* b,
                         float eps, float momentum, float* rmean, float* rvar, float* save_mean, float* save_invstd,
                         float* coef, hipStream_t s) {
  hipLaunchKernelGGL(c1bn::stats_finalize, dim3((c + 7) / 8), dim3(8 * c1bn::kFinG), 0, s, part, g, c, n, shift, w, b, eps,
                     momentum, rmean, rvar, save_mean, save_invstd, coef);
  check_launch("conv1x1_bn_finalize");
}

// =============================================================================================
// Weight gradient of a 1x1 convolution with the producing batch norm (+ReLU) applied to the
// activation on load: dW[n][k] = sum_m G[m][n] . pro(X[m][k]), G = dY [M][N], X [M][K].
// Split over M (the pixels): each workgroup owns a [NT][KT] block of dW for a contiguous row
// range, streams 64-row chunks of G and X global -> registers (pro applied once per element
// here) -> LDS (row-major images, rows padded so the 4 rows a 16-lane transposed read touches
// start 64 B apart in the bank space), and feeds the MFMAs with ds_read_b64_tr_b16 fragments
// (both operands are m-major).  The next chunk's loads are in flight under the current chunk's
// MFMAs; one barrier per chunk.  fp32 partials [S][N][K] are summed in a fixed order by
// wgrad_reduce (deterministic, no atomics).
// =============================================================================================
namespace c1w {
using namespace mfma;

struct Args {
  const uint16_t* g;   // [M][N]
  const uint16_t* x;   // [M][K]
  float* ws;           // [S][N][K]
  int64_t m;
  int n, k;
  int64_t rows;        // rows per split (multiple of 64)
  const float* xcoef;  // PRO: [2][K] scale | shift, pro(x) = relu(x * scale + shift)
  // GATHER (3x3, pad 1): x is the [N][H][W][C] input, K = 9 C with column (tap t, channel c) at
  // t * C + c, and row m = (n, oh, ow) of G reads input pixel (oh * st + t / 3 - 1, ow * st + t % 3 - 1)
  // (zero outside the image); xcoef is then per channel [2][C]
  int h, w, c, oh, ow, st;
};

constexpr int MB = 64;

template <int NT, int KT>
constexpr int lds_bytes() {
  return 2 * MB * ((NT + 32) + (KT + 32)) * 2;
}

template <typename T, int NT, int KT, bool PRO, bool GATHER = false>
__global__ void __launch_bounds__(256, 1) wgrad1x1(Args p) {
  constexpr int GS = NT + 32, XS = KT + 32;   // LDS row strides (elements)
  constexpr int GL = MB * NT / 8 / 256;       // 16-byte loads per thread per chunk
  constexpr int XL = MB * KT / 8 / 256;
  constexpr int WN = NT / 64, WK = KT / 64;   // 32x32 blocks per wave (2 x 2 waves)
  static_assert(GL >= 1 && XL >= 1 && WN * WK <= 8, "wgrad tile");
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, lr = lane & 31, lh = lane >> 5;
  const int wn = wid & 1, wk = wid >> 1;
  const int n0 = blockIdx.y * NT, k0 = blockIdx.z * KT;
  const int64_t r0 = (int64_t)blockIdx.x * p.rows;
  const int64_t r1 = r0 + p.rows < p.m ? r0 + p.rows : p.m;

  // this thread's X columns are the same for every load (256 is a multiple of KT / 8)
  const int xc8 = (tid % (KT / 8)) * 8;
  float xs[8], xb[8];
  if constexpr (PRO && !GATHER) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xs[j] = p.xcoef[k0 + xc8 + j];
      xb[j] = p.xcoef[p.k + k0 + xc8 + j];
    }
  }
  unsigned xvalid = 0;  // GATHER: bit i = load i read a real pixel (padding stays exactly 0)

  uint4 gr[GL], xr[XL];
  auto gload = [&](int64_t base) {
#pragma unroll
    for (int i = 0; i < GL; ++i) {
      const int idx = tid + 256 * i, row = idx / (NT / 8), c8 = (idx % (NT / 8)) * 8;
      const int64_t rr = base + row;
      gr[i] = rr < r1 ? *reinterpret_cast<const uint4*>(p.g + rr * p.n + n0 + c8) : make_uint4(0, 0, 0, 0);
    }
    if constexpr (GATHER) xvalid = 0;
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + 256 * i, row = idx / (KT / 8);
      const int64_t rr = base + row;
      if constexpr (GATHER) {
        // 192-wide tiles: 256 is not a multiple of KT / 8, so the column is per load
        const int gcol = k0 + (idx % (KT / 8)) * 8;
        const int gtap = gcol / p.c, gch = gcol - gtap * p.c;
        const int tdh = gtap / 3 - 1, tdw = gtap % 3 - 1;
        bool ok = rr < r1;
        int64_t src = 0;
        if (ok) {
          const int ohw = p.oh * p.ow;
          const int nimg = (int)(rr / ohw), rem = (int)(rr - (int64_t)nimg * ohw);
          const int oy = rem / p.ow, ox = rem - oy * p.ow;
          const int iy = oy * p.st + tdh, ix = ox * p.st + tdw;
          ok = (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
          src = (((int64_t)nimg * p.h + iy) * p.w + ix) * p.c + gch;
        }
        xr[i] = ok ? *reinterpret_cast<const uint4*>(p.x + src) : make_uint4(0, 0, 0, 0);
        xvalid |= (ok ? 1u : 0u) << i;
      } else {
        xr[i] = rr < r1 ? *reinterpret_cast<const uint4*>(p.x + rr * p.k + k0 + xc8) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lwrite = [&](int buf) {
    uint16_t* gi = lds + buf * MB * (GS + XS);
    uint16_t* xi = gi + MB * GS;
#pragma unroll
    for (int i = 0; i < GL; ++i) {
      const int idx = tid + 256 * i, row = idx / (NT / 8), c8 = (idx % (NT / 8)) * 8;
      *reinterpret_cast<uint4*>(gi + row * GS + c8) = gr[i];
    }
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + 256 * i, row = idx / (KT / 8);
      const int lcol = GATHER ? (idx % (KT / 8)) * 8 : xc8;
      uint4 v = xr[i];
      if constexpr (PRO && GATHER) {
        const int gcol = k0 + lcol, gch = gcol % p.c;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xs[j] = p.xcoef[gch + j];
          xb[j] = p.xcoef[p.c + gch + j];
        }
      }
      if constexpr (PRO) {
        uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float lo = fmaxf(fmaf(to_f(T{(uint16_t)(w4[j] & 0xffffu)}), xs[2 * j], xb[2 * j]), 0.f);
          const float hi = fmaxf(fmaf(to_f(T{(uint16_t)(w4[j] >> 16)}), xs[2 * j + 1], xb[2 * j + 1]), 0.f);
          w4[j] = (uint32_t)from_f<T>(lo).x | ((uint32_t)from_f<T>(hi).x << 16);
        }
        v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        if (GATHER && !((xvalid >> i) & 1u)) v = make_uint4(0, 0, 0, 0);
      }
      *reinterpret_cast<uint4*>(xi + row * XS + lcol) = v;
    }
  };

  f32x16 acc[WN][WK];
#pragma unroll
  for (int i = 0; i < WN; ++i)
#pragma unroll
    for (int j = 0; j < WK; ++j) acc[i][j] = zero16();

  auto compute = [&](int buf) {
    const uint16_t* gi = lds + buf * MB * (GS + XS);
    const uint16_t* xi = gi + MB * GS;
#pragma unroll
    for (int kk = 0; kk < MB / 16; ++kk) {
      const int klo = 16 * kk + 8 * lh;
      s16x8 a[WN], b[WK];
#pragma unroll
      for (int i = 0; i < WN; ++i) a[i] = frag_tr<GS>(gi, wn * (NT / 2) + 32 * i, klo, klo + 4, lane);
#pragma unroll
      for (int j = 0; j < WK; ++j) b[j] = frag_tr<XS>(xi, wk * (KT / 2) + 32 * j, klo, klo + 4, lane);
#pragma unroll
      for (int i = 0; i < WN; ++i)
#pragma unroll
        for (int j = 0; j < WK; ++j) acc[i][j] = mma<T>(a[i], b[j], acc[i][j]);
    }
  };

  int buf = 0;
  if (r0 < r1) {
    gload(r0);
    lwrite(0);
  }
  __syncthreads();
  for (int64_t base = r0; base < r1; base += MB) {
    const bool more = base + MB < r1;
    if (more) gload(base + MB);
    compute(buf);
    if (more) lwrite(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  float* out = p.ws + (int64_t)blockIdx.x * p.n * p.k;
#pragma unroll
  for (int i = 0; i < WN; ++i)
#pragma unroll
    for (int j = 0; j < WK; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int nn = n0 + wn * (NT / 2) + 32 * i + crow(r, lh);
        const int kc = k0 + wk * (KT / 2) + 32 * j + lr;
        out[(int64_t)nn * p.k + kc] = acc[i][j][r];
      }
}

// Ring variant: the same tile loop with the operands moved global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, no staging registers) into a 3-slot ring, two chunks (80 KB / CU at
// 256 x 64) in flight under the MFMAs of the current one — the register-staged loop above keeps
// only one chunk in flight and reads HBM at 2-3 TB/s on the 56x56 shapes.  The DMA image is
// lane-linear per 1-KB instruction, so the bank swizzle goes on the source address: logical
// 16-byte chunk c of pixel row r sits at c ^ ((r & 3) << 1), which puts the 4 rows x 2 chunks a
// 16-lane ds_read_b64_tr_b16 touches on 8 distinct bank chunks.  The BN prologue moves to the
// fragment: an X^T fragment is one channel per lane, so its scale / shift are two registers.
constexpr int kRing = 3;

__device__ __forceinline__ void dma16(const uint16_t* src, uint16_t* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// wait until at most N of this wave's DMA instructions are in flight (N = one chunk's worth)
template <int N>
__device__ __forceinline__ void vm_wait_ring() {
  static_assert(N >= 0 && N <= 6 || N == 8 || N == 10 || N == 12, "ring vmcnt");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

template <int COLS, int RMB>
__device__ __forceinline__ void issue_img(const uint16_t* __restrict__ src, int64_t ld, int col0, int64_t base,
                                          int64_t mlast, uint16_t* img, int wave, int lane) {
  constexpr int CPR = COLS / 8;               // 16-byte chunks per row
  constexpr int RPI = 64 / CPR;               // rows per 1-KB instruction
  constexpr int NI = RMB * COLS / 512;        // instructions per image
  static_assert(NI % 4 == 0, "image instructions split over 4 waves");
#pragma unroll
  for (int i = 0; i < NI / 4; ++i) {
    const int j = i * 4 + wave;
    const int row = RPI * j + lane / CPR;
    const int c = (lane % CPR) ^ ((row & 3) << 1);
    int64_t rr = base + row;
    rr = rr <= mlast ? rr : mlast;  // past-the-end rows: valid memory, zeroed in the fragment
    dma16(src + rr * ld + col0 + 8 * c, img + j * 512);
  }
}

template <int STR>
__device__ __forceinline__ s16x8 frag_ring(const uint16_t* img, int colbase, int klo, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int col = colbase + 16 * (g & 1) + 4 * p;
  const int ck = col >> 3, off = col & 7;
  const int r0 = klo + q, r1 = klo + 4 + q;
  const s16x4 lo = tr_read(img + r0 * STR + ((ck ^ ((r0 & 3) << 1)) << 3) + off);
  const s16x4 hi = tr_read(img + r1 * STR + ((ck ^ ((r1 & 3) << 1)) << 3) + off);
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// 32-row chunks: 60 KB of ring at 256 x 64, so two workgroups (8 waves) share a CU and one's
// barrier stalls overlap the other's loads
constexpr int RMB = 32;

template <int NT, int KT>
constexpr int ring_lds_bytes() {
  return kRing * RMB * (NT + KT) * 2;
}

template <typename T, int NT, int KT, bool PRO>
__global__ void __launch_bounds__(256, 2) wgrad1x1_ring(Args p) {
  constexpr int MB = RMB;
  constexpr int WN = NT / 64, WK = KT / 64;
  constexpr int GI = MB * NT / 512 / 4, XI = MB * KT / 512 / 4;  // DMA instructions per wave per chunk
  constexpr int PER = GI + XI;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, lr = lane & 31, lh = lane >> 5;
  const int wn = wid & 1, wk = wid >> 1;
  const int n0 = blockIdx.y * NT, k0 = blockIdx.z * KT;
  const int64_t r0 = (int64_t)blockIdx.x * p.rows;
  const int64_t r1 = r0 + p.rows < p.m ? r0 + p.rows : p.m;
  const int nch = r1 > r0 ? (int)((r1 - r0 + MB - 1) / MB) : 0;
  const int64_t mlast = p.m - 1;

  float xs[WK], xb[WK];
  if constexpr (PRO) {
#pragma unroll
    for (int j = 0; j < WK; ++j) {
      const int kc = k0 + wk * (KT / 2) + 32 * j + lr;
      xs[j] = p.xcoef[kc];
      xb[j] = p.xcoef[p.k + kc];
    }
  }

  auto slot_g = [&](int c) { return lds + (c % kRing) * MB * (NT + KT); };
  auto issue = [&](int c) {
    uint16_t* gi = slot_g(c);
    const int64_t base = r0 + (int64_t)c * MB;
    issue_img<NT, MB>(p.g, p.n, n0, base, mlast, gi, wid, lane);
    issue_img<KT, MB>(p.x, p.k, k0, base, mlast, gi + MB * NT, wid, lane);
  };

  f32x16 acc[WN][WK];
#pragma unroll
  for (int i = 0; i < WN; ++i)
#pragma unroll
    for (int j = 0; j < WK; ++j) acc[i][j] = zero16();

  if (nch > 0) issue(0);
  if (nch > 1) issue(1);
  for (int c = 0; c < nch; ++c) {
    // this wave's part of chunk c has landed (chunk c+1 may still be in flight); its reads of
    // chunk c-1 are complete; the barrier makes both true for every wave
    if (c + 1 < nch) vm_wait_ring<PER>();
    else vm_wait_ring<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + 2 < nch) issue(c + 2);        // into chunk c-1's slot
    const uint16_t* gi = slot_g(c);
    const uint16_t* xi = gi + MB * NT;
    const int64_t base = r0 + (int64_t)c * MB;
    const bool tail = base + MB > r1;
#pragma unroll
    for (int kk = 0; kk < MB / 16; ++kk) {
      const int klo = 16 * kk + 8 * lh;
      s16x8 a[WN], b[WK];
#pragma unroll
      for (int i = 0; i < WN; ++i) {
        a[i] = frag_ring<NT>(gi, wn * (NT / 2) + 32 * i, klo, lane);
        if (tail) {  // rows past this split's end contribute nothing
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (base + klo + (e & 3) + 4 * (e >> 2) >= r1) a[i][e] = 0;
        }
      }
#pragma unroll
      for (int j = 0; j < WK; ++j) {
        b[j] = frag_ring<KT>(xi, wk * (KT / 2) + 32 * j, klo, lane);
        if constexpr (PRO) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = fmaxf(fmaf(to_f(T{(uint16_t)b[j][e]}), xs[j], xb[j]), 0.f);
            b[j][e] = (short)from_f<T>(v).x;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < WN; ++i)
#pragma unroll
        for (int j = 0; j < WK; ++j) acc[i][j] = mma<T>(a[i], b[j], acc[i][j]);
    }
  }

  float* out = p.ws + (int64_t)blockIdx.x * p.n * p.k;
#pragma unroll
  for (int i = 0; i < WN; ++i)
#pragma unroll
    for (int j = 0; j < WK; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int nn = n0 + wn * (NT / 2) + 32 * i + crow(r, lh);
        const int kc = k0 + wk * (KT / 2) + 32 * j + lr;
        out[(int64_t)nn * p.k + kc] = acc[i][j][r];
      }
}

// dW = sum over the S split partials in a fixed order.  A block owns 16 consecutive 8-element
// vectors; its 16 thread groups each sum every 16th split (splits g, g+16, ...), then one fixed-
// order LDS pass adds the 16 group sums — S / 16 loads per thread instead of S, and nk / 128
// blocks (a [256][64] weight: 128 blocks, not 8).
template <typename TO>
__global__ void __launch_bounds__(256) wgrad_reduce(const float* __restrict__ ws, int s, int64_t nk,
                                                    TO* __restrict__ out) {
  __shared__ float red[16][16 * 8 + 4];
  const int v = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t i = ((int64_t)blockIdx.x * 16 + v) * 8;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < nk) {
    for (int q = grp; q < s; q += 16) {
      float t[8];
      Vec8<float>::load(t, ws + (int64_t)q * nk + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += t[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[grp][v * 8 + j] = a[j];
  __syncthreads();
  if (grp != 0 || i >= nk) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.f;
  for (int g2 = 0; g2 < 16; ++g2)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += red[g2][v * 8 + j];
  Vec8<TO>::store(out + i, a);
}

// tile: 256 x 64, 64 x 256, 128 x 128 (16K accumulators / workgroup) or a 256 x 128 / 128 x 256
// block (32K) when the other dimension is read once either way
inline void tile_gather(int n, int k, int& nt, int& kt) {
  // 3x3: K = 9 C; the 192-wide tiles (3 taps at C = 64) keep G re-reads at 3 instead of 9
  static const int cand[][2] = {{256, 128}, {128, 192}, {128, 256}, {128, 128}, {64, 192}, {256, 64},
                                {64, 256}, {128, 64}, {64, 128}, {64, 64}};
  double best = 1e30;
  nt = kt = 64;
  for (const auto& c : cand) {
    if (n % c[0] || k % c[1]) continue;
    const double cost = 1.0 / c[1] + 1.0 / c[0];
    if (cost < best - 1e-12) {
      best = cost;
      nt = c[0];
      kt = c[1];
    }
  }
}

inline void tile(int n, int k, int& nt, int& kt) {
  // every N-tile re-reads X and every K-tile re-reads G, so the operand traffic goes as
  // n k (1 / KT + 1 / NT): take the dividing tile with the smallest 1/KT + 1/NT (ties: the
  // order below), up to 32K accumulators per workgroup
  static const int cand[][2] = {{256, 128}, {128, 256}, {128, 128}, {256, 64}, {64, 256},
                                {128, 64}, {64, 128}, {64, 64}};
  double best = 1e30;
  nt = kt = 64;
  for (const auto& c : cand) {
    if (n % c[0] || k % c[1]) continue;
    const double cost = 1.0 / c[1] + 1.0 / c[0];
    if (cost < best - 1e-12) {
      best = cost;
      nt = c[0];
      kt = c[1];
    }
  }
}

// APEX_AMD_WGRAD_RING=1: the LDS-DMA ring variant (A/B; the register-staged loop measured
// faster on every ResNet-50 shape, profiles/bn1x1_kernels_r03a.jsonl vs the ring run)
inline bool ring_on() {
  static const bool on = [] {
    const char* e = std::getenv("APEX_AMD_WGRAD_RING");
    return e && e[0] == '1';
  }();
  return on;
}

inline int splits(int64_t m, int n, int k, int cus, bool gather = false) {
  int nt, kt;
  if (gather) tile_gather(n, k, nt, kt);
  else tile(n, k, nt, kt);
  const int tiles = (n / nt) * (k / kt);
  // one workgroup per CU (register-staged loop) or two (ring kernel)
  int s = ((ring_on() ? 2 : 1) * cus + tiles - 1) / tiles;
  const int64_t maxs = (m + MB - 1) / MB;
  if (s > maxs) s = (int)maxs;
  return s < 1 ? 1 : s;
}

template <typename T, bool PRO>
void launch(const Args& a, int s, int cus, hipStream_t st) {
  int nt, kt;
  tile(a.n, a.k, nt, kt);
  dim3 grid(s, a.n / nt, a.k / kt);
#define C1W_CASE(NT_, KT_)                                                                                 \
  if (nt == NT_ && kt == KT_) {                                                                            \
    constexpr int lds = lds_bytes<NT_, KT_>();                                                             \
    static bool attr = false;                                                                              \
    if (!attr) {                                                                                           \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad1x1<T, NT_, KT_, PRO>),                      \
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);                                \
      attr = true;                                                                                         \
    }                                                                                                      \
    if (ring_on()) {                                                                                       \
      constexpr int rl = ring_lds_bytes<NT_, KT_>();                                                       \
      static bool rattr = false;                                                                           \
      if (!rattr) {                                                                                        \
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad1x1_ring<T, NT_, KT_, PRO>),         \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, rl);                         \
        rattr = true;                                                                                      \
      }                                                                                                    \
      hipLaunchKernelGGL((wgrad1x1_ring<T, NT_, KT_, PRO>), grid, dim3(256), rl, st, a);                   \
      return;                                                                                              \
    }                                                                                                      \
    hipLaunchKernelGGL((wgrad1x1<T, NT_, KT_, PRO>), grid, dim3(256), lds, st, a);                         \
    return;                                                                                                \
  }
  C1W_CASE(256, 64) C1W_CASE(128, 64) C1W_CASE(64, 256) C1W_CASE(64, 128) C1W_CASE(256, 128)
  C1W_CASE(128, 256) C1W_CASE(128, 128) C1W_CASE(64, 64)
#undef C1W_CASE
  (void)cus;
  throw std::runtime_error("conv1x1 wgrad: no tile");
}

template <typename T, bool PRO>
void launch_gather(const Args& a, int s, hipStream_t st) {
  int nt, kt;
  tile_gather(a.n, a.k, nt, kt);
  dim3 grid(s, a.n / nt, a.k / kt);
#define C3W_CASE(NT_, KT_)                                                                                \
  if (nt == NT_ && kt == KT_) {                                                                           \
    constexpr int lds = lds_bytes<NT_, KT_>();                                                            \
    static bool attr = false;                                                                             \
    if (!attr) {                                                                                          \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad1x1<T, NT_, KT_, PRO, true>),         \
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds);                         \
      attr = true;                                                                                        \
    }                                                                                                     \
    hipLaunchKernelGGL((wgrad1x1<T, NT_, KT_, PRO, true>), grid, dim3(256), lds, st, a);                  \
    return;                                                                                               \
  }
  C3W_CASE(256, 128) C3W_CASE(128, 192) C3W_CASE(128, 256) C3W_CASE(128, 128) C3W_CASE(64, 192)
  C3W_CASE(256, 64) C3W_CASE(64, 256) C3W_CASE(128, 64) C3W_CASE(64, 128) C3W_CASE(64, 64)
#undef C3W_CASE
  throw std::runtime_error("conv3x3 wgrad: no tile");
}

}  // namespace c1w

bool conv3x3_wgrad_supported(int c, int kout) { return c % 64 == 0 && kout % 64 == 0 && c > 0 && kout > 0; }

int64_t conv3x3_wgrad_workspace_floats(int64_t m, int kout, int c, int cus) {
  return (int64_t)c1w::splits(m, kout, 9 * c, cus, true) * kout * 9 * c;
}

void conv3x3_wgrad(const void* g, const void* x, void* dw, int out_dtype, int nimg, int h, int w, int c, int oh,
                   int ow, int stride, int kout, int dtype, const float* xcoef, float* ws, int cus, hipStream_t s) {
  if (!conv3x3_wgrad_supported(c, kout)) throw std::runtime_error("conv3x3 wgrad: C, K must be multiples of 64");
  c1w::Args a{};
  a.g = static_cast<const uint16_t*>(g);
  a.x = static_cast<const uint16_t*>(x);
  a.ws = ws;
  a.m = (int64_t)nimg * oh * ow;
  a.n = kout;
  a.k = 9 * c;
  a.xcoef = xcoef;
  a.h = h;
  a.w = w;
  a.c = c;
  a.oh = oh;
  a.ow = ow;
  a.st = stride;
  const int sp = c1w::splits(a.m, kout, 9 * c, cus, true);
  a.rows = ((a.m + sp - 1) / sp + c1w::MB - 1) / c1w::MB * c1w::MB;
  dispatch_16(dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (xcoef) c1w::launch_gather<T, true>(a, sp, s);
    else c1w::launch_gather<T, false>(a, sp, s);
  }, "conv3x3 wgrad");
  const int64_t nk = (int64_t)kout * 9 * c;
  const unsigned blocks = (unsigned)((nk / 8 + 15) / 16);
  dispatch_float(out_dtype, [&](auto tag) {
    using TO = typename decltype(tag)::type;
    hipLaunchKernelGGL((c1w::wgrad_reduce<TO>), dim3(blocks), dim3(256), 0, s, ws, sp, nk, static_cast<TO*>(dw));
  }, "conv3x3 wgrad reduce");
  check_launch("conv3x3_wgrad");
}

bool conv1x1_wgrad_supported(int64_t m, int n, int k) {
  return m > 0 && n % 64 == 0 && k % 64 == 0 && n >= 64 && k >= 64;
}

int64_t conv1x1_wgrad_workspace_floats(int64_t m, int n, int k, int cus) {
  return (int64_t)c1w::splits(m, n, k, cus) * n * k;
}

void conv1x1_wgrad(const void* g, const void* x, void* dw, int out_dtype, int64_t m, int n, int k, int dtype,
                   const float* xcoef, float* ws, int cus, hipStream_t s) {
  if (!conv1x1_wgrad_supported(m, n, k)) throw std::runtime_error("conv1x1 wgrad: unsupported shape");
  c1w::Args a;
  a.g = static_cast<const uint16_t*>(g);
  a.x = static_cast<const uint16_t*>(x);
  a.ws = ws;
  a.m = m;
  a.n = n;
  a.k = k;
  a.xcoef = xcoef;
  const int sp = c1w::splits(m, n, k, cus);
  a.rows = ((m + sp - 1) / sp + c1w::MB - 1) / c1w::MB * c1w::MB;
  dispatch_16(dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (xcoef) c1w::launch<T, true>(a, sp, cus, s);
    else c1w::launch<T, false>(a, sp, cus, s);
  }, "conv1x1 wgrad");
  const int64_t nk = (int64_t)n * k;
  const unsigned blocks = (unsigned)((nk / 8 + 15) / 16);
  dispatch_float(out_dtype, [&](auto tag) {
    using TO = typename decltype(tag)::type;
    hipLaunchKernelGGL((c1w::wgrad_reduce<TO>), dim3(blocks), dim3(256), 0, s, ws, sp, nk, static_cast<TO*>(dw));
  }, "conv1x1 wgrad reduce");
  check_launch("conv1x1_wgrad");
}

void conv1x1_bn_part_payload(const float* part, int g, int c, float n, const float* shift, float* payload,
                             hipStream_t s) {
  hipLaunchKernelGGL(c1bn::part_payload, dim3((c + 7) / 8), dim3(8 * c1bn::kFinG), 0, s, part, g, c, n, shift, payload);
  check_launch("conv1x1_bn_part_payload");
}

void conv1x1_bnbwd_finalize(const float* part, int g, int c, float inv_n, const float* mean, const float* istd,
                            const float* w, float* gw, float* gb, float* coef, hipStream_t s) {
  hipLaunchKernelGGL(c1bn::bwd_finalize, dim3((c + 7) / 8), dim3(8 * c1bn::kFinG), 0, s, part, g, c, inv_n, mean, istd, w, gw, gb,
                     coef);
  check_launch("conv1x1_bnbwd_finalize");
}

}  // namespace apex_amd
