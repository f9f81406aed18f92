// Fused 1x1 convolutions with a DEEP reduction (K = 1024 / 2048: the ResNet-50 stage-3 / 4 1x1s
// whose reduction runs over the 4w block channels) — the K-streamed sibling of conv1x1_bn.hip.
//
// conv1x1_bn.hip keeps the whole weight tile [NC][K] resident in LDS and streams each activation
// row exactly once; at K >= 1024 that image no longer fits (256 x 1024 x 2 B = 512 KB), so those
// layers ran on hipBLASLt with the batch norms as separate passes: the block output apply
// (relu(bn3(y3) + shortcut), read 2 + write 1 tensors), the statistics pass of conv1's output and
// the bn3 dx pass before conv3's data gradient (profiles/r06/resnet50_step_timeline_r06b.md:
// 55 + 37 + 18 us per stage-3 block forward, 54 + 37 + 15 backward).  Here:
//   * 8 waves x 32 rows = 256-row tiles x NC output columns per workgroup, one workgroup per CU,
//     persistent over the tiles of its column block;
//   * the weights stream through a 3-slot LDS ring in 64-deep chunks by LDS-DMA
//     (buffer_load ... lds, no staging registers), issued two chunks ahead under counted vmcnt
//     waits, one barrier per chunk.  (A register-staged ring with the next chunk loaded under the
//     current one waited ~1-2 us per chunk on the L2 and ran the stage-3 deferred-output conv at
//     190 us: profiles/r06/resnet50_step_timeline_r06e.md.)  The images are XOR-swizzled on the
//     source address (the DMA writes 1-KB lane-linear pieces): [NC][64] chunk c of row r at
//     c ^ ((r >> 1) & 7) for ds_read_b128 fragments; the dgrad form (weights [K][ncols]) keeps the
//     chunk k-major, chunk c of k-row r at c ^ ((r & 3) << 1), and reads B fragments with
//     ds_read_b64_tr_b16, so no transposed copy of the weight is needed;
//   * the activation operand goes HBM -> registers (the MFMA A-operand map, wave-private, two
//     chunks ahead), so the operand prologues of conv1x1_bn.hip apply unchanged: the block below's
//     output BN + shortcut + ReLU (kProBnAddRelu: the deferred output, written with its ReLU bits
//     as by-products) and the BN backward dx (kProBnBwd: dx written for the weight gradient);
//   * epilogues: the consuming BN's statistics partials (forward), or the output BN's backward
//     reduction with its ReLU mask recomputed from its input (dgrad form: bn2's sums under
//     conv3's data gradient).
// The arithmetic of every prologue / epilogue is conv1x1_bn.hip's, so results are bitwise those of
// the apply passes they replace.
#include "apex_amd/conv_ks.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/mfma.h"

#include <cstdlib>
#include <stdexcept>

namespace apex_amd {
namespace c1ks {
using namespace mfma;

struct Args {
  const uint16_t* a;    // [M][K]
  const uint16_t* w;    // !WT: [ncols][K]   WT: [K][ncols]
  uint16_t* y;          // [M][ncols]
  int64_t m;
  int k, ncols, ntiles;
  const float* pcoef;   // PRO rows [rows][K]
  const float* pc_res;  // kProBnAddRelu split form: the residual BN's [2][K] (null: identity)
  int pc_split;
  const float* shift;   // STATS: per-output-channel shift [ncols] (nullable)
  float* part;          // STATS / RED: [2][gridDim.x][ncols]
  const uint16_t* py;   // two-operand prologue: second tensor [M][K]
  uint16_t* aout;       // nullable: the transformed operand [M][K]
  uint8_t* bout;        // nullable (kProBnAddRelu): its ReLU bits [M K / 8]
  const float* rcoef;   // RED: the output BN's forward coefficients [2][ncols] (mask recomputed)
  const uint16_t* rx;   // RED: that BN's input [M][ncols]
  const float* rmean;   // RED: its batch mean [ncols]
};

constexpr int kProNone = 0, kProBnBwd = 2, kProBnAddRelu = 3;  // codes of conv1x1_bn.hip
constexpr int pro_rows(int pro) { return pro == kProBnBwd ? 3 : pro == kProBnAddRelu ? 4 : 0; }
constexpr bool pro_two(int pro) { return pro != kProNone; }
constexpr int NW = 8, NT = NW * 64, ROWS = NW * 32;
constexpr int kSS = 64 + 8;  // staging row stride (elements)
// 64-deep chunks: with 32 (the register budget of a 256-column tile beside a two-operand prologue)
// the stage-3 deferred-output conv ran 190 us, latency-bound on one chunk of operands in flight per
// wave; the two-operand prologues therefore take at most 128 columns (col_tile) and 64-deep chunks
// two ahead (profiles/r06/resnet50_step_timeline_r06e.md)
constexpr int KCH = 64;        // reduction depth of one weight chunk
// weight ring slots: at step j the wave reads slot j % 3, chunk j + 1 is landing and chunk j + 2 is
// issued (after the step's barrier) into the slot every wave finished reading in step j - 1
constexpr int WS = 3;
constexpr int slot_el(int nc) { return nc * KCH; }

// (RED: the per-wave backward sums stay in registers and meet in the weight ring after the loop)
inline size_t lds_bytes(int nc, int pro, int k) {
  return (size_t)WS * slot_el(nc) * 2 + (size_t)NW * 32 * kSS * 2 + (size_t)pro_rows(pro) * k * 4;
}

__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint16_t* lds_dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff, 0, 0,
                                           0);
}

// B fragment of a [KCH][NC] k-major swizzled image (chunk c of k-row r at c ^ ((r & 3) << 1)):
// lane gets n = colbase + (lane & 31), k rows klo + 0..3 and khi + 0..3 (klo, khi multiples of 4)
template <int NC>
__device__ __forceinline__ s16x8 frag_tr_swz(const uint16_t* img, int colbase, int klo, int khi, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int col = colbase + 16 * (g & 1) + 4 * pp;
  const int off = ((((col >> 3) ^ (q << 1))) << 3) + (col & 7);
  const s16x4 lo = tr_read(img + (klo + q) * NC + off);
  const s16x4 hi = tr_read(img + (khi + q) * NC + off);
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <typename T, int NC, bool WT, int PRO, bool STATS, bool RED, int DEPTH>
__global__ void __launch_bounds__(NT, 1) fused1x1_ks(Args p) {
  constexpr int KC = KCH / 16;  // k-steps per chunk
  constexpr int CN = NC / 32;   // accumulator blocks per wave
  constexpr int SLOT = slot_el(NC);
  constexpr int PW = NC * KCH * 2 / 1024 / NW;  // 1-KB DMA pieces per wave per chunk
  constexpr int LA = pro_two(PRO) ? 2 * KC : KC;  // operand loads per wave per chunk
  static_assert(PW >= 1 && NC * KCH * 2 == PW * NW * 1024, "weight chunk must split into whole pieces per wave");
  // (the counted DMA wait below holds for any DEPTH: the DMA runs two chunks ahead of its use and
  // every step issues PW pieces + LA operand loads)
  static_assert(DEPTH >= 2, "operand fragments at least one step ahead");
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* bimg = lds;                                            // [WS][SLOT]
  uint16_t* stg = lds + WS * SLOT;                                 // [NW][32][kSS]
  float* pc = reinterpret_cast<float*>(stg + NW * 32 * kSS);       // [rows][K]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, lr = lane & 31, lh = lane >> 5;
  const int col0 = blockIdx.y * NC;
  const int K = p.k;
  const int nch = K / KCH;

  // ---- weight chunk DMA: this wave's PW pieces of chunk ch into ring slot `slot` ----
  const int wave = __builtin_amdgcn_readfirstlane(wid);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.w, 0, __builtin_amdgcn_readfirstlane((int)((int64_t)K * p.ncols * 2)), 0x00020000);
  uint32_t wrel[PW];  // per-lane byte offset of its 16-byte piece, chunk 0
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int pid = wave + NW * i;
    if constexpr (!WT) {  // [NC][64]: piece = 8 rows of 128 B
      const int row = 8 * pid + (lane >> 3), cl = lane & 7, cs = cl ^ ((row >> 1) & 7);
      wrel[i] = (uint32_t)(((col0 + row) * K + 8 * cs) * 2);
    } else {  // [64][NC]: piece = 1024 / (2 NC) k-rows
      constexpr int CPR = NC / 8;  // 16-byte chunks per k-row
      const int row = (64 / CPR) * pid + lane / CPR, cl = lane % CPR, cs = cl ^ ((row & 3) << 1);
      wrel[i] = (uint32_t)((row * p.ncols + col0 + 8 * cs) * 2);
    }
  }
  auto wdma = [&](int ch, int slot) {
    const uint32_t cofs = !WT ? (uint32_t)(ch * KCH * 2) : (uint32_t)(ch * KCH * p.ncols * 2);
#pragma unroll
    for (int i = 0; i < PW; ++i) bdma16(wr, wrel[i] + cofs, bimg + slot * SLOT + (wave + NW * i) * 512);
  };
  // coefficient rows by 16-byte loads (K % 64 == 0; the rows start 16-byte aligned when the
  // tensors do), several in flight per thread
  const bool pc_vec = ((reinterpret_cast<uintptr_t>(p.pcoef) | reinterpret_cast<uintptr_t>(p.pc_res)) & 15) == 0;
  if constexpr (PRO == kProBnAddRelu) {
    if (p.pc_split && pc_vec) {
#pragma unroll 4
      for (int i = tid; i < K; i += NT) {  // 4 rows x K / 4 vectors
        const int row = i / (K / 4), kk = (i - row * (K / 4)) * 4;
        float4 v;
        if (row == 0 || row == 2) v = *reinterpret_cast<const float4*>(p.pcoef + (row >> 1) * K + kk);
        else if (p.pc_res) v = *reinterpret_cast<const float4*>(p.pc_res + (row >> 1) * K + kk);
        else v = row == 1 ? make_float4(1.f, 1.f, 1.f, 1.f) : make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(pc + row * K + kk) = v;
      }
    } else if (p.pc_split) {
      for (int i = tid; i < 4 * K; i += NT) {
        const int row = i / K, kk = i - row * K;
        float v;
        if (row == 0 || row == 2) v = p.pcoef[(row >> 1) * K + kk];
        else if (p.pc_res) v = p.pc_res[(row >> 1) * K + kk];
        else v = row == 1 ? 1.f : 0.f;
        pc[i] = v;
      }
    } else if (pc_vec) {
#pragma unroll 4
      for (int i = tid; i < K; i += NT) reinterpret_cast<float4*>(pc)[i] = reinterpret_cast<const float4*>(p.pcoef)[i];
    } else {
      for (int i = tid; i < 4 * K; i += NT) pc[i] = p.pcoef[i];
    }
  } else if constexpr (PRO != kProNone) {
    if (pc_vec) {
#pragma unroll 4
      for (int i = tid; i < pro_rows(PRO) * K / 4; i += NT)
        reinterpret_cast<float4*>(pc)[i] = reinterpret_cast<const float4*>(p.pcoef)[i];
    } else {
      for (int i = tid; i < pro_rows(PRO) * K; i += NT) pc[i] = p.pcoef[i];
    }
  }
  float sh[CN], s1[CN], s2[CN];
  float racc[RED ? CN / 2 : 1][2] = {};  // RED: this lane's column of each 64-column group (see epilogue)
#pragma unroll
  for (int cb = 0; cb < CN; ++cb) {
    sh[cb] = (STATS && p.shift) ? p.shift[col0 + 32 * cb + lr] : 0.f;
    s1[cb] = s2[cb] = 0.f;
  }

  f32x16 acc[CN];
#pragma unroll
  for (int cb = 0; cb < CN; ++cb) acc[cb] = zero16();

  constexpr int KY = pro_two(PRO) ? KC : 1;
  struct Frags {
    s16x8 a[KC];
    s16x8 y[KY];
  };
  auto load = [&](Frags& f, int t, int ch) {
    int64_t row = (int64_t)t * ROWS + wid * 32 + lr;
    if (row >= p.m) row = p.m - 1;  // tail rows: valid memory, masked in the epilogue
    const int64_t off = row * K + ch * KCH + 8 * lh;
#pragma unroll
    for (int s = 0; s < KC; ++s) f.a[s] = *reinterpret_cast<const s16x8*>(p.a + off + 16 * s);
    if constexpr (pro_two(PRO)) {
#pragma unroll
      for (int s = 0; s < KC; ++s) f.y[s] = *reinterpret_cast<const s16x8*>(p.py + off + 16 * s);
    }
  };

  auto compute = [&](const Frags& f, int t, int ch, int slot) {
    const uint16_t* b = bimg + slot * SLOT;
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      s16x8 a = f.a[s];
      if constexpr (pro_two(PRO)) {
        const int kb = ch * KCH + 16 * s + 8 * lh;
        constexpr int NQ = pro_rows(PRO);
        float c[NQ][8];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const float4 u0 = *reinterpret_cast<const float4*>(pc + q * K + kb);
          const float4 u1 = *reinterpret_cast<const float4*>(pc + q * K + kb + 4);
          c[q][0] = u0.x; c[q][1] = u0.y; c[q][2] = u0.z; c[q][3] = u0.w;
          c[q][4] = u1.x; c[q][5] = u1.y; c[q][6] = u1.z; c[q][7] = u1.w;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v;
          if constexpr (PRO == kProBnAddRelu) {
            v = fmaf(to_f(T{(uint16_t)a[j]}), c[0][j], c[2][j]) + fmaf(to_f(T{(uint16_t)f.y[s][j]}), c[1][j], c[3][j]);
            v = fmaxf(v, 0.f);
          } else {
            v = fmaf(c[0][j], to_f(T{(uint16_t)a[j]}), fmaf(c[1][j], to_f(T{(uint16_t)f.y[s][j]}), c[2][j]));
          }
          a[j] = (short)from_f<T>(v).x;
        }
        if (p.aout && blockIdx.y == 0)
          *reinterpret_cast<s16x8*>(stg + wid * 32 * kSS + lr * kSS + 16 * s + 8 * lh) = a;
      }
#pragma unroll
      for (int cb = 0; cb < CN; ++cb) {
        s16x8 bf;
        if constexpr (!WT) {
          const int r = 32 * cb + lr, c = 2 * s + lh;
          bf = *reinterpret_cast<const s16x8*>(b + r * KCH + ((c ^ ((r >> 1) & 7)) << 3));
        } else {
          bf = frag_tr_swz<NC>(b, 32 * cb, 16 * s + 8 * lh, 16 * s + 8 * lh + 4, lane);
        }
        acc[cb] = mma<T>(a, bf, acc[cb]);
      }
    }
    if constexpr (pro_two(PRO)) {
      // the chunk's transformed operand [32 rows][KCH] (and its ReLU bits) out of the wave's slab
      // as whole-row runs
      if (p.aout && blockIdx.y == 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint16_t* sl = stg + wid * 32 * kSS;
        constexpr int LPR = KCH / 8;
        const int64_t row0 = (int64_t)t * ROWS + wid * 32;
#pragma unroll
        for (int i = 0; i < 32 * LPR / 64; ++i) {
          const int qid = lane + 64 * i, rr = qid / LPR, c8 = (qid % LPR) * 8;
          const s16x8 v = *reinterpret_cast<const s16x8*>(sl + rr * kSS + c8);
          if (row0 + rr < p.m) {
            const int64_t off = (row0 + rr) * K + ch * KCH + c8;
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
    const int64_t row0 = (int64_t)t * ROWS + wid * 32;
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
      uint4 xq[4];
      if constexpr (RED) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qid = lane + 64 * i, rr = qid >> 3, c8 = (qid & 7) * 8;
          const int64_t off = (row0 + rr) * p.ncols + col0 + 64 * g + c8;
          xq[i] = row0 + rr < p.m ? *reinterpret_cast<const uint4*>(p.rx + off) : make_uint4(0, 0, 0, 0);
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) st[crow(r, lh) * kSS + 32 * q + lr] = from_f<T>(acc[2 * g + q][r]).x;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      float rs[8], rq[8], mu[8], rsc[8], rsh[8];
      if constexpr (RED) {
#pragma unroll
        for (int j = 0; j < 8; ++j) rs[j] = rq[j] = 0.f;
        const int cc = col0 + 64 * g + (lane & 7) * 8;
        Vec8<float>::load(mu, p.rmean + cc);
        Vec8<float>::load(rsc, p.rcoef + cc);
        Vec8<float>::load(rsh, p.rcoef + p.ncols + cc);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qid = lane + 64 * i, rr = qid >> 3, c8 = (qid & 7) * 8;
        uint4 v = *reinterpret_cast<const uint4*>(st + rr * kSS + c8);
        const int64_t off = (row0 + rr) * p.ncols + col0 + 64 * g + c8;
        if (row0 + rr < p.m) {
          if constexpr (RED) {
            float a[8], xv[8];
            Vec8<T>::load(a, reinterpret_cast<const T*>(&v));
            Vec8<T>::load(xv, reinterpret_cast<const T*>(&xq[i]));
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              // the stored (rounded) gradient, masked by the BN's forward ReLU recomputed from x
              const float gq = fmaf(xv[j], rsc[j], rsh[j]) > 0.f ? a[j] : 0.f;
              a[j] = gq;
              rs[j] += gq;
              rq[j] = fmaf(gq, xv[j] - mu[j], rq[j]);
            }
            Vec8<T>::store(reinterpret_cast<T*>(&v), a);
          }
          *reinterpret_cast<uint4*>(p.y + off) = v;
        }
      }
      if constexpr (RED) {
        // reduce-scatter over lane bits 5, 4, 3 (lanes l ^ 8k hold the same 8 columns), then the
        // 64 lanes own 64 distinct columns of this wave's LDS accumulators (see conv1x1_bn.hip)
#pragma unroll
        for (int sp = 0; sp < 3; ++sp) {
          const int msk = 32 >> sp, half = 4 >> sp;
          const bool up = (lane & msk) != 0;
#pragma unroll
          for (int j = 0; j < half; ++j) {
            const float ss = up ? rs[j] : rs[j + half];
            const float sq = up ? rq[j] : rq[j + half];
            const float gs = __shfl_xor(ss, msk, 64);
            const float gq = __shfl_xor(sq, msk, 64);
            rs[j] = (up ? rs[j + half] : rs[j]) + gs;
            rq[j] = (up ? rq[j + half] : rq[j]) + gq;
          }
        }
        racc[g][0] += rs[0];
        racc[g][1] += rq[0];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int cb = 0; cb < CN; ++cb) acc[cb] = zero16();
  };

  // ---- flat (tile, chunk) stream: operand fragments DEPTH - 1 steps ahead in registers, weight
  // chunks two steps ahead by DMA into the 3-slot ring, one barrier per chunk.  At the top of step
  // j this wave's DMA of chunk j has landed once at most 2 LA + PW of its vector-memory operations
  // are outstanding (two steps of operand loads and the next chunk's pieces were issued after it;
  // conditional stores only add to that count); the barrier then publishes every wave's pieces and
  // retires every read of the slot refilled next (read two steps earlier). ----
  const int tlast = p.ntiles - 1;
  auto adv = [&](int& tt, int& cc) {
    if (++cc == nch) {
      cc = 0;
      tt += gridDim.x;
    }
  };
  int t = blockIdx.x, ch = 0;
  wdma(0, 0);
  wdma(nch > 1 ? 1 : 0, 1);
  Frags f[DEPTH];
  int tn = t, cn = ch;
#pragma unroll
  for (int j = 0; j < DEPTH - 1; ++j) {
    load(f[j], min(tn, tlast), cn);
    adv(tn, cn);
  }
  int step = 0, chw = nch > 2 ? 2 : 2 % nch;  // chunk index of the next DMA (chunks cycle per tile)
  bool done = t >= p.ntiles;
  while (!done) {
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) {
      if (!done) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LA + PW) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (step 0: the coefficient / sum writes)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        wdma(chw, (step + 2) % WS);
        chw = chw + 1 == nch ? 0 : chw + 1;
        load(f[(j + DEPTH - 1) % DEPTH], min(tn, tlast), cn);
        adv(tn, cn);
        compute(f[j], t, ch, step % WS);
        if (ch == nch - 1) epilogue(t);
        ++step;
        adv(t, ch);
        done = t >= p.ntiles;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup's LDS is released

  if constexpr (RED) {
    // per-wave sums [NW][2][NC] into the (now idle) weight ring, then a fixed-order wave reduction
    float* rsum = reinterpret_cast<float*>(bimg);
    __syncthreads();
    const int jc = ((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1);
#pragma unroll
    for (int g = 0; g < CN / 2; ++g) {
      float* r0p = rsum + (wid * 2) * NC + 64 * g + (lane & 7) * 8 + jc;
      r0p[0] = racc[g][0];
      r0p[NC] = racc[g][1];
    }
    __syncthreads();
    for (int i = tid; i < 2 * NC; i += NT) {
      const int which = i / NC, n = i % NC;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += rsum[(w * 2 + which) * NC + n];
      p.part[((int64_t)which * gridDim.x + blockIdx.x) * p.ncols + col0 + n] = v;
    }
  }
  if constexpr (STATS) {
    float* red = reinterpret_cast<float*>(stg);  // [NW][2][NC] (16 KB at NC = 256 <= the staging slab)
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
      for (int w = 0; w < NW; ++w) v += red[(w * 2 + which) * NC + n];
      p.part[((int64_t)which * gridDim.x + blockIdx.x) * p.ncols + col0 + n] = v;
    }
  }
}

// ---- launch planning ----
inline int env_nc() {
  static const int v = [] {
    const char* e = std::getenv("APEX_AMD_C1KS_NC");  // A/B knob: force a column tile
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

// column tile: the widest that still gives ~3/4 of the CUs a tile (stage 4's 12544 rows are only
// 49 tiles of 256), dividing ncols
inline int col_tile(int64_t m, int ncols, int cus, int pro) {
  const int f = env_nc();
  if (f == 64 || f == 128 || f == 256) {
    if (ncols % f == 0) return f;
  }
  const int64_t ntiles = (m + ROWS - 1) / ROWS;
  for (int nc : {256, 128, 64}) {
    if (nc == 256 && pro_two(pro)) continue;
    if (ncols % nc) continue;
    if (nc == 64 || ntiles * (ncols / nc) * 4 >= (int64_t)cus * 3) return nc;
  }
  return 64;
}

inline int grid_x(int64_t m, int nc, int ncols, int cus) {
  const int64_t ntiles = (m + ROWS - 1) / ROWS;
  const int gy = ncols / nc;
  int64_t gx = ((int64_t)cus + gy - 1) / gy;
  if (gx > ntiles) gx = ntiles;
  return (int)(gx < 1 ? 1 : gx);
}

template <typename T, int NC, bool WT, int PRO, bool STATS, bool RED>
void launch(const Args& a0, int cus, hipStream_t s) {
  // operand fragments in flight per wave: two chunks ahead, one beside 256 columns with a two-operand
  // prologue (the register file holds 8 accumulator blocks + one chunk of both operands)
  constexpr int DEPTH = (NC == 256 && pro_two(PRO)) ? 2 : 3;
  const size_t lds = lds_bytes(NC, PRO, a0.k);
  if (lds > 160 * 1024) throw std::runtime_error("conv1x1_ks: LDS budget exceeded (reduction too deep for the prologue)");
  auto kern = &fused1x1_ks<T, NC, WT, PRO, STATS, RED, DEPTH>;
  static size_t attr = 0;
  if (attr < lds) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(160 * 1024));
    attr = 160 * 1024;
  }
  Args a = a0;
  a.ntiles = (int)((a.m + ROWS - 1) / ROWS);
  const int gx = grid_x(a.m, NC, a.ncols, cus);
  hipLaunchKernelGGL(kern, dim3(gx, a.ncols / NC), dim3(NT), lds, s, a);
}

template <typename T, bool WT, int PRO, bool STATS, bool RED>
void dispatch_nc(const Args& a, int nc, int cus, hipStream_t s) {
  if (nc == 256) return launch<T, 256, WT, PRO, STATS, RED>(a, cus, s);
  if (nc == 128) launch<T, 128, WT, PRO, STATS, RED>(a, cus, s);
  else launch<T, 64, WT, PRO, STATS, RED>(a, cus, s);
}

}  // namespace c1ks

bool conv1x1_ks_supported(int64_t m, int k, int ncols) {
  return m > 0 && k >= 64 && k % 64 == 0 && k <= 4096 && ncols > 0 && ncols % 64 == 0 && m * (int64_t)k < (1ll << 40);
}

int conv1x1_ks_partials(int64_t m, int k, int ncols, int cus, int pro) {
  (void)k;
  return c1ks::grid_x(m, c1ks::col_tile(m, ncols, cus, pro), ncols, cus);
}

void conv1x1_ks(const void* a, const void* w, void* y, int64_t m, int k, int ncols, bool wt, int dtype,
                const float* pcoef, int pro, bool pc_split, const float* pc_res, const float* shift, float* part,
                const void* py, void* aout, uint8_t* bout, const float* rcoef, const void* rx, const float* rmean,
                int cus, hipStream_t s) {
  if (!conv1x1_ks_supported(m, k, ncols)) throw std::runtime_error("conv1x1_ks: unsupported shape");
  if (pro != c1ks::kProNone && pro != c1ks::kProBnBwd && pro != c1ks::kProBnAddRelu)
    throw std::runtime_error("conv1x1_ks: prologue must be none / BN backward / BN + add + ReLU");
  if ((pro != c1ks::kProNone) != (pcoef != nullptr && py != nullptr))
    throw std::runtime_error("conv1x1_ks: a prologue needs pcoef and py");
  if (wt && pro == c1ks::kProBnAddRelu) throw std::runtime_error("conv1x1_ks: the add + ReLU prologue is a forward option");
  if (!wt && pro == c1ks::kProBnBwd) throw std::runtime_error("conv1x1_ks: the BN-backward prologue is a dgrad option");
  const bool red = rx != nullptr;
  if (red && (!wt || !rcoef || !rmean || !part)) throw std::runtime_error("conv1x1_ks: RED needs the dgrad form, rcoef, rmean, part");
  const bool stats = !wt && part != nullptr;
  if (bout && pro != c1ks::kProBnAddRelu) throw std::runtime_error("conv1x1_ks: bout needs the add + ReLU prologue");
  if (((uintptr_t)a | (uintptr_t)w | (uintptr_t)y) & 15) throw std::runtime_error("conv1x1_ks: operands must be 16-byte aligned");
  c1ks::Args args{};
  args.a = static_cast<const uint16_t*>(a);
  args.w = static_cast<const uint16_t*>(w);
  args.y = static_cast<uint16_t*>(y);
  args.m = m;
  args.k = k;
  args.ncols = ncols;
  args.pcoef = pcoef;
  args.pc_res = pc_res;
  args.pc_split = pc_split ? 1 : 0;
  args.shift = shift;
  args.part = part;
  args.py = static_cast<const uint16_t*>(py);
  args.aout = static_cast<uint16_t*>(aout);
  args.bout = bout;
  args.rcoef = rcoef;
  args.rx = static_cast<const uint16_t*>(rx);
  args.rmean = rmean;
  const int nc = c1ks::col_tile(m, ncols, cus, pro);
  dispatch_16(dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (wt) {
      if (pro == c1ks::kProBnBwd) {
        if (red) c1ks::dispatch_nc<T, true, c1ks::kProBnBwd, false, true>(args, nc, cus, s);
        else c1ks::dispatch_nc<T, true, c1ks::kProBnBwd, false, false>(args, nc, cus, s);
      } else {
        if (red) c1ks::dispatch_nc<T, true, c1ks::kProNone, false, true>(args, nc, cus, s);
        else c1ks::dispatch_nc<T, true, c1ks::kProNone, false, false>(args, nc, cus, s);
      }
    } else {
      if (pro == c1ks::kProBnAddRelu) {
        if (stats) c1ks::dispatch_nc<T, false, c1ks::kProBnAddRelu, true, false>(args, nc, cus, s);
        else c1ks::dispatch_nc<T, false, c1ks::kProBnAddRelu, false, false>(args, nc, cus, s);
      } else {
        if (stats) c1ks::dispatch_nc<T, false, c1ks::kProNone, true, false>(args, nc, cus, s);
        else c1ks::dispatch_nc<T, false, c1ks::kProNone, false, false>(args, nc, cus, s);
      }
    }
  }, "conv1x1_ks");
  check_launch("conv1x1_ks");
}

}  // namespace apex_amd
