// Backward of a bottleneck block's expanding 1x1 convolution (conv3: W -> C4 channels) with both
// neighbouring batch norms fused, in ONE pass over the pixels:
//
//   dx3 = A3 dm + B3 y3 + K3                 bn3's data gradient (dm = the masked block-output
//                                            gradient, y3 = bn3's input): the operand prologue
//   dz2 = mask2 . (dx3 W3)                   conv3's data gradient, masked with bn2's ReLU
//                                            (recomputed from y2) -> bn2's backward sums
//   dW3 += dx3^T relu(bn2(y2))               conv3's weight gradient, bn2's apply+ReLU on load
//
// The unfused sequence (dgrad kernel writing dx3 as a by-product, weight-gradient kernel re-reading
// dx3 and y2) moves dm, y3, y2 once plus dx3 twice (write + read) and y2 twice; here dx3 lives only
// in LDS: per 64-pixel tile the workgroup reads dm, y3 [64][C4] and y2 [64][W], writes dz2 [64][W].
// At ResNet-50 stage 1 (C4 = 256, W = 64, 802,816 pixels) that is 1.03 GB instead of 1.95 GB.
//
// gfx950 layout (one persistent workgroup per CU, 64-pixel tiles, LDS double-buffered), 8 waves in
// two roles so the matrix work never waits on HBM:
//  * 4 loader waves: 16-byte global loads of dm / y3 / y2 into registers TWO tiles ahead; dx3
//    computed in registers (fp32 FMA, rounded to the storage type like the unfused path's dx3
//    tensor) and written with y2 into the free LDS stage; one barrier per tile;
//  * 4 math waves, as follows:
//  * GEMM 1, swapped (dz2^T = W3^T dx3^T): the W3^T fragments are the A operand, resident in
//    registers for the whole kernel; B fragments are 16-byte row reads of the dx3 image; rows of
//    W3^T permuted so each lane ends with 16 consecutive channels of one pixel (16-byte y2 reads
//    from LDS, two 16-byte dz2 stores, per-lane bn2 sums);
//  * GEMM 2: dW3 [C4][W] accumulated across all tiles in AGPRs (4 32x32 tiles per wave), both
//    operands read with ds_read_b64_tr_b16 from the pixel-major images; bn2's apply+ReLU applied
//    to the B fragments in registers (one channel per lane: two coefficients);
//  * per-workgroup fp32 dW3 partials and bn2 partial rows, reduced in a fixed order.
// Reference capability: the fused dgrad / wgrad graphs with the BN-backward "dscale / dbias"
// fusions of apex/contrib/csrc/bottleneck/bottleneck.cpp:1104-1534.
#include "apex_amd/conv_api.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/mfma.h"

#include <stdexcept>

namespace apex_amd {
namespace c3b {
using namespace mfma;

constexpr int TM = 64;  // pixels per tile

// LDS-only barrier: this wave's LDS accesses complete, then a raw s_barrier.  __syncthreads()
// also drains every outstanding GLOBAL load (its workgroup fence waits vmcnt), which would
// serialize the register prefetch that is meant to stay in flight across the barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct Args {
  const uint16_t* dm;    // [M][C4]
  const uint16_t* y3;    // [M][C4]
  const uint16_t* y2;    // [M][W]
  const uint16_t* w3;    // [C4][W]  (conv3 weight, [Cout][Cin])
  const float* cb3;      // [3][C4]  bn3 backward coefficients
  const float* c2;       // [2][W]   bn2 forward scale | shift
  const float* mean2;    // [W]
  uint16_t* dz2;         // [M][W]
  float* part2;          // [2][G][W]
  float* ws;             // [G][C4][W]
  int64_t m;
  int ntiles;
};

template <int C4, int W>
struct Cfg {
  static constexpr int DS = C4 + 16;  // dx3 row stride: 2 DS bytes = 32 mod 256
  static constexpr int YS = W + 32;   // y2 row stride: rows 64 B apart in bank space (transposed reads)
  static constexpr int BUF = TM * DS + TM * YS;  // elements per LDS stage
  static constexpr int LDS = 2 * BUF * 2;
  static constexpr int KS1 = C4 / 16;  // GEMM 1 k-steps
  static constexpr int CPR = C4 / 8;   // 16-byte chunks per dm / y3 row
  static constexpr int NQ = TM * CPR / 256;      // dm / y3 chunks per loader thread per tile
  static constexpr int NY = TM * (W / 8) / 256;  // y2 chunks per loader thread per tile
  static_assert(C4 == 256 && W == 64, "register plan: 4 math waves = 2 channel tiles x 2 pixel halves");
  static_assert(NQ * 256 == TM * CPR && NY * 256 == TM * (W / 8), "staging split");
  static_assert(4 * 64 * 17 * 4 <= LDS, "statistics fold aliases the stages");
};

__device__ __forceinline__ int chan_of_row(int r) { return 16 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3); }

// 8 waves: waves 0-3 are the math waves (both GEMMs, epilogue, accumulators), waves 4-7 the
// loader waves (global -> registers two tiles ahead, dx3 -> LDS).  Iteration j: loaders commit
// tile j into stage j % 2 and issue tile j + 2; math waves compute tile j - 1 from stage
// (j - 1) % 2; one barrier.  The math waves never wait on HBM, the loaders keep two tiles
// (144 KB per CU) of loads in flight.
template <typename T, int C4, int W>
__global__ void __launch_bounds__(512, 1) fused_kernel(const Args p) {
  using C = Cfg<C4, W>;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  __shared__ __attribute__((aligned(16))) float ec[3 * W];  // bn2 scale | shift | mean (math waves)
  auto dxb = [&](int b) { return lds + b * C::BUF; };
  auto y2b = [&](int b) { return lds + b * C::BUF + TM * C::DS; };
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, pl = lane & 31;
  const bool loader = wave >= 4;
  // this workgroup's tiles: blockIdx.x, + gridDim.x, ...
  const int nmine = p.ntiles > (int)blockIdx.x ? (p.ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  auto tile_of = [&](int i) { return (int)blockIdx.x + i * (int)gridDim.x; };
  const int nsync = (nmine + 2) & ~1;  // barriers per role: >= nmine + 1, even (loader unroll)

  if (loader) {
    const int tid = threadIdx.x - 256;
    const int qc = (tid % C::CPR) * 8, qr = tid / C::CPR;  // dm / y3: rows qr + (256 / CPR) i
    const int yc = (tid % (W / 8)) * 8, yr = tid / (W / 8);
    float cA[8], cB[8], cK[8];
    Vec8<float>::load(cA, p.cb3 + qc);
    Vec8<float>::load(cB, p.cb3 + C4 + qc);
    Vec8<float>::load(cK, p.cb3 + 2 * C4 + qc);
    uint4 rdm[2][C::NQ], ry3[2][C::NQ], ry2[2][C::NY];
    auto issue = [&](int set, int t) {
#pragma unroll
      for (int i = 0; i < C::NQ; ++i) {
        int64_t row = (int64_t)t * TM + qr + (256 / C::CPR) * i;
        if (row >= p.m) row = p.m - 1;  // tail: valid memory, zeroed at commit
        rdm[set][i] = *reinterpret_cast<const uint4*>(p.dm + row * C4 + qc);
        ry3[set][i] = *reinterpret_cast<const uint4*>(p.y3 + row * C4 + qc);
      }
#pragma unroll
      for (int i = 0; i < C::NY; ++i) {
        int64_t row = (int64_t)t * TM + yr + (256 / (W / 8)) * i;
        if (row >= p.m) row = p.m - 1;
        ry2[set][i] = *reinterpret_cast<const uint4*>(p.y2 + row * W + yc);
      }
    };
    auto commit = [&](int set, int t, int b) {
#pragma unroll
      for (int i = 0; i < C::NQ; ++i) {
        const int lr = qr + (256 / C::CPR) * i;
        const bool ok = (int64_t)t * TM + lr < p.m;
        float g[8], y[8], d[8];
        Vec8<T>::load(g, reinterpret_cast<const T*>(&rdm[set][i]));
        Vec8<T>::load(y, reinterpret_cast<const T*>(&ry3[set][i]));
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = ok ? fmaf(cA[j], g[j], fmaf(cB[j], y[j], cK[j])) : 0.f;
        Vec8<T>::store(reinterpret_cast<T*>(dxb(b) + lr * C::DS + qc), d);
      }
#pragma unroll
      for (int i = 0; i < C::NY; ++i) {
        const int lr = yr + (256 / (W / 8)) * i;
        // component-wise (the aggregate copy kept ry2 in a scratch alloca)
        const uint32_t v0 = ry2[set][i].x, v1 = ry2[set][i].y, v2 = ry2[set][i].z, v3 = ry2[set][i].w;
        *reinterpret_cast<uint4*>(y2b(b) + lr * C::YS + yc) = make_uint4(v0, v1, v2, v3);
      }
    };
    // loads are issued unconditionally (past the end: the last tile again, discarded) and the
    // loop is unrolled by the two register sets, so every trip issues the same loads in the same
    // order and the compiler's vmcnt waits stay counted (a conditional issue makes it wait for
    // everything, which serializes the two tiles in flight)
    const int last = nmine > 0 ? nmine - 1 : 0;
    issue(0, tile_of(0));
    issue(1, tile_of(min(1, last)));
    for (int j = 0; j < nsync; j += 2) {
      if (j < nmine) commit(0, tile_of(j), 0);
      issue(0, tile_of(min(j + 2, last)));
      lds_barrier();
      if (j + 1 < nmine) commit(1, tile_of(j + 1), 1);
      issue(1, tile_of(min(j + 3, last)));
      lds_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the discarded tail prefetch
    __syncthreads();  // statistics fold (math waves)
    __syncthreads();
    __syncthreads();
    __syncthreads();
    return;
  }

  // ---------------- math waves ----------------
  const int ct = wave & 1, mh = wave >> 1;  // GEMM 1: channel tile, pixel half
  s16x8 wa[C::KS1];
  {
    const int c = 32 * ct + chan_of_row(pl);
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) wa[ks][j] = (short)p.w3[(size_t)(16 * ks + 8 * h + j) * W + c];
  }
  const int c0 = 32 * ct + 16 * h;
  // bn2 coefficients of the epilogue's channels: an LDS table (registers go to the accumulators)
  for (int i = threadIdx.x; i < 3 * W; i += 256) ec[i] = i < 2 * W ? p.c2[i] : p.mean2[i - 2 * W];
  float s1[16], s2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) s1[r] = s2[r] = 0.f;
  const float b_sc0 = p.c2[pl], b_sh0 = p.c2[W + pl], b_sc1 = p.c2[32 + pl], b_sh1 = p.c2[W + 32 + pl];
  f32x16 dw[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) dw[i][0] = dw[i][1] = zero16();

  for (int j = 0; j < nsync; ++j) {
    if (j >= 1 && j <= nmine) {
      const int t = tile_of(j - 1), cur = (j - 1) & 1;
      const uint16_t* dx = dxb(cur);
      const uint16_t* yy = y2b(cur);
      // GEMM 1: dz2^T tile [32 channels][32 pixels of half mh]
      f32x16 acc = zero16();
#pragma unroll
      for (int ks = 0; ks < C::KS1; ++ks) {
        const s16x8 bf = *reinterpret_cast<const s16x8*>(dx + (32 * mh + pl) * C::DS + 16 * ks + 8 * h);
        acc = mma<T>(wa[ks], bf, acc);
      }
      // GEMM 2: dW3 [k4 tiles 2 wave, 2 wave + 1][c tiles 0, 1] over the tile's 64 pixels
#pragma unroll
      for (int s = 0; s < TM / 16; ++s) {
        const int klo = 16 * s + 8 * h;
        const s16x8 a0 = frag_tr<C::DS>(dx, 64 * wave, klo, klo + 4, lane);
        const s16x8 a1 = frag_tr<C::DS>(dx, 64 * wave + 32, klo, klo + 4, lane);
        s16x8 b0 = frag_tr<C::YS>(yy, 0, klo, klo + 4, lane);
        s16x8 b1 = frag_tr<C::YS>(yy, 32, klo, klo + 4, lane);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          b0[e] = (short)from_f<T>(fmaxf(fmaf(to_f(T{(uint16_t)b0[e]}), b_sc0, b_sh0), 0.f)).x;
          b1[e] = (short)from_f<T>(fmaxf(fmaf(to_f(T{(uint16_t)b1[e]}), b_sc1, b_sh1), 0.f)).x;
        }
        dw[0][0] = mma<T>(a0, b0, dw[0][0]);
        dw[0][1] = mma<T>(a0, b1, dw[0][1]);
        dw[1][0] = mma<T>(a1, b0, dw[1][0]);
        dw[1][1] = mma<T>(a1, b1, dw[1][1]);
      }
      // GEMM 1 epilogue: bn2's ReLU mask, rounded gradient out, bn2 backward sums
      const int lm = 32 * mh + pl;
      const int64_t row = (int64_t)t * TM + lm;
      if (row < p.m) {
        // two separate 8-element arrays: pointer casts into one 16-element array kept it (and the
        // gradient row) in scratch, 80 B per lane (profiles/r06/scratch_census_r06s.md)
        float ylo[8], yhi[8], glo[8], ghi[8];
        Vec8<T>::load(ylo, reinterpret_cast<const T*>(yy + lm * C::YS + c0));
        Vec8<T>::load(yhi, reinterpret_cast<const T*>(yy + lm * C::YS + c0 + 8));
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float yv = r < 8 ? ylo[r & 7] : yhi[r & 7];
          const float gq = fmaf(yv, ec[c0 + r], ec[W + c0 + r]) > 0.f ? to_f(from_f<T>(acc[r])) : 0.f;
          if (r < 8) glo[r & 7] = gq;
          else ghi[r & 7] = gq;
          s1[r] += gq;
          s2[r] = fmaf(gq, yv - ec[2 * W + c0 + r], s2[r]);
        }
        T* dst = reinterpret_cast<T*>(p.dz2 + row * W + c0);
        Vec8<T>::store(dst, glo);
        Vec8<T>::store(dst + 8, ghi);
      }
    }
    lds_barrier();
  }

  // bn2 partial row: lanes (wave, h) own channels 32 (wave & 1) + 16 h + r; sum over pixels
  // (the stages are free now: the fold reuses them)
  float* red = reinterpret_cast<float*>(lds);
  const int tid = threadIdx.x;
  for (int pass = 0; pass < 2; ++pass) {
    float* rrow = red + (wave * 64 + lane) * 17;
#pragma unroll
    for (int r = 0; r < 16; ++r) rrow[r] = pass == 0 ? s1[r] : s2[r];
    __syncthreads();
    if (tid < W) {
      const int c = tid, t2 = c >> 5, hh = (c >> 4) & 1, r = c & 15;
      float a = 0.f;
      for (int w2 = t2; w2 < 4; w2 += 2)
        for (int l = 0; l < 32; ++l) a += red[(w2 * 64 + 32 * hh + l) * 17 + r];
      p.part2[((size_t)pass * gridDim.x + blockIdx.x) * W + c] = a;
    }
    __syncthreads();
  }
  // dW3 partial [C4][W]: C layout of GEMM 2 — rows k4 = 64 wave + 32 i + crow(r, h), column c = 32 j + pl
  float* ws = p.ws + (size_t)blockIdx.x * C4 * W;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int r = 0; r < 16; ++r) ws[(size_t)(64 * wave + 32 * i + crow(r, h)) * W + 32 * jj + pl] = dw[i][jj][r];
}

// out[n] = sum over the G slabs (fixed order): 8 consecutive outputs per lane, the slabs split
// over 16 lane groups of the block (G / 16 loads each), then a fixed-order LDS sum of the groups
template <typename TO>
__global__ void __launch_bounds__(256) reduce_kernel(const float* __restrict__ ws, int g, int64_t n,
                                                     TO* __restrict__ out) {
  __shared__ float red[16][16 * 8 + 4];
  const int v = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t i = ((int64_t)blockIdx.x * 16 + v) * 8;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < n)
    for (int q = grp; q < g; q += 16) {
      float t[8];
      Vec8<float>::load(t, ws + (int64_t)q * n + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += t[j];
    }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[grp][v * 8 + j] = a[j];
  __syncthreads();
  if (grp != 0 || i >= n) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.f;
  for (int g2 = 0; g2 < 16; ++g2)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += red[g2][v * 8 + j];
  Vec8<TO>::store(out + i, a);
}

}  // namespace c3b

bool conv3_bwd_fused_supported(int c4, int w) { return c4 == 256 && w == 64; }
int conv3_bwd_fused_parts(int cus) { return cus; }

void conv3_bwd_fused(const void* dm, const void* y3, const void* y2, const void* w3, const float* cb3, const float* c2,
                     const float* mean2, void* dz2, float* part2, float* ws, void* dw3, int dw_t, int64_t m, int c4,
                     int w, int t, int cus, hipStream_t s) {
  if (!conv3_bwd_fused_supported(c4, w)) throw std::runtime_error("conv3_bwd_fused: supported for C4 = 256, W = 64");
  if (m <= 0 || m * c4 >= (1ll << 40)) throw std::runtime_error("conv3_bwd_fused: bad pixel count");
  c3b::Args a;
  a.dm = (const uint16_t*)dm;
  a.y3 = (const uint16_t*)y3;
  a.y2 = (const uint16_t*)y2;
  a.w3 = (const uint16_t*)w3;
  a.cb3 = cb3;
  a.c2 = c2;
  a.mean2 = mean2;
  a.dz2 = (uint16_t*)dz2;
  a.part2 = part2;
  a.ws = ws;
  a.m = m;
  a.ntiles = (int)((m + c3b::TM - 1) / c3b::TM);
  const int G = conv3_bwd_fused_parts(cus);
  using C = c3b::Cfg<256, 64>;
  dispatch_16(t, [&](auto tag) {
    using T = typename decltype(tag)::type;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&c3b::fused_kernel<T, 256, 64>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
      attr = true;
    }
    hipLaunchKernelGGL((c3b::fused_kernel<T, 256, 64>), dim3(G), dim3(512), C::LDS, s, a);
  }, "conv3_bwd_fused");
  const int64_t n = (int64_t)c4 * w;
  dispatch_float(dw_t, [&](auto tag) {
    using TO = typename decltype(tag)::type;
    hipLaunchKernelGGL((c3b::reduce_kernel<TO>), dim3((unsigned)((n / 8 + 15) / 16)), dim3(256), 0, s, ws, G, n,
                       (TO*)dw3);
  }, "conv3_bwd_fused reduce");
  check_launch("conv3_bwd_fused");
}

}  // namespace apex_amd
