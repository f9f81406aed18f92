// gfx950 MFMA GEMM with fused bias / activation / activation-gradient epilogues.
//
// Reference: csrc/fused_dense_cuda.cu (cuBLASLt epilogues BIAS / GELU_AUX_BIAS / DGELU / BGRADB;
// on ROCm the reference falls back to rocBLAS + a bias copy, never computes d_bias and returns
// status 1 for the GeLU variants — :64-68, :1290, :1361-1495) and csrc/mlp_cuda.cu (rocBLAS GEMM
// + separate bias/activation kernels, :528-1041).
//
// Kernel (one launch per GEMM):
//  * 128 x 128 output tile per 256-thread workgroup (4 wave64s in 2 x 2, each 64 x 64 as 2 x 2
//    v_mfma_f32_32x32x16 tiles -> 64 fp32 accumulators per lane), BK = 64.
//  * global -> registers -> LDS staging, double-buffered: the next K-tile's 16-byte loads are
//    issued before the current tile's MFMAs and written to the other LDS buffer after them
//    (issue-early / write-late), one barrier per K-tile.
//  * k-major operands: LDS rows padded to 144 B (row r starts at 16-B slot 9r mod 16) so the
//    ds_read_b128 fragment reads of 16 different rows hit 16 different slots (conflict-free).
//    m/n-major operands keep the global [k][row] image with 320-B rows (4 consecutive k-rows
//    start 64 B apart) and are read with ds_read_b64_tr_b16 (hardware transpose), two reads per
//    8-deep k fragment.
//  * epilogue through LDS: fp32 accumulators are parked in a [128][132] fp32 tile, then every
//    thread applies bias / activation / activation-gradient on 8 consecutive columns and writes
//    16-byte vectors (and the 16-byte aux pre-activation for GeLU).
//  * XCD-aware tile order: consecutive workgroups are dealt round-robin over the 8 XCDs, so the
//    tile id is remapped to give every XCD a contiguous band of tiles (L2 reuse of A / B panels).
#include <cstdlib>

#include "apex_amd/colreduce.h"
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/gemm_api.h"

#include <algorithm>
#include "apex_amd/launch_plan.h"

namespace apex_amd {
namespace gemm {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int KSTR = BK + 8;    // k-major LDS row stride (elements) -> 144 B
constexpr int MSTR = 128 + 32;  // m/n-major LDS row stride (elements) -> 320 B
constexpr int CSTR = BN + 4;    // epilogue fp32 tile row stride (floats) -> 528 B

template <bool KMAJ>
constexpr int tile_elems() { return KMAJ ? BM * KSTR : BK * MSTR; }

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct Stage {
  uint4 r[4];
};

// ---- global -> registers (16 B per load, zero fill outside the matrix) ----
template <bool KMAJ>
__device__ __forceinline__ void stage_load(Stage& s, const uint16_t* __restrict__ base, int64_t ld, int rows_total,
                                           int k_total, int row0, int k0, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bool ok;
    const uint16_t* p;
    if constexpr (KMAJ) {
      const int row = (tid >> 3) + 32 * i, ch = tid & 7;
      const int gr = row0 + row, gk = k0 + ch * 8;
      ok = gr < rows_total && gk < k_total;
      p = base + (int64_t)gr * ld + gk;
    } else {
      const int kr = (tid >> 4) + 16 * i, ch = tid & 15;
      const int gk = k0 + kr, gc = row0 + ch * 8;
      ok = gk < k_total && gc < rows_total;
      p = base + (int64_t)gk * ld + gc;
    }
    s.r[i] = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
  }
}

// ---- registers -> LDS ----
template <bool KMAJ>
__device__ __forceinline__ void stage_store(const Stage& s, uint16_t* lds, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (KMAJ) {
      const int row = (tid >> 3) + 32 * i, ch = tid & 7;
      *reinterpret_cast<uint4*>(lds + row * KSTR + ch * 8) = s.r[i];
    } else {
      const int kr = (tid >> 4) + 16 * i, ch = tid & 15;
      *reinterpret_cast<uint4*>(lds + kr * MSTR + ch * 8) = s.r[i];
    }
  }
}

__device__ __forceinline__ s16x4 tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)((__attribute__((address_space(3))) uint16_t*)p));
}

// fragment of a 32-row subtile at k-step kk (16 deep): lane l gets rows rowbase + (l & 31),
// k = 16 kk + 8 (l >> 5) + j, j = 0..7 (the v_mfma_f32_32x32x16 A/B operand map)
template <bool KMAJ>
__device__ __forceinline__ s16x8 frag(const uint16_t* lds, int rowbase, int kk, int lane) {
  if constexpr (KMAJ) {
    const int row = rowbase + (lane & 31);
    const int k = kk * 16 + 8 * (lane >> 5);
    return *reinterpret_cast<const s16x8*>(lds + row * KSTR + k);
  } else {
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int rb = rowbase + 16 * (g & 1), kb = kk * 16 + 8 * (g >> 1);
    const uint16_t* a0 = lds + (kb + q) * MSTR + rb + 4 * p;
    const s16x4 lo = tr_read(a0);
    const s16x4 hi = tr_read(a0 + 4 * MSTR);
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
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

// tanh-GeLU as x * sigmoid(2u), u = k0 (x + k1 x^3): one v_exp_f32 + one v_rcp_f32 instead of a
// libm tanhf in the epilogue
__device__ __forceinline__ float gelu_sig(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return __builtin_amdgcn_rcpf(1.f + __expf(-2.f * k0 * (x + k1 * x * x * x)));
}
__device__ __forceinline__ float gelu_tanh(float x) { return x * gelu_sig(x); }
__device__ __forceinline__ float dgelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float s = gelu_sig(x);  // (1 + tanh u) / 2;  1 - tanh^2 u = 4 s (1 - s)
  return s + 2.f * x * s * (1.f - s) * k0 * (1.f + 3.f * k1 * x * x);
}

// XCD-aware, bijective remap of the linear workgroup id, then GROUP_M-grouped tile order
__device__ __forceinline__ void tile_coords(int nwg, int tiles_m, int tiles_n, int& bm, int& bn) {
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  constexpr int GROUP_M = 8;
  const int group = wgid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gm = min(tiles_m - first_m, GROUP_M);
  bm = first_m + (wgid % (GROUP_M * tiles_n)) % gm;
  bn = (wgid % (GROUP_M * tiles_n)) / gm;
}

template <typename T, bool AK, bool BKM, int EPI>
__global__ void __launch_bounds__(256, 2)
gemm_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, T* __restrict__ C, int64_t lda,
            int64_t ldb, int64_t ldc, int M, int N, int K, const T* __restrict__ bias, const T* __restrict__ aux_in,
            T* __restrict__ aux_out) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  constexpr int TA = tile_elems<AK>(), TB = tile_elems<BKM>();
  // buffer b: A tile at b*(TA+TB), B tile right after it
  auto a_buf = [&](int b) { return lds + b * (TA + TB); };
  auto b_buf = [&](int b) { return lds + b * (TA + TB) + TA; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  int bm, bn;
  tile_coords(tiles_m * tiles_n, tiles_m, tiles_n, bm, bn);
  const int row0 = bm * BM, col0 = bn * BN;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  Stage sa, sb;
  stage_load<AK>(sa, A, lda, M, K, row0, 0, tid);
  stage_load<BKM>(sb, B, ldb, N, K, col0, 0, tid);
  stage_store<AK>(sa, a_buf(0), tid);
  stage_store<BKM>(sb, b_buf(0), tid);
  __syncthreads();

  const int nk = (K + BK - 1) / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      stage_load<AK>(sa, A, lda, M, K, row0, (kt + 1) * BK, tid);
      stage_load<BKM>(sb, B, ldb, N, K, col0, (kt + 1) * BK, tid);
    }
    const uint16_t* a_t = a_buf(cur);
    const uint16_t* b_t = b_buf(cur);
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const s16x8 a0 = frag<AK>(a_t, wm * 64, kk, lane);
      const s16x8 a1 = frag<AK>(a_t, wm * 64 + 32, kk, lane);
      const s16x8 b0 = frag<BKM>(b_t, wn * 64, kk, lane);
      const s16x8 b1 = frag<BKM>(b_t, wn * 64 + 32, kk, lane);
      acc[0][0] = mfma<T>(a0, b0, acc[0][0]);
      acc[0][1] = mfma<T>(a0, b1, acc[0][1]);
      acc[1][0] = mfma<T>(a1, b0, acc[1][0]);
      acc[1][1] = mfma<T>(a1, b1, acc[1][1]);
    }
    if (more) {
      stage_store<AK>(sa, a_buf(cur ^ 1), tid);
      stage_store<BKM>(sb, b_buf(cur ^ 1), tid);
    }
    __syncthreads();
  }

  // ---- epilogue: park fp32 accumulators in LDS, then 16-byte row-vector stores ----
  float* cs = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int cl = wn * 64 + j * 32 + (lane & 31);
        cs[rl * CSTR + cl] = acc[i][j][r];
      }
  __syncthreads();
  const int ch = tid & 15;
  const int gc = col0 + ch * 8;
  if (gc >= N) return;
  float bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = 0.f;
  if (bias != nullptr) Vec8<T>::load(bv, bias + gc);
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int rl = (tid >> 4) + 16 * it;
    const int gr = row0 + rl;
    if (gr >= M) break;
    float v[8];
    const float4 lo = *reinterpret_cast<const float4*>(cs + rl * CSTR + ch * 8);
    const float4 hi = *reinterpret_cast<const float4*>(cs + rl * CSTR + ch * 8 + 4);
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    const int64_t off = (int64_t)gr * ldc + gc;
    if constexpr (EPI == kEpiNone) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bv[e];
    } else if constexpr (EPI == kEpiGelu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bv[e];
      if (aux_out != nullptr) Vec8<T>::store(aux_out + off, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
    } else if constexpr (EPI == kEpiRelu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] + bv[e], 0.f);
    } else if constexpr (EPI == kEpiSigmoid) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 1.f / (1.f + __expf(-(v[e] + bv[e])));
    } else {
      float a[8];
      Vec8<T>::load(a, aux_in + off);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if constexpr (EPI == kEpiDGelu) v[e] *= dgelu_tanh(a[e]);
        else if constexpr (EPI == kEpiDRelu) v[e] = a[e] > 0.f ? v[e] : 0.f;
        else v[e] *= a[e] * (1.f - a[e]);
      }
    }
    Vec8<T>::store(C + off, v);
  }
}

// ---- column sums (bias gradients): partial [P][N] then fixed-order finalize ----
template <typename T>
__global__ void __launch_bounds__(256) colsum_partial(const T* __restrict__ x, int64_t m, int n, int64_t ldx,
                                                      float* __restrict__ part) {
  // block = 32 column-vectors (8 columns each) x 8 row groups
  const int cv = blockIdx.x * 32 + (threadIdx.x & 31);
  const int rg = threadIdx.x >> 5;
  const int c0 = cv * 8;
  __shared__ float red[8][32 * 8];
  float s[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = 0.f;
  if (c0 < n) {
    for (int64_t r = (int64_t)blockIdx.y * 8 + rg; r < m; r += (int64_t)gridDim.y * 8) {
      float v[8];
      Vec8<T>::load(v, x + r * ldx + c0);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rg][(threadIdx.x & 31) * 8 + e] = s[e];
  __syncthreads();
  if (rg == 0 && c0 < n) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = 0.f;
      for (int g = 0; g < 8; ++g) t += red[g][(threadIdx.x & 31) * 8 + e];
      part[(int64_t)blockIdx.y * n + c0 + e] = t;
    }
  }
}

// dz = dy * gelu'(aux) written out and its column sums in the same pass (the dGeLU + bias-grad
// of a dense layer whose GEMM ran on the library: cuBLASLt's DGELU_BGRAD capability,
// reference csrc/fused_dense_cuda.cu:977, for the bf16 case hipBLASLt has no working kernel for).
// Block layout as colsum_partial; two rows in flight per lane.  The sums are of the ROUNDED dz
// (what the unfused dz.sum(0) would add).
template <typename T>
__global__ void __launch_bounds__(256) dgelu_colsum_partial(const T* __restrict__ dy, const T* __restrict__ aux,
                                                            T* __restrict__ dz, int64_t m, int n,
                                                            float* __restrict__ part) {
  const int cv = blockIdx.x * 32 + (threadIdx.x & 31);
  const int rg = threadIdx.x >> 5;
  const int c0 = cv * 8;
  __shared__ float red[8][32 * 8];
  float s[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = 0.f;
  if (c0 < n) {
    const int64_t step = (int64_t)gridDim.y * 8;
    for (int64_t r = (int64_t)blockIdx.y * 8 + rg; r < m; r += 2 * step) {
      const int64_t r1 = r + step;
      const bool two = r1 < m;
      float g0[8], a0[8], g1[8], a1[8];
      Vec8<T>::load(g0, dy + r * n + c0);
      Vec8<T>::load(a0, aux + r * n + c0);
      if (two) {
        Vec8<T>::load(g1, dy + r1 * n + c0);
        Vec8<T>::load(a1, aux + r1 * n + c0);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) g0[e] = to_f(from_f<T>(g0[e] * dgelu_tanh(a0[e])));
      Vec8<T>::store(dz + r * n + c0, g0);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += g0[e];
      if (two) {
#pragma unroll
        for (int e = 0; e < 8; ++e) g1[e] = to_f(from_f<T>(g1[e] * dgelu_tanh(a1[e])));
        Vec8<T>::store(dz + r1 * n + c0, g1);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += g1[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rg][(threadIdx.x & 31) * 8 + e] = s[e];
  __syncthreads();
  if (rg == 0 && c0 < n) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = 0.f;
      for (int g = 0; g < 8; ++g) t += red[g][(threadIdx.x & 31) * 8 + e];
      part[(int64_t)blockIdx.y * n + c0 + e] = t;
    }
  }
}

// y = gelu_tanh(z), 8 elements per lane per iteration (one 16-byte load + store), grid-stride:
// the activation pass after a library GEMM whose bias epilogue wrote the pre-activation z (kept
// as the backward's aux) — gfx950 bf16 hipBLASLt has no GELU_AUX_BIAS kernel
template <typename T>
__global__ void __launch_bounds__(256) gelu_fwd_kernel(const T* __restrict__ z, T* __restrict__ y, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    Vec8<T>::load(v, z + i * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
    Vec8<T>::store(y + i * 8, v);
  }
}

template <typename TO>
__global__ void __launch_bounds__(256) colsum_finalize(const float* __restrict__ part, int p, int n,
                                                       TO* __restrict__ out) {
  __shared__ float red[16][17];
  const float v = colreduce16(part, p, n, red);
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  if ((threadIdx.x >> 4) == 0 && c < n) out[c] = from_f<TO>(v);
}

inline int colsum_parts(int64_t m, int n, int cus) { return plan::colsum_parts(m, n, cus); }

template <typename T, bool AK, bool BKM>
void launch_epi(const GemmArgs& g, hipStream_t s) {
  const int tiles = ((g.m + BM - 1) / BM) * ((g.n + BN - 1) / BN);
  const size_t op_bytes = (size_t)2 * (tile_elems<AK>() + tile_elems<BKM>()) * sizeof(uint16_t);
  const size_t epi_bytes = (size_t)BM * CSTR * sizeof(float);
  const size_t lds = op_bytes > epi_bytes ? op_bytes : epi_bytes;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(256), lds, s, (const uint16_t*)g.a, (const uint16_t*)g.b, (T*)g.c,
                       g.lda, g.ldb, g.ldc, g.m, g.n, g.k, (const T*)g.bias, (const T*)g.aux_in, (T*)g.aux_out);
  };
  switch (g.epilogue) {
    case kEpiNone: go(gemm_kernel<T, AK, BKM, kEpiNone>); break;
    case kEpiGelu: go(gemm_kernel<T, AK, BKM, kEpiGelu>); break;
    case kEpiRelu: go(gemm_kernel<T, AK, BKM, kEpiRelu>); break;
    case kEpiSigmoid: go(gemm_kernel<T, AK, BKM, kEpiSigmoid>); break;
    case kEpiDGelu: go(gemm_kernel<T, AK, BKM, kEpiDGelu>); break;
    case kEpiDRelu: go(gemm_kernel<T, AK, BKM, kEpiDRelu>); break;
    case kEpiDSigmoid: go(gemm_kernel<T, AK, BKM, kEpiDSigmoid>); break;
    default: throw std::runtime_error("gemm: unknown epilogue");
  }
}


// =============================================================================================
// 256 x 256 x 64 tile (all four operand-major combinations), 8 waves (2 x 4), each wave
// 128 x 64 = 4 x 2 v_mfma_f32_32x32x16 tiles (128 accumulator registers).  Operands move
// global -> LDS by LDS-DMA (global_load_lds_dwordx4: no staging registers, no ds_write pass),
// 2 LDS buffers x (A 32 KB + B 32 KB), the next K-tile's DMA in flight under the current tile's
// 32 MFMAs per wave, one barrier per K-tile.  The LDS image is lane-linear per DMA instruction
// (1 KB = 8 rows of 128 B), so the bank swizzle is applied on the SOURCE address: 16-byte chunk
// c of row r is stored at chunk c ^ ((r >> 1) & 7), which makes the 16 rows read by each
// 16-lane group of a ds_read_b128 fragment load hit 16 distinct 16-byte slots.
// Epilogue: accumulators staged through LDS as fp32 in two 128-row halves, then 16-byte
// row-vector stores with the same bias / activation / derivative epilogues as above.
// =============================================================================================
namespace g256 {

constexpr int BM = plan::kGemmBM, BN = plan::kGemmBN, BK = plan::kGemmBK;
constexpr int TILE = BM * BK;          // elements per operand tile (32 KB)
constexpr int CST = BN + 4;            // epilogue fp32 row stride
constexpr size_t LDS_BYTES = (size_t)128 * CST * 4 > (size_t)4 * TILE * 2 ? (size_t)128 * CST * 4 : (size_t)4 * TILE * 2;

__device__ __forceinline__ void dma16(const uint16_t* src, uint16_t* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// Issue this wave's 4 DMA pieces for one operand tile.
// k-major operand (rows = M/N, k contiguous): image [256][64], 1-KB piece = 8 rows of 128 B,
//   chunk c of row r at c ^ ((r >> 1) & 7)  (row-fragment ds_read_b128, 16 rows -> 16 slots).
// m-major operand (k rows, M/N contiguous): image [64][256], 1-KB piece = 2 k-rows of 512 B,
//   chunk c of k-row r at c ^ ((r & 3) << 1) (transposed ds_read_b64_tr_b16: the 4 k-rows a
//   16-lane group reads start 32 B apart -> conflict-free).
template <bool KMAJ, int NW = 8>
__device__ __forceinline__ void issue_tile(const uint16_t* __restrict__ X, int64_t ld, int rows, int r0, int k0,
                                           uint16_t* dst, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 32 / NW; ++i) {
    const int j = i * NW + wave;
    if constexpr (KMAJ) {
      const int row = 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int gr = r0 + row;
      gr = gr < rows ? gr : rows - 1;  // rows past the edge are computed but never stored
      dma16(X + (int64_t)gr * ld + k0 + 8 * c, dst + j * 512);
    } else {
      const int krow = 2 * j + (lane >> 5);
      const int c = (lane & 31) ^ ((krow & 3) << 1);
      int col = r0 + 8 * c;
      col = col <= rows - 8 ? col : rows - 8;  // rows % 8 == 0 for m-major operands
      dma16(X + (int64_t)(k0 + krow) * ld + col, dst + j * 512);
    }
  }
}

template <bool KMAJ>
__device__ __forceinline__ s16x8 frag_sw(const uint16_t* tile, int rowbase, int kk, int lane) {
  if constexpr (KMAJ) {
    const int row = rowbase + (lane & 31);
    const int c = (2 * kk + (lane >> 5)) ^ ((row >> 1) & 7);
    return *reinterpret_cast<const s16x8*>(tile + row * BK + 8 * c);
  } else {
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int kb = 16 * kk + 8 * (g >> 1);
    const int col = rowbase + 16 * (g & 1) + 4 * p;
    const int ck = col >> 3, off = col & 7;
    const int r0 = kb + q, r1 = kb + 4 + q;
    const s16x4 lo = tr_read(tile + r0 * 256 + ((ck ^ ((r0 & 3) << 1)) << 3) + off);
    const s16x4 hi = tr_read(tile + r1 * 256 + ((ck ^ ((r1 & 3) << 1)) << 3) + off);
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

// NW = 8: 2 x 4 waves of 128 x 64 (two waves per SIMD hide each other's LDS latency);
// NW = 4: 2 x 2 waves of 128 x 128 (one wave per SIMD, 256 fp32 accumulators each, half the
// LDS fragment traffic per MFMA: every A/B fragment read feeds 4 MFMAs instead of 2 / 4).
template <typename T, bool AK, bool BKM, int EPI, int NW>
__global__ void __launch_bounds__(NW * 64, 1)
gemm256_nt(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, T* __restrict__ C, int64_t lda,
           int64_t ldb, int64_t ldc, int M, int N, int K, const T* __restrict__ bias, const T* __restrict__ aux_in,
           T* __restrict__ aux_out, float* __restrict__ part, int kchunk, float* __restrict__ colpart) {
  constexpr int WN = NW / 2;           // waves along N
  constexpr int NJ = BN / WN / 32;     // 32-wide column fragments per wave (2 or 4)
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  auto a_buf = [&](int b) { return lds + b * 2 * TILE; };
  auto b_buf = [&](int b) { return lds + b * 2 * TILE + TILE; };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  int bm, bn;
  tile_coords(tiles_m * tiles_n, tiles_m, tiles_n, bm, bn);
  const int row0 = bm * BM, col0 = bn * BN;

  f32x16 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // split-K (part != null): blockIdx.y picks the K chunk, the epilogue stores an fp32 partial
  const int kbeg = (int)blockIdx.y * kchunk;
  const int nk = (min(K, kbeg + kchunk) - kbeg) / BK;
  issue_tile<AK, NW>(A, lda, M, row0, kbeg, a_buf(0), wave, lane);
  issue_tile<BKM, NW>(B, ldb, N, col0, kbeg, b_buf(0), wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      issue_tile<AK, NW>(A, lda, M, row0, kbeg + (kt + 1) * BK, a_buf(cur ^ 1), wave, lane);
      issue_tile<BKM, NW>(B, ldb, N, col0, kbeg + (kt + 1) * BK, b_buf(cur ^ 1), wave, lane);
    }
    const uint16_t* at = a_buf(cur);
    const uint16_t* bt = b_buf(cur);
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      s16x8 af[4], bf[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag_sw<AK>(at, wm * 128 + 32 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bf[j] = frag_sw<BKM>(bt, wn * (32 * NJ) + 32 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma<T>(af[i], bf[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  float* cs = reinterpret_cast<float*>(lds);
  const int ch = tid & 31, rsub = tid >> 5;  // rsub in [0, NT / 32)
  const int gc = col0 + ch * 8;
  float bv[8], csum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = csum[e] = 0.f;
  if (bias != nullptr && gc < N) Vec8<T>::load(bv, bias + gc);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    // activation-gradient epilogues: this half's aux_in rows are fetched before the LDS staging
    // (clamped addresses, no per-row branch) so their HBM latency overlaps it instead of
    // serializing one row load per pass
    constexpr int IT = 128 / (NT / 32);
    uint4 apre[EPI >= kEpiDGelu ? IT : 1];
    if constexpr (EPI >= kEpiDGelu) {
      const int gcc = gc < N ? gc : N - 8;
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        int gr = row0 + half * 128 + rsub + (NT / 32) * it;
        gr = gr < M ? gr : M - 1;
        apre[it] = *reinterpret_cast<const uint4*>(aux_in + (int64_t)gr * ldc + gcc);
      }
    }
    if (wm == half) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rl = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            cs[rl * CST + wn * (32 * NJ) + 32 * j + (lane & 31)] = acc[i][j][r];
          }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 128 / (NT / 32); ++it) {
      const int rl = rsub + (NT / 32) * it;
      const int gr = row0 + half * 128 + rl;
      if (gr < M && gc < N) {
        float v[8];
        const float4 lo = *reinterpret_cast<const float4*>(cs + rl * CST + ch * 8);
        const float4 hi = *reinterpret_cast<const float4*>(cs + rl * CST + ch * 8 + 4);
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        const int64_t off = (int64_t)gr * ldc + gc;
        if (EPI == kEpiNone && part != nullptr) {
          float* dst = part + ((int64_t)blockIdx.y * M + gr) * N + gc;
          *reinterpret_cast<float4*>(dst) = lo;
          *reinterpret_cast<float4*>(dst + 4) = hi;
          continue;
        }
        if constexpr (EPI == kEpiNone) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += bv[e];
        } else if constexpr (EPI == kEpiGelu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += bv[e];
          if (aux_out != nullptr) Vec8<T>::store(aux_out + off, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
        } else if constexpr (EPI == kEpiRelu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] + bv[e], 0.f);
        } else if constexpr (EPI == kEpiSigmoid) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = 1.f / (1.f + __expf(-(v[e] + bv[e])));
        } else {
          float a[8];
          Vec8<T>::load(a, reinterpret_cast<const T*>(&apre[it]));
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            if constexpr (EPI == kEpiDGelu) v[e] *= dgelu_tanh(a[e]);
            else if constexpr (EPI == kEpiDRelu) v[e] = a[e] > 0.f ? v[e] : 0.f;
            else v[e] *= a[e] * (1.f - a[e]);
          }
        }
        Vec8<T>::store(C + off, v);
        if (colpart != nullptr) {
          // column sums of the STORED (rounded) values: the bias gradient of this GEMM's output,
          // as the reference's DGELU_BGRAD epilogue (csrc/fused_dense_cuda.cu:977)
#pragma unroll
          for (int e = 0; e < 8; ++e) csum[e] += to_f(from_f<T>(v[e]));
        }
      }
    }
    __syncthreads();
  }
  if (colpart != nullptr) {
    // fold the NT / 32 row groups of each column (fixed order), one fp32 partial per (M tile, column)
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[rsub * BN + ch * 8 + e] = csum[e];
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < NT / 32; ++r) t += cs[r * BN + c];
      if (col0 + c < N) colpart[(int64_t)bm * N + col0 + c] = t;
    }
  }
}

// sum of the split-K fp32 partials [S][M][N] (+ bias) -> C, 8 consecutive columns per thread
template <typename T>
__global__ void __launch_bounds__(256) splitk_reduce(const float* __restrict__ part, int S, int M, int N,
                                                     const T* __restrict__ bias, T* __restrict__ C, int64_t ldc) {
  const int64_t nvec = (int64_t)M * N / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * 8;
    const int r = (int)(e / N), c = (int)(e % N);
    float v[8], t[8];
    Vec8<float>::load(v, part + e);
    for (int s = 1; s < S; ++s) {
      Vec8<float>::load(t, part + (int64_t)s * M * N + e);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += t[k];
    }
    if (bias != nullptr) {
      Vec8<T>::load(t, bias + c);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += t[k];
    }
    Vec8<T>::store(C + (int64_t)r * ldc + c, v);
  }
}

inline int splitk_parts(const GemmArgs& g, int cus, int* kchunk) { return plan::gemm_splitk_parts(g, cus, kchunk); }

// waves per 256 x 256 tile: 8 (default) or 4 (APEX_AMD_GEMM256_WAVES=4, A/B)
inline int waves_cfg() {
  const char* e = std::getenv("APEX_AMD_GEMM256_WAVES");
  return (e != nullptr && e[0] == '4') ? 4 : 8;
}

template <typename T, bool AK, bool BKM, int NW>
void launch_nw(const GemmArgs& g, hipStream_t s, int cus);

template <typename T, bool AK, bool BKM>
void launch(const GemmArgs& g, hipStream_t s, int cus) {
  if (waves_cfg() == 4) launch_nw<T, AK, BKM, 4>(g, s, cus);
  else launch_nw<T, AK, BKM, 8>(g, s, cus);
}

template <typename T, bool AK, bool BKM, int NW>
void launch_nw(const GemmArgs& g, hipStream_t s, int cus) {
  const int tiles = ((g.m + BM - 1) / BM) * ((g.n + BN - 1) / BN);
  constexpr int THREADS = NW * 64;
  int kchunk = g.k;
  const int sp = g.splitk_ws != nullptr ? splitk_parts(g, cus, &kchunk) : 1;
  if (sp > 1) {
    hipLaunchKernelGGL((gemm256_nt<T, AK, BKM, kEpiNone, NW>), dim3(tiles, sp), dim3(THREADS), LDS_BYTES, s,
                       (const uint16_t*)g.a, (const uint16_t*)g.b, (T*)g.c, g.lda, g.ldb, g.ldc, g.m, g.n, g.k,
                       (const T*)nullptr, (const T*)nullptr, (T*)nullptr, g.splitk_ws, kchunk, (float*)nullptr);
    const int64_t nvec = (int64_t)g.m * g.n / 8;
    int64_t grid = (nvec + 255) / 256;
    if (grid > (int64_t)cus * 8) grid = (int64_t)cus * 8;
    hipLaunchKernelGGL((splitk_reduce<T>), dim3((unsigned)grid), dim3(256), 0, s, (const float*)g.splitk_ws, sp, g.m,
                       g.n, (const T*)g.bias, (T*)g.c, g.ldc);
    return;
  }
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(THREADS), LDS_BYTES, s, (const uint16_t*)g.a, (const uint16_t*)g.b,
                       (T*)g.c, g.lda, g.ldb, g.ldc, g.m, g.n, g.k, (const T*)g.bias, (const T*)g.aux_in,
                       (T*)g.aux_out, (float*)nullptr, g.k, g.colpart);
  };
  switch (g.epilogue) {
    case kEpiNone: go(gemm256_nt<T, AK, BKM, kEpiNone, NW>); break;
    case kEpiGelu: go(gemm256_nt<T, AK, BKM, kEpiGelu, NW>); break;
    case kEpiRelu: go(gemm256_nt<T, AK, BKM, kEpiRelu, NW>); break;
    case kEpiSigmoid: go(gemm256_nt<T, AK, BKM, kEpiSigmoid, NW>); break;
    case kEpiDGelu: go(gemm256_nt<T, AK, BKM, kEpiDGelu, NW>); break;
    case kEpiDRelu: go(gemm256_nt<T, AK, BKM, kEpiDRelu, NW>); break;
    case kEpiDSigmoid: go(gemm256_nt<T, AK, BKM, kEpiDSigmoid, NW>); break;
    default: throw std::runtime_error("gemm256: unknown epilogue");
  }
}

// the 256-tile kernel needs K % 64 == 0 and enough tiles to fill the chip.
// APEX_AMD_GEMM256=force|off overrides the size heuristic (tests / A-B timing).
inline bool usable(const GemmArgs& g, int cus) {
  if (g.k % BK) return false;
  const char* env = std::getenv("APEX_AMD_GEMM256");
  if (env != nullptr && env[0] == 'o') return false;
  if (env != nullptr && env[0] == 'f') return true;
  const int64_t tiles = (int64_t)((g.m + BM - 1) / BM) * ((g.n + BN - 1) / BN);
  int kc;
  return tiles >= cus / 2 || (g.splitk_ws != nullptr && splitk_parts(g, cus, &kc) > 1);
}

}  // namespace g256

// =============================================================================================
// g8p: 256 x 256 x 64 tile for two k-major operands, phase-pipelined ("ping-pong") main loop.
//
// 8 waves as 2 (M) x 4 (N), each a 128 x 64 block of 16x16 accumulators (v_mfma_f32_16x16x32).
// A K-tile is computed in 4 phases, one 64 x 32 output quadrant each (16 MFMAs):
//   phase 0: (rows 0-63,  cols 0-31)  reads A rows 0-63 (8 x ds_read_b128) + B cols 0-31 (4)
//   phase 1: (rows 0-63,  cols 32-63) reads B cols 32-63 (4)
//   phase 2: (rows 64-127, cols 32-63) reads A rows 64-127 (8)
//   phase 3: (rows 64-127, cols 0-31)  no reads (operands still in registers)
// so the tile is staged as four 16-KB "half-tiles" in the order the phases consume them:
//   h0 = A rows {0-63, 128-191}, h1 = B cols {0-31} of every wave column, h2 = B cols {32-63},
//   h3 = A rows {64-127, 192-255}
// and every phase issues ONE half-tile of LDS-DMA (2 global_load_lds_dwordx4 per lane) six
// half-tiles ahead, into a 2 x 4 ring (128 KB).  Each phase then waits with a counted
// vmcnt(8) — 4 half-tiles stay in flight across every barrier — and the data it retired is
// read one phase later at the earliest; a slot is refilled >= 2 phases after its last read.
// Measured (profiles/gemm8p_r02.jsonl): 1180 TF at 8192^3 vs 1085 for g256; moving the DMA
// issue into the MFMA block (1098 TF) or the next phase's ds_reads into it (984 TF) lost.
// The two wave rows run one barrier apart (group 1 takes an extra barrier up front): while
// one group's MFMAs run between its two barriers, the other group issues its ds_reads and
// DMA, so each SIMD (one wave of each group) alternates MFMA and load work.
// =============================================================================================
namespace g8p {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int HT = 128 * BK;  // elements per half-tile image (16 KB)
constexpr int CST = BN + 4;
constexpr size_t LDS_BYTES = (size_t)128 * CST * 4 > (size_t)8 * HT * 2 ? (size_t)128 * CST * 4 : (size_t)8 * HT * 2;

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ f32x4 mfma16(s16x8 a, s16x8 b, f32x4 c);
template <>
__device__ __forceinline__ f32x4 mfma16<bf16_t>(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma16<f16_t>(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// wait until at most n (wave-uniform, even, 0..8) of this wave's DMAs are outstanding
__device__ __forceinline__ void wait_vm(int n) {
  if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Issue this lane's 2 DMA pieces of half-tile h (0..3) of the K-tile at k0 into dst.
// Image: [128 rows][64 k], 128-B rows, 16-B chunk c of row r stored at c ^ ((r >> 1) & 7).
__device__ __forceinline__ void issue_half(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, int64_t lda,
                                           int64_t ldb, int M, int N, int row0, int col0, int k0, int h,
                                           uint16_t* dst, int wave, int lane) {
  const bool isA = (h == 0 || h == 3);
  const int s = (h == 0 || h == 1) ? 0 : 1;  // first / second half of the rows (A) or columns (B)
  const uint16_t* X = isA ? A : B;
  const int64_t ld = isA ? lda : ldb;
  const int lim = isA ? M : N;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = i * 8 + wave;
    const int r = 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int t = isA ? (r & 63) + (r >> 6) * 128 + s * 64 : (r >> 5) * 64 + (r & 31) + s * 32;
    int gr = (isA ? row0 : col0) + t;
    gr = gr < lim ? gr : lim - 1;  // rows past the edge are computed but never stored
    g256::dma16(X + (int64_t)gr * ld + k0 + 8 * c, dst + j * 512);
  }
}

// fragment (16 rows x 32 k) at image row rb, k-step kk of a swizzled half-tile image:
// lane l gets row rb + (l & 15), k = 32 kk + 8 (l >> 4) + e
__device__ __forceinline__ s16x8 frag16(const uint16_t* img, int rb, int kk, int lane) {
  const int r = rb + (lane & 15);
  const int c = (4 * kk + (lane >> 4)) ^ ((r >> 1) & 7);
  return *reinterpret_cast<const s16x8*>(img + r * BK + 8 * c);
}

template <typename T, int EPI>
__global__ void __launch_bounds__(512, 1)
gemm8p_nt(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, T* __restrict__ C, int64_t lda, int64_t ldb,
          int64_t ldc, int M, int N, int K, const T* __restrict__ bias, const T* __restrict__ aux_in,
          T* __restrict__ aux_out, float* __restrict__ part, int kchunk) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  int bm, bn;
  tile_coords(tiles_m * tiles_n, tiles_m, tiles_n, bm, bn);
  const int row0 = bm * BM, col0 = bn * BN;
  const int kbeg = (int)blockIdx.y * kchunk;
  const int nk = (min(K, kbeg + kchunk) - kbeg) / BK;
  const int nloads = 4 * nk;  // half-tile loads of this workgroup
  auto slot = [&](int load) { return lds + ((load >> 2) & 1) * 4 * HT + (load & 3) * HT; };
  auto issue = [&](int load) {
    issue_half(A, B, lda, ldb, M, N, row0, col0, kbeg + (load >> 2) * BK, load & 3, slot(load), wave, lane);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: loads 0..5 (K-tile 0 and the first two half-tiles of K-tile 1); retire 0 and 1
  const int pre = nloads < 6 ? nloads : 6;
  for (int l = 0; l < pre; ++l) issue(l);
  wait_vm(2 * (pre - 2));
  barrier();
  if (wr == 1) barrier();  // stagger the second wave row by one barrier

  s16x8 af[4][2], bf0[2][2], bf1[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    const uint16_t* tA0 = slot(4 * kt + 0);
    const uint16_t* tB0 = slot(4 * kt + 1);
    const uint16_t* tB1 = slot(4 * kt + 2);
    const uint16_t* tA1 = slot(4 * kt + 3);
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int p = 4 * kt + ph;
      // 1. this phase's operand fragments (they land while the other wave row runs its MFMAs)
      if (ph == 0) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) bf0[j][kk] = frag16(tB0, wc * 32 + 16 * j, kk, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) af[i][kk] = frag16(tA0, wr * 64 + 16 * i, kk, lane);
      } else if (ph == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) bf1[j][kk] = frag16(tB1, wc * 32 + 16 * j, kk, lane);
      } else if (ph == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) af[i][kk] = frag16(tA1, wr * 64 + 16 * i, kk, lane);
      }
      // 2. one half-tile of DMA six loads ahead; retire the load issued four phases ago
      const int l = p + 6;
      if (l < nloads) issue(l);
      const int last = (l < nloads ? l : nloads - 1);
      const int fly = last - (p + 2);
      wait_vm(fly > 0 ? 2 * fly : 0);
      barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // 3. 16 MFMAs of this phase's 64 x 32 quadrant
      __builtin_amdgcn_s_setprio(1);
      const int qm = (ph >= 2) ? 1 : 0;
      const int qn = (ph == 1 || ph == 2) ? 1 : 0;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const s16x8 b = qn ? bf1[j][kk] : bf0[j][kk];
            acc[4 * qm + i][2 * qn + j] = mfma16<T>(af[i][kk], b, acc[4 * qm + i][2 * qn + j]);
          }
      __builtin_amdgcn_s_setprio(0);
      barrier();
    }
  }
  if (wr == 0) barrier();  // re-align the two wave rows
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: two 128-row halves staged as fp32 through LDS, 16-byte row stores ----
  float* cs = reinterpret_cast<float*>(lds);
  const int ch = tid & 31, rsub = tid >> 5;  // 16 rows per pass
  const int gc = col0 + ch * 8;
  float bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = 0.f;
  if (bias != nullptr && gc < N) Vec8<T>::load(bv, bias + gc);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    uint4 apre[EPI >= kEpiDGelu ? 8 : 1];  // aux_in rows fetched ahead of the staging (see g256)
    if constexpr (EPI >= kEpiDGelu) {
      const int gcc = gc < N ? gc : N - 8;
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        int gr = row0 + half * 128 + rsub + 16 * it;
        gr = gr < M ? gr : M - 1;
        apre[it] = *reinterpret_cast<const uint4*>(aux_in + (int64_t)gr * ldc + gcc);
      }
    }
    if (wr == half) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            cs[(16 * i + 4 * (lane >> 4) + r) * CST + wc * 64 + 16 * j + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int rl = rsub + 16 * it;
      const int gr = row0 + half * 128 + rl;
      if (gr < M && gc < N) {
        float v[8];
        const float4 lo = *reinterpret_cast<const float4*>(cs + rl * CST + ch * 8);
        const float4 hi = *reinterpret_cast<const float4*>(cs + rl * CST + ch * 8 + 4);
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        const int64_t off = (int64_t)gr * ldc + gc;
        if (EPI == kEpiNone && part != nullptr) {
          float* dst = part + ((int64_t)blockIdx.y * M + gr) * N + gc;
          *reinterpret_cast<float4*>(dst) = lo;
          *reinterpret_cast<float4*>(dst + 4) = hi;
          continue;
        }
        if constexpr (EPI == kEpiNone) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += bv[e];
        } else if constexpr (EPI == kEpiGelu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += bv[e];
          if (aux_out != nullptr) Vec8<T>::store(aux_out + off, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
        } else if constexpr (EPI == kEpiRelu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] + bv[e], 0.f);
        } else if constexpr (EPI == kEpiSigmoid) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = 1.f / (1.f + __expf(-(v[e] + bv[e])));
        } else {
          float a[8];
          Vec8<T>::load(a, reinterpret_cast<const T*>(&apre[it]));
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            if constexpr (EPI == kEpiDGelu) v[e] *= dgelu_tanh(a[e]);
            else if constexpr (EPI == kEpiDRelu) v[e] = a[e] > 0.f ? v[e] : 0.f;
            else v[e] *= a[e] * (1.f - a[e]);
          }
        }
        Vec8<T>::store(C + off, v);
      }
    }
    __syncthreads();
  }
}

// APEX_AMD_GEMM8P=0 routes k-major x k-major GEMMs back to the g256 kernel (A/B timing)
inline bool enabled() {
  const char* e = std::getenv("APEX_AMD_GEMM8P");
  return e == nullptr || e[0] != '0';
}

template <typename T>
void launch(const GemmArgs& g, hipStream_t s, int cus) {
  const int tiles = ((g.m + BM - 1) / BM) * ((g.n + BN - 1) / BN);
  int kchunk = g.k;
  const int sp = g.splitk_ws != nullptr ? g256::splitk_parts(g, cus, &kchunk) : 1;
  if (sp > 1) {
    hipLaunchKernelGGL((gemm8p_nt<T, kEpiNone>), dim3(tiles, sp), dim3(512), LDS_BYTES, s, (const uint16_t*)g.a,
                       (const uint16_t*)g.b, (T*)g.c, g.lda, g.ldb, g.ldc, g.m, g.n, g.k, (const T*)nullptr,
                       (const T*)nullptr, (T*)nullptr, g.splitk_ws, kchunk);
    const int64_t nvec = (int64_t)g.m * g.n / 8;
    int64_t grid = (nvec + 255) / 256;
    if (grid > (int64_t)cus * 8) grid = (int64_t)cus * 8;
    hipLaunchKernelGGL((g256::splitk_reduce<T>), dim3((unsigned)grid), dim3(256), 0, s, (const float*)g.splitk_ws, sp,
                       g.m, g.n, (const T*)g.bias, (T*)g.c, g.ldc);
    return;
  }
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(512), LDS_BYTES, s, (const uint16_t*)g.a, (const uint16_t*)g.b,
                       (T*)g.c, g.lda, g.ldb, g.ldc, g.m, g.n, g.k, (const T*)g.bias, (const T*)g.aux_in,
                       (T*)g.aux_out, (float*)nullptr, g.k);
  };
  switch (g.epilogue) {
    case kEpiNone: go(gemm8p_nt<T, kEpiNone>); break;
    case kEpiGelu: go(gemm8p_nt<T, kEpiGelu>); break;
    case kEpiRelu: go(gemm8p_nt<T, kEpiRelu>); break;
    case kEpiSigmoid: go(gemm8p_nt<T, kEpiSigmoid>); break;
    case kEpiDGelu: go(gemm8p_nt<T, kEpiDGelu>); break;
    case kEpiDRelu: go(gemm8p_nt<T, kEpiDRelu>); break;
    case kEpiDSigmoid: go(gemm8p_nt<T, kEpiDSigmoid>); break;
    default: throw std::runtime_error("gemm8p: unknown epilogue");
  }
}

}  // namespace g8p

}  // namespace gemm

bool gemm_supported(const GemmArgs& g) {
  if (g.dtype != kF16 && g.dtype != kBF16) return false;
  if (g.m <= 0 || g.n <= 0 || g.k <= 0) return false;
  auto al = [](const void* p) { return p == nullptr || ((uintptr_t)p & 15u) == 0; };
  if (!al(g.a) || !al(g.b) || !al(g.c) || !al(g.bias) || !al(g.aux_in) || !al(g.aux_out)) return false;
  // k-major operands are read as 16-byte k-vectors (K % 8); m/n-major operands are read as
  // 16-byte row vectors with per-k-row bounds checks, so their K may be ragged (weight grads
  // over an arbitrary token count).
  if ((g.a_kmajor || g.b_kmajor) && g.k % 8) return false;
  if (g.n % 8 || g.ldc % 8 || g.lda % 8 || g.ldb % 8) return false;
  if (!g.a_kmajor && g.m % 8) return false;
  if ((g.epilogue >= kEpiDGelu) && g.aux_in == nullptr) return false;
  return true;
}

bool gemm_colsum_fusable(const GemmArgs& g, int cus) {
  if (!gemm_supported(g) || !gemm::g256::usable(g, cus)) return false;
  if (g.a_kmajor && g.b_kmajor && gemm::g8p::enabled()) return false;
  int kc;
  return g.splitk_ws == nullptr || gemm::g256::splitk_parts(g, cus, &kc) <= 1;
}

void gemm_mfma(const GemmArgs& g, int cus, hipStream_t s) {
  if (!gemm_supported(g)) throw std::runtime_error("gemm_mfma: unsupported shape/alignment/dtype");
  if (g.colpart != nullptr && !gemm_colsum_fusable(g, cus))
    throw std::runtime_error("gemm_mfma: the column-sum epilogue needs the 256-tile kernel (gemm_colsum_fusable)");
  dispatch_16(g.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (gemm::g256::usable(g, cus)) {
      if (g.a_kmajor && g.b_kmajor && gemm::g8p::enabled()) gemm::g8p::launch<T>(g, s, cus);
      else if (g.a_kmajor && g.b_kmajor) gemm::g256::launch<T, true, true>(g, s, cus);
      else if (g.a_kmajor) gemm::g256::launch<T, true, false>(g, s, cus);
      else if (g.b_kmajor) gemm::g256::launch<T, false, true>(g, s, cus);
      else gemm::g256::launch<T, false, false>(g, s, cus);
    } else if (g.a_kmajor && g.b_kmajor) gemm::launch_epi<T, true, true>(g, s);
    else if (g.a_kmajor && !g.b_kmajor) gemm::launch_epi<T, true, false>(g, s);
    else if (!g.a_kmajor && g.b_kmajor) gemm::launch_epi<T, false, true>(g, s);
    else gemm::launch_epi<T, false, false>(g, s);
  }, "gemm_mfma");
  check_launch("gemm_mfma");
}

int64_t gemm_splitk_workspace_floats(const GemmArgs& g, int cus) {
  if (!gemm_supported(g)) return 0;
  int kc;
  const int sp = gemm::g256::splitk_parts(g, cus, &kc);
  return sp > 1 ? (int64_t)sp * g.m * g.n : 0;
}

void column_sum_finalize(const float* part, int p, int n, void* out, int out_dtype, hipStream_t s) {
  dispatch_float(out_dtype, [&](auto tag) {
    using TO = typename decltype(tag)::type;
    hipLaunchKernelGGL((gemm::colsum_finalize<TO>), dim3((n + 15) / 16), dim3(256), 0, s, part, p, n, (TO*)out);
  }, "column_sum_finalize");
  check_launch("column_sum_finalize");
}

int64_t column_sum_workspace_floats(int64_t m, int n, int cus) { return (int64_t)gemm::colsum_parts(m, n, cus) * n; }

void column_sum(const void* x, int dtype, int64_t m, int n, int64_t ldx, void* out, int out_dtype, float* ws, int cus,
                hipStream_t s) {
  if (n <= 0) return;
  if (n % 8 || ldx % 8 || ((uintptr_t)x & 15u)) throw std::runtime_error("column_sum: n, ldx must be multiples of 8");
  const int p = gemm::colsum_parts(m, n, cus);
  dispatch_float(dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    hipLaunchKernelGGL((gemm::colsum_partial<T>), dim3((n / 8 + 31) / 32, p), dim3(256), 0, s, (const T*)x, m, n, ldx,
                       ws);
  }, "column_sum");
  dispatch_float(out_dtype, [&](auto tag) {
    using TO = typename decltype(tag)::type;
    hipLaunchKernelGGL((gemm::colsum_finalize<TO>), dim3((n + 15) / 16), dim3(256), 0, s, ws, p, n, (TO*)out);
  }, "column_sum out");
  check_launch("column_sum");
}

void gelu_tanh_forward(const void* z, void* y, int dtype, int64_t numel, int cus, hipStream_t s) {
  if (numel % 8 || ((uintptr_t)z & 15) || ((uintptr_t)y & 15))
    throw std::runtime_error("gelu_tanh_forward: numel must be a multiple of 8, operands 16-byte aligned");
  const int64_t n8 = numel / 8;
  const int64_t blocks = std::min<int64_t>((n8 + 255) / 256, (int64_t)cus * 8);
  dispatch_16(dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    hipLaunchKernelGGL((gemm::gelu_fwd_kernel<T>), dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, s,
                       (const T*)z, (T*)y, n8);
  }, "gelu_tanh_forward");
  check_launch("gelu_tanh_forward");
}

void dgelu_column_sum(const void* dy, const void* aux, void* dz, int dtype, int64_t m, int n, void* out, int out_dtype,
                      float* ws, int cus, hipStream_t s) {
  if (n <= 0) return;
  if (n % 8 || ((uintptr_t)dy & 15u) || ((uintptr_t)aux & 15u) || ((uintptr_t)dz & 15u))
    throw std::runtime_error("dgelu_column_sum: n must be a multiple of 8, operands 16-byte aligned");
  const int p = gemm::colsum_parts(m, n, cus);
  dispatch_16(dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    hipLaunchKernelGGL((gemm::dgelu_colsum_partial<T>), dim3((n / 8 + 31) / 32, p), dim3(256), 0, s, (const T*)dy,
                       (const T*)aux, (T*)dz, m, n, ws);
  }, "dgelu_column_sum");
  dispatch_float(out_dtype, [&](auto tag) {
    using TO = typename decltype(tag)::type;
    hipLaunchKernelGGL((gemm::colsum_finalize<TO>), dim3((n + 15) / 16), dim3(256), 0, s, ws, p, n, (TO*)out);
  }, "dgelu_column_sum out");
  check_launch("dgelu_column_sum");
}

}  // namespace apex_amd
