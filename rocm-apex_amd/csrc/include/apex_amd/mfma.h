// gfx950 MFMA building blocks shared by the GEMM and attention kernels.
//
// v_mfma_f32_32x32x16_{bf16,f16} operand map (wave64):
//   A[m][k]: lane l holds m = l & 31, k = 8 (l >> 5) + j, j = 0..7 (one 16-byte register quad)
//   B[k][n]: lane l holds n = l & 31, k = 8 (l >> 5) + j
//   C[m][n]: lane l holds n = l & 31, m = (r & 3) + 8 (r >> 2) + 4 (l >> 5), r = 0..15
// Because the contraction index k is only a label, any fixed permutation of k shared by A and B
// is legal: an accumulator's registers 8s..8s+7 are directly the B operand of a follow-up MFMA
// whose k runs over C's m (rows) in the order crow(r) — the attention kernels use that to feed
// P (or dS) from registers into P·V without any LDS round trip.
#pragma once
#include "apex_amd/device.h"

namespace apex_amd {
namespace mfma {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename T>
__device__ __forceinline__ f32x16 mma(s16x8 a, s16x8 b, f32x16 c);
template <>
__device__ __forceinline__ f32x16 mma<bf16_t>(s16x8 a, s16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}
template <>
__device__ __forceinline__ f32x16 mma<f16_t>(s16x8 a, s16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// C-layout row of accumulator register r for this lane's half (h = lane >> 5)
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ds_read_b64_tr_b16: each 16-lane group reads a 4-row x 16-column block; the lane that supplies
// (row R + (li >> 2), col C + 4 (li & 3)) receives column C + li of rows R..R+3.
__device__ __forceinline__ s16x4 tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)((__attribute__((address_space(3))) uint16_t*)p));
}

// Row-major ("k-major") fragment: rows rowbase + (lane & 31), k = 16 kk + 8 (lane >> 5) .. + 7.
template <int STR>
__device__ __forceinline__ s16x8 frag_rows(const uint16_t* lds, int rowbase, int kk, int lane) {
  return *reinterpret_cast<const s16x8*>(lds + (rowbase + (lane & 31)) * STR + kk * 16 + 8 * (lane >> 5));
}

// Transposed fragment from a [k][m] image (m contiguous): lane gets m = colbase + (lane & 31) and
// k rows klo + 0..3 (j = 0..3) and khi + 0..3 (j = 4..7), where klo / khi are the row bases of this
// lane's 32-lane half.  The plain layout is klo = 16 kk + 8 h, khi = klo + 4; the attention kernels
// pass the crow() permutation klo = 16 s + 4 h, khi = klo + 8.
template <int STR>
__device__ __forceinline__ s16x8 frag_tr(const uint16_t* lds, int colbase, int klo, int khi, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int col = colbase + 16 * (g & 1) + 4 * p;
  const s16x4 lo = tr_read(lds + (klo + q) * STR + col);
  const s16x4 hi = tr_read(lds + (khi + q) * STR + col);
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// Pack 8 fp32 accumulator values (registers 8s..8s+7) into a 16-bit B/A operand.
template <typename T>
__device__ __forceinline__ s16x8 pack8(const float* v) {
  s16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)from_f<T>(v[j]).x;
  return r;
}

}  // namespace mfma
}  // namespace apex_amd
