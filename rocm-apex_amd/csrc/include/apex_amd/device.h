// Device-side building blocks shared by every gfx950 kernel in this package.
//
// Design notes (MI355X / CDNA4):
//  * wave64 everywhere: lane = threadIdx.x & 63, reductions use 6 xor-shuffle steps.
//    (The reference hard-codes a 16-lane start in its max reduction, csrc/type_shim.h:441,
//    which is wrong on wave64; we never use warp-sized constants.)
//  * 16-bit storage is handled as raw uint16 and converted with the native clang types
//    (_Float16 / __bf16); a plain cast lowers to v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN-safe).
//  * Memory-bound kernels move 8 elements per lane per step: 2 x dwordx4 for fp32,
//    1 x dwordx4 for 16-bit types (Guideline 13: never scalar 16-bit loads).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

// dtype tags understood by the host dispatchers (must match python/bindings side)
enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2, kF64 = 3, kU8 = 4, kI32 = 5, kI64 = 6, kFP8E5M2 = 7, kFP8E4M3 = 8 };

struct f16_t { uint16_t x; };
struct bf16_t { uint16_t x; };
// OCP fp8 storage (gfx950 converts natively: v_cvt_pk_{bf8,fp8}_f32 / v_cvt_[pk_]f32_{bf8,fp8}).
// e5m2 == torch.float8_e5m2, e4m3 == torch.float8_e4m3fn.
struct fp8e5m2_t { uint8_t x; };
struct fp8e4m3_t { uint8_t x; };

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(double v) { return (float)v; }
__device__ __forceinline__ float to_f(f16_t v) { return (float)__builtin_bit_cast(_Float16, v.x); }
__device__ __forceinline__ float to_f(bf16_t v) { return __uint_as_float(((uint32_t)v.x) << 16); }

__device__ __forceinline__ float to_f(fp8e5m2_t v) { return __builtin_amdgcn_cvt_f32_bf8((int)v.x, 0); }
__device__ __forceinline__ float to_f(fp8e4m3_t v) { return __builtin_amdgcn_cvt_f32_fp8((int)v.x, 0); }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ double from_f<double>(float v) { return (double)v; }
template <> __device__ __forceinline__ f16_t from_f<f16_t>(float v) {
  return f16_t{__builtin_bit_cast(uint16_t, (_Float16)v)};
}
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float v) {
  return bf16_t{__builtin_bit_cast(uint16_t, (__bf16)v)};
}

template <> __device__ __forceinline__ fp8e5m2_t from_f<fp8e5m2_t>(float v) {
  return fp8e5m2_t{(uint8_t)(__builtin_amdgcn_cvt_pk_bf8_f32(v, v, 0, false) & 0xffu)};
}
template <> __device__ __forceinline__ fp8e4m3_t from_f<fp8e4m3_t>(float v) {
  return fp8e4m3_t{(uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false) & 0xffu)};
}

__device__ __forceinline__ bool is_finite(float v) { return __builtin_isfinite(v); }

// ---------------------------------------------------------------------------------------------
// 8-wide vector load/store to float registers.
// ---------------------------------------------------------------------------------------------
template <typename T> struct Vec8;

template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(float (&r)[8], const float* p) {
    const float4 a = reinterpret_cast<const float4*>(p)[0];
    const float4 b = reinterpret_cast<const float4*>(p)[1];
    r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
    r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&r)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(r[0], r[1], r[2], r[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(r[4], r[5], r[6], r[7]);
  }
};

template <typename T16> struct Vec8_16 {
  static __device__ __forceinline__ void load(float (&r)[8], const T16* p) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      r[2 * i] = to_f(T16{(uint16_t)(w[i] & 0xffffu)});
      r[2 * i + 1] = to_f(T16{(uint16_t)(w[i] >> 16)});
    }
  }
  static __device__ __forceinline__ void store(T16* p, const float (&r)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = (uint32_t)from_f<T16>(r[2 * i]).x | ((uint32_t)from_f<T16>(r[2 * i + 1]).x << 16);
    }
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct Vec8<f16_t> : Vec8_16<f16_t> {};
template <> struct Vec8<bf16_t> : Vec8_16<bf16_t> {};

// fp8: 8 elements = one dwordx2; packed converts handle two values per instruction
template <bool E5M2> struct Vec8_8 {
  static __device__ __forceinline__ void load(float (&r)[8], const void* p) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    const uint32_t w[2] = {u.x, u.y};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const auto lo = E5M2 ? __builtin_amdgcn_cvt_pk_f32_bf8((int)w[i], false)
                           : __builtin_amdgcn_cvt_pk_f32_fp8((int)w[i], false);
      const auto hi = E5M2 ? __builtin_amdgcn_cvt_pk_f32_bf8((int)w[i], true)
                           : __builtin_amdgcn_cvt_pk_f32_fp8((int)w[i], true);
      r[4 * i] = lo[0];
      r[4 * i + 1] = lo[1];
      r[4 * i + 2] = hi[0];
      r[4 * i + 3] = hi[1];
    }
  }
  static __device__ __forceinline__ void store(void* p, const float (&r)[8]) {
    uint32_t w[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int acc = 0;
      if constexpr (E5M2) {
        acc = __builtin_amdgcn_cvt_pk_bf8_f32(r[4 * i], r[4 * i + 1], acc, false);
        acc = __builtin_amdgcn_cvt_pk_bf8_f32(r[4 * i + 2], r[4 * i + 3], acc, true);
      } else {
        acc = __builtin_amdgcn_cvt_pk_fp8_f32(r[4 * i], r[4 * i + 1], acc, false);
        acc = __builtin_amdgcn_cvt_pk_fp8_f32(r[4 * i + 2], r[4 * i + 3], acc, true);
      }
      w[i] = (uint32_t)acc;
    }
    *reinterpret_cast<uint2*>(p) = make_uint2(w[0], w[1]);
  }
};
template <> struct Vec8<fp8e5m2_t> : Vec8_8<true> {};
template <> struct Vec8<fp8e4m3_t> : Vec8_8<false> {};

// ---------------------------------------------------------------------------------------------
// wave64 / block reductions
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum; `smem` needs blockDim.x/64 floats. Result valid in every lane.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  T r = 0;
  for (int i = 0; i < nw; ++i) r += smem[i];  // fixed order: deterministic
  return r;
}
__device__ __forceinline__ float block_max(float v, float* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, smem[i]);
  return r;
}

// A scalar that is either a host immediate or read from device memory at kernel time
// (device form keeps optimizer steps sync-free and CUDA/HIP-graph capturable).
struct DevScalar {
  float v;
  const float* p;
  __device__ __forceinline__ float get() const { return p ? *p : v; }
};

}  // namespace apex_amd
