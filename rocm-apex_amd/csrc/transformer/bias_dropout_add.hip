// Fused bias + dropout + residual add for the transformer block epilogues (Megatron's
// bias_dropout_add, reference apex/transformer/testing/standalone_gpt.py:530-560, which runs it as
// three torch ops: x + bias, dropout (philox, byte mask saved), residual + ...).
//
//   forward : out = residual + keep(i) * (x + bias[col]) / (1 - p)
//   backward: dx = g * keep(i) / (1 - p);  d_residual = g (no kernel);  d_bias = column sum of dx
// keep(i) is regenerated from a counter-based hash of (seed, offset, element index), so no mask is
// stored: the forward moves 3 tensors' bytes (x, residual in; out) instead of ~8.5, the backward 2
// instead of ~2.5 + a mask.  16 hash bits decide each element (two elements per 32-bit hash), so
// p is honoured to 1/65536.  Every thread handles 8 consecutive elements (16-byte I/O).
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"

namespace apex_amd {
namespace bda {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__host__ __device__ inline uint32_t seed_mix(uint64_t seed, uint64_t offset) {
  uint32_t x = (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x27d4eb2du) ^ ((uint32_t)offset * 0x165667b1u) ^
               ((uint32_t)(offset >> 32) * 0xd3a2646cu);
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// the mix for this launch: host (seed, offset) plus the optional device RNG step (graph-safe
// dropout: a hipGraph replay after the step counter advanced draws a fresh mask)
__device__ __forceinline__ uint32_t launch_mix(uint64_t seed, uint64_t offset, const int64_t* step) {
  return seed_mix(seed, offset + (step ? ((uint64_t)(*step) << 32) : 0ull));
}

// keep bits of elements e8 .. e8+7 (e8 a multiple of 8): one hash per element pair
__device__ __forceinline__ uint32_t keep8(uint32_t smix, uint64_t e8, uint32_t t16) {
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint64_t pair = (e8 >> 1) + j;
    const uint32_t h = mix32(smix ^ mix32((uint32_t)pair * 0x9E3779B9u ^ (uint32_t)(pair >> 32)));
    bits |= (uint32_t)((h & 0xffffu) >= t16) << (2 * j);
    bits |= (uint32_t)((h >> 16) >= t16) << (2 * j + 1);
  }
  return bits;
}

template <typename T, bool BIAS>
__global__ void __launch_bounds__(256) fwd_kernel(const T* __restrict__ x, const T* __restrict__ bias,
                                                  const T* __restrict__ res, T* __restrict__ out, int64_t nvec,
                                                  int h, uint64_t seed, uint64_t offset,
                                                  const int64_t* __restrict__ step, uint32_t t16, float scale) {
  const uint32_t smix = launch_mix(seed, offset, step);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * 8;
    float v[8], r[8], b[8];
    Vec8<T>::load(v, x + e);
    Vec8<T>::load(r, res + e);
    if constexpr (BIAS) Vec8<T>::load(b, bias + (int)(e % h));
    const uint32_t k = keep8(smix, (uint64_t)e, t16);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float xv = v[j];
      if constexpr (BIAS) xv += b[j];
      v[j] = r[j] + (((k >> j) & 1u) ? xv * scale : 0.f);
    }
    Vec8<T>::store(out + e, v);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bwd_kernel(const T* __restrict__ g, T* __restrict__ dx, int64_t nvec,
                                                  uint64_t seed, uint64_t offset, const int64_t* __restrict__ step,
                                                  uint32_t t16, float scale) {
  const uint32_t smix = launch_mix(seed, offset, step);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * 8;
    float v[8];
    Vec8<T>::load(v, g + e);
    const uint32_t k = keep8(smix, (uint64_t)e, t16);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ((k >> j) & 1u) ? v[j] * scale : 0.f;
    Vec8<T>::store(dx + e, v);
  }
}


inline uint32_t thresh16(float p) {
  const float t = p * 65536.f;
  return t >= 65536.f ? 65536u : (uint32_t)t;
}

inline unsigned grid_for(int64_t nvec, int cus) {
  int64_t g = (nvec + 255) / 256;
  if (g > (int64_t)cus * 8) g = (int64_t)cus * 8;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace bda

void bias_dropout_add_fwd(const void* x, const void* bias, const void* res, void* out, int64_t n, int h, int dtype,
                          float p, uint64_t seed, uint64_t offset, int cus, hipStream_t s, const int64_t* step) {
  if (n % 8 || h % 8) throw std::runtime_error("bias_dropout_add: numel and hidden size must be multiples of 8");
  const int64_t nvec = n / 8;
  const uint32_t t16 = bda::thresh16(p);
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  dispatch_float(dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    if (bias != nullptr)
      hipLaunchKernelGGL((bda::fwd_kernel<T, true>), dim3(bda::grid_for(nvec, cus)), dim3(256), 0, s, (const T*)x,
                         (const T*)bias, (const T*)res, (T*)out, nvec, h, seed, offset, step, t16, scale);
    else
      hipLaunchKernelGGL((bda::fwd_kernel<T, false>), dim3(bda::grid_for(nvec, cus)), dim3(256), 0, s, (const T*)x,
                         (const T*)nullptr, (const T*)res, (T*)out, nvec, h, seed, offset, step, t16, scale);
  }, "bias_dropout_add fwd");
  check_launch("bias_dropout_add fwd");
}

void bias_dropout_add_bwd(const void* g, void* dx, int64_t n, int dtype, float p, uint64_t seed, uint64_t offset, int cus,
                          hipStream_t s, const int64_t* step) {
  if (n % 8) throw std::runtime_error("bias_dropout_add: numel must be a multiple of 8");
  const int64_t nvec = n / 8;
  const uint32_t t16 = bda::thresh16(p);
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  dispatch_float(dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    hipLaunchKernelGGL((bda::bwd_kernel<T>), dim3(bda::grid_for(nvec, cus)), dim3(256), 0, s, (const T*)g, (T*)dx,
                       nvec, seed, offset, step, t16, scale);
  }, "bias_dropout_add bwd");
  check_launch("bias_dropout_add bwd");
}

}  // namespace apex_amd
