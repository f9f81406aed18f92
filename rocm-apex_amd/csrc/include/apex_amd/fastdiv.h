// Exact unsigned 32-bit division by a runtime-constant divisor (Granlund-Montgomery, round-up
// multiplier with the "add" fix-up): q = (t + ((n - t) >> s1)) >> s2, t = umulhi(n, mul).  Four
// VALU ops instead of the ~30 of a v_rcp-based integer divide.  Host builds the constants once
// per launch; kernels decompose flat pixel indices with it.
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace apex_amd {

struct FastDiv {
  uint32_t d, mul, s1, s2;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.mul = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  f.s1 = l > 0 ? 1 : 0;
  f.s2 = l > 0 ? l - 1 : 0;
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  const uint32_t t = __umulhi(n, f.mul);
  return (t + ((n - t) >> f.s1)) >> f.s2;
}

}  // namespace apex_amd
