// NHWC (channels_last) max pooling with 1-byte window indices (host interface).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

struct PoolArgs {
  int N, H, W, C, OH, OW, KH, KW, SH, SW, PH, PW;
  int dtype;
};

// y [N, OH, OW, C], idx [N, OH, OW, C] uint8 (kh * KW + kw of the max)
void maxpool_nhwc_fwd(const PoolArgs& a, const void* x, void* y, uint8_t* idx, int cus, hipStream_t s);
// dx [N, H, W, C] from dy [N, OH, OW, C] and idx (gather form: no atomics, no zero-fill pass)
void maxpool_nhwc_bwd(const PoolArgs& a, const void* dy, const uint8_t* idx, void* dx, int cus, hipStream_t s);

}  // namespace apex_amd
