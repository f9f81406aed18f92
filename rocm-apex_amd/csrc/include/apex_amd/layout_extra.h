// Layout passes declared apart from conv_api.h (csrc/conv/layout.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace apex_amd {
// y [N][hw][C] = g [N][C] * scale (16-bit, C % 8 == 0, 16-byte aligned): the channels_last input
// gradient of a global average pool
void spatial_broadcast(const void* g, void* y, int n, int hw, int c, float scale, int dtype, int cus, hipStream_t s);
}  // namespace apex_amd
