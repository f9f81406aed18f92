// Host-side dtype dispatch for device TUs (no torch dependency).
#pragma once
#include <cstdlib>
#include <stdexcept>
#include <string>
#include "apex_amd/device.h"

namespace apex_amd {

template <typename T> struct Tag { using type = T; };

template <typename F>
inline void dispatch_float(int dt, F&& f, const char* what) {
  switch (dt) {
    case kF32: f(Tag<float>{}); break;
    case kF16: f(Tag<f16_t>{}); break;
    case kBF16: f(Tag<bf16_t>{}); break;
    default: throw std::runtime_error(std::string(what) + ": unsupported dtype " + std::to_string(dt));
  }
}

template <typename F>
inline void dispatch_16(int dt, F&& f, const char* what) {
  switch (dt) {
    case kF16: f(Tag<f16_t>{}); break;
    case kBF16: f(Tag<bf16_t>{}); break;
    default: throw std::runtime_error(std::string(what) + ": expected fp16/bf16, got dtype " + std::to_string(dt));
  }
}

// model-copy outputs of the fused optimizers: 16-bit weights or an fp8 all-gather payload
template <typename F>
inline void dispatch_model_out(int dt, F&& f, const char* what) {
  switch (dt) {
    case kF16: f(Tag<f16_t>{}); break;
    case kBF16: f(Tag<bf16_t>{}); break;
    case kFP8E5M2: f(Tag<fp8e5m2_t>{}); break;
    case kFP8E4M3: f(Tag<fp8e4m3_t>{}); break;
    default: throw std::runtime_error(std::string(what) + ": expected fp16/bf16/fp8, got dtype " + std::to_string(dt));
  }
}

// any storage type the elementwise engine can convert (casts)
template <typename F>
inline void dispatch_any(int dt, F&& f, const char* what) {
  switch (dt) {
    case kFP8E5M2: f(Tag<fp8e5m2_t>{}); break;
    case kFP8E4M3: f(Tag<fp8e4m3_t>{}); break;
    default: dispatch_float(dt, f, what);
  }
}

// APEX_AMD_SYNC_LAUNCH=1: debug mode — every native launch is followed by a
// device synchronize, so an asynchronous fault (out-of-bounds access, trap) is reported as an
// exception naming the op that caused it instead of surfacing at some later sync point.  Like
// AMD_SERIALIZE_KERNEL it serialises the process; not for use under hipGraph capture.
inline bool sync_launch_debug() {
  static const bool on = [] {
    const char* v = std::getenv("APEX_AMD_SYNC_LAUNCH");
    return v != nullptr && v[0] != '\0' && v[0] != '0';
  }();
  return on;
}

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && sync_launch_debug()) e = hipDeviceSynchronize();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace apex_amd
