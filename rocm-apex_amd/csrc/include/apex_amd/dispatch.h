// Host-side dtype dispatch for device TUs (no torch dependency).
#pragma once
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

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace apex_amd
