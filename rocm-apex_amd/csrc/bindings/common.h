// Shared helpers for the pybind layer (torch-aware host code only).
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>
#include <hip/hip_runtime.h>
#include <vector>
#include "apex_amd/mta_api.h"

namespace apex_amd {

inline int dtype_code(const at::ScalarType t) {
  switch (t) {
    case at::kFloat: return kF32;
    case at::kHalf: return kF16;
    case at::kBFloat16: return kBF16;
    case at::kDouble: return kF64;
    case at::kByte: return kU8;
    case at::kInt: return kI32;
    case at::kLong: return kI64;
    case at::kFloat8_e5m2: return kFP8E5M2;
    case at::kFloat8_e4m3fn: return kFP8E4M3;
    default: TORCH_CHECK(false, "apex_amd: unsupported dtype ", t);
  }
  return -1;
}

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline int device_cus(int dev) {
  static int cache[64] = {0};
  if (dev < 0 || dev >= 64) dev = 0;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
    cache[dev] = n > 0 ? n : 256;
  }
  return cache[dev];
}

// Persistent-grid cap for streaming kernels: 8 resident 256-thread blocks per CU.
inline Launch make_launch(const at::Tensor& like) {
  Launch L;
  L.stream = cur_stream();
  L.max_blocks = device_cus(like.get_device()) * 8;
  return L;
}

inline DevScalar dev_scalar(const c10::optional<at::Tensor>& t, float v) {
  DevScalar s;
  s.v = v;
  s.p = nullptr;
  if (t.has_value() && t->defined()) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() >= 1,
                "device scalar must be a 1-element float32 GPU tensor");
    s.p = t->data_ptr<float>();
  }
  return s;
}

// Returns (and caches) the device work table for a list-of-lists of tensors.
MtaMeta mta_meta(const std::vector<std::vector<at::Tensor>>& lists, int chunk_size);

}  // namespace apex_amd
