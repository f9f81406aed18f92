// Torch-free launchers for the row-normalisation kernels (csrc/norm/*.hip).
//
// Reference behaviour: csrc/layer_norm_cuda.cpp:121-266 / csrc/layer_norm_cuda_kernel.cu
// (LayerNorm fwd/bwd, affine / non-affine / "mixed dtypes").  RMSNorm shares the machinery
// (mean == 0).  All statistics are fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

struct NormFwdArgs {
  const void* x;       // [n1, n2] input (in_t)
  const void* gamma;   // [n2] or null (w_t)
  const void* beta;    // [n2] or null (w_t)
  void* y;             // [n1, n2] output (out_t)
  float* mean;         // [n1] (LayerNorm only)
  float* invvar;       // [n1]
  int64_t n1;
  int n2;
  float eps;
  int in_t, w_t, out_t;
  bool rms;
};

struct NormBwdArgs {
  const void* dy;      // [n1, n2] (out_t)
  const void* x;       // [n1, n2] (in_t)
  const float* mean;   // [n1] (null for RMSNorm)
  const float* invvar; // [n1]
  const void* gamma;   // [n2] or null
  void* dx;            // [n1, n2] (in_t)
  void* dgamma;        // [n2] or null (w_t)
  void* dbeta;         // [n2] or null (w_t)
  float* workspace;    // [norm_bwd_workspace_floats()] fp32 partials
  int64_t n1;
  int n2;
  int in_t, w_t, out_t;
  bool rms;
  // nullable [n1, n2] (out_t): a gradient added to dx in the same pass — the residual branch's
  // gradient of a pre-LN transformer block (x feeds both the norm and the residual add), so the
  // autograd sum of the two is not a separate elementwise kernel
  const void* dres = nullptr;
};

// fp32 scratch needed by norm_bwd for (n1, n2) on a device with `cus` compute units.
int64_t norm_bwd_workspace_floats(int64_t n1, int n2, int cus);

void norm_fwd(const NormFwdArgs& a, int cus, hipStream_t s);
void norm_bwd(const NormBwdArgs& a, int cus, hipStream_t s);

}  // namespace apex_amd
