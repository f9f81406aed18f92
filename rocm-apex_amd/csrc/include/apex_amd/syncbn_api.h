// Torch-free launchers for the batch-norm statistics / apply kernels (csrc/syncbn/welford.hip).
//
// Reference: csrc/syncbn.cpp:8-109, csrc/welford.cu (welford_kernel :272, batchnorm_forward
// :314, reduce_bn :344, batchnorm_backward :411, c_last variants :454-895, welford_parallel :597).
//
// Layouts: "c_last" = a dense [M, C] view (NHWC activations, or torch channels_last memory seen
// through a permuted view); "nchw" = dense [N, C, S] with S = prod(spatial).
//
// Fused ReLU (c_last): forward computes relu(bn(x) + z); the backward kernels can recompute that
// output in registers and mask dy on the fly (FusedRelu), so no masked-gradient tensor has to
// be written and re-read unless the residual branch needs it (bn_relu_backward).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

struct BnShape {
  int64_t n;   // nchw: N ; c_last: M (rows)
  int c;
  int64_t s;   // nchw: spatial size ; c_last: 1
  bool c_last;
};

struct BnParams {
  const float* mean;     // [C]
  const float* inv_std;  // [C]
  const void* w;         // [C] or null
  const void* b;         // [C] or null
  int w_t;               // dtype of w/b (when present)
};

struct FusedRelu {
  bool on = false;
  const void* z = nullptr;  // residual added before the ReLU (x dtype) or null
};

// fp32 scratch (floats) the reductions need for this shape on `cus` CUs
int64_t bn_workspace_floats(const BnShape& sh, int cus);

// mean[C], var_biased[C]
void bn_welford(const void* x, int x_t, const BnShape& sh, float* mean, float* var_biased, float* ws, int cus,
                hipStream_t s);

// merge `world` (mean, biased var, count) rows -> mean, unbiased var, inv_std
void bn_welford_parallel(const float* mean_all, const float* var_all, const int* count_all, int world, int c,
                         float eps, float* mean, float* var_unbiased, float* inv_std, hipStream_t s);

// y = (x - mean) * inv_std * w + b [+ z] [relu]
void bn_forward(const void* x, int x_t, const BnParams& p, const FusedRelu& r, void* y, const BnShape& sh,
                int cus, hipStream_t s);

// dy_out = dy masked by the recomputed fused-ReLU output (c_last)
void bn_relu_backward(const void* dy, const void* x, int x_t, const BnParams& p, const FusedRelu& r, void* dy_out,
                      const BnShape& sh, int cus, hipStream_t s);

// sum_dy[C], sum_dy_xmu[C], and (if grad_w) grad_weight = sum_dy_xmu * inv_std, grad_bias = sum_dy
void bn_reduce(const void* dy, const void* x, int x_t, const BnParams& p, const FusedRelu& r, float* sum_dy,
               float* sum_dy_xmu, void* grad_w, void* grad_b, const BnShape& sh, float* ws, int cus, hipStream_t s);

// dx from globally reduced sums; elements per channel = sum(count[0..world))
void bn_backward(const void* dy, const void* x, int x_t, const BnParams& p, const FusedRelu& r, const float* sum_dy,
                 const float* sum_dy_xmu, const int* count, int world, void* dx, const BnShape& sh, int cus,
                 hipStream_t s);

}  // namespace apex_amd
