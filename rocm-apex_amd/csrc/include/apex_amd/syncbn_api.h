// Torch-free launchers for the batch-norm statistics / apply kernels (csrc/syncbn/welford.hip).
//
// Reference: csrc/syncbn.cpp:8-109, csrc/welford.cu (welford_kernel :272, batchnorm_forward
// :314, reduce_bn :344, batchnorm_backward :411, c_last variants :454-895, welford_parallel :597).
//
// Layouts: "c_last" = a dense [M, C] view (NHWC activations, or torch channels_last memory seen
// through a permuted view); "nchw" = dense [N, C, S] with S = prod(spatial).
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

// fp32 scratch (floats) the reductions need for this shape on `cus` CUs
int64_t bn_workspace_floats(const BnShape& sh, int cus);

// mean[C], var_biased[C]
void bn_welford(const void* x, int x_t, const BnShape& sh, float* mean, float* var_biased, float* ws, int cus,
                hipStream_t s);

// merge `world` (mean, biased var, count) rows -> mean, unbiased var, inv_std
void bn_welford_parallel(const float* mean_all, const float* var_all, const int* count_all, int world, int c,
                         float eps, float* mean, float* var_unbiased, float* inv_std, hipStream_t s);

// y = (x - mean) * inv_std * w + b [+ z] [relu]
void bn_forward(const void* x, int x_t, const void* z, const float* mean, const float* inv_std, const void* w,
                const void* b, int w_t, void* y, const BnShape& sh, bool relu, hipStream_t s);

// grad_out masked by the recomputed fused-ReLU output (c_last only)
void bn_relu_backward(const void* dy, const void* x, int x_t, const void* z, const float* mean, const float* inv_std,
                      const void* w, const void* b, int w_t, void* dy_out, const BnShape& sh, hipStream_t s);

// sum_dy[C], sum_dy_xmu[C], and (if w_t >= 0) grad_weight = sum_dy_xmu * inv_std, grad_bias = sum_dy
void bn_reduce(const void* dy, const void* x, int x_t, const float* mean, const float* inv_std, float* sum_dy,
               float* sum_dy_xmu, void* grad_w, void* grad_b, int w_t, const BnShape& sh, float* ws, int cus,
               hipStream_t s);

// dx from globally reduced sums; total element count per channel = sum(count[0..world))
void bn_backward(const void* dy, const void* x, int x_t, const float* mean, const float* inv_std, const void* w,
                 int w_t, const float* sum_dy, const float* sum_dy_xmu, const int* count, int world, void* dx,
                 const BnShape& sh, hipStream_t s);

}  // namespace apex_amd
