// Torch-free launchers for the fused NHWC batch-norm pipeline (csrc/groupbn/bn_nhwc.hip) behind
// apex.contrib.groupbn.BatchNorm2d_NHWC (reference apex/contrib/groupbn/batch_norm.py:24-260,
// apex/contrib/csrc/groupbn/batch_norm.cu, batch_norm_add_relu.cu).
//
// Data: x / z / y / dy / dx are dense [M, C] (C % 8 == 0, 16-byte aligned), bf16/fp16/fp32.
// Parameters and statistics are fp32.  The per-channel epilogue constants are precomputed once
// per layer by the finalize kernels so the streaming kernels do one FMA per element:
//   forward   y  = relu?(x * scale + shift [+ z])           coef_fwd = {scale, shift}[2][C]
//   backward  dx = A * dy' + B * x + K                     coef_bwd = {A, B, K}[3][C]
// where dy' is dy masked by the (recomputed) ReLU output.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

struct BnNhwcWorkspace {
  float* part;    // [2 * gy * C + gy] statistics / gradient-sum partials
  int gy;         // partials per channel (set by bn_nhwc_plan)
};

// number of partial rows the stats / reduce kernels will use, and the fp32 scratch they need
int bn_nhwc_plan(int64_t m, int c, int cus, int64_t* ws_floats);

// training forward statistics: mean, inv_std (saved for backward), coef_fwd, running stats update
void bn_nhwc_stats(const void* x, int x_t, int64_t m, int c, const float* w, const float* b, float eps,
                   float momentum, float* running_mean, float* running_var, float* save_mean, float* save_invstd,
                   float* coef_fwd, float* ws, int gy, int cus, hipStream_t s);

// eval / precomputed statistics: coef_fwd from given mean / inv_std (or running stats when
// `use_running` — then mean/inv_std are running_mean / running_var and eps is applied)
void bn_nhwc_coef_from_stats(const float* mean, const float* var_or_invstd, bool is_var, const float* w,
                             const float* b, float eps, int c, float* coef_fwd, hipStream_t s);

// mask_out (relu only, optional): one bit per element of (y > 0), [m * c / 8] bytes
void bn_nhwc_apply(const void* x, int x_t, const void* z, const float* coef_fwd, bool relu, void* y, int64_t m, int c,
                   int cus, hipStream_t s, uint8_t* mask_out = nullptr);

// y = relu(x * coef_x + z * coef_z) — two batch norms (coef_* = {scale, shift}[2][C]) summed under
// one ReLU in a single pass; optional ReLU bit mask as in bn_nhwc_apply
void bn_nhwc_apply_dual(const void* x, const void* z, int x_t, const float* coef_x, const float* coef_z, void* y,
                        int64_t m, int c, int cus, hipStream_t s, uint8_t* mask_out = nullptr);

// pooled = maxpool(relu(x * coef)) over an [n, h, w, c] NHWC tensor, plus the 1-byte window
// argmax per output element (the layout of csrc/pool/maxpool_nhwc.hip, so its backward applies)
void bn_nhwc_apply_relu_maxpool(const void* x, int x_t, const float* coef_fwd, int n, int h, int w, int c, int kh,
                                int kw, int sh, int sw, int ph, int pw, int oh, int ow, void* y, uint8_t* idx, int cus,
                                hipStream_t s);

// backward reduction: grad_w / grad_b (fp32) and coef_bwd; optionally writes the ReLU-masked dy
// (needed as grad_z for the add+relu variant); dy2 (optional, relu + dy_masked_out only) is a
// second gradient of the same output, summed into dy in registers
void bn_nhwc_bwd_reduce(const void* dy, const void* x, int x_t, const void* z, const float* coef_fwd, bool relu,
                        const float* save_mean, const float* save_invstd, const float* w, float* grad_w,
                        float* grad_b, float* coef_bwd, void* dy_masked_out, int64_t m, int c, float* ws, int gy,
                        int cus, hipStream_t s, const void* dy2 = nullptr, const uint8_t* mask_in = nullptr,
                        float* group_payload = nullptr);

// ---- bn_group > 1 (statistics shared by a group of ranks) ----
// forward, step 1: local payload [mean(C) | M2(C) | count] (fp32, 2C+1) for the group exchange
void bn_nhwc_stats_local(const void* x, int x_t, int64_t m, int c, float* payload, float* ws, int gy, int cus,
                         hipStream_t s);
// forward, step 2: merge the gathered [world][2C+1] payloads (fixed rank order: identical on every
// member) into save_mean / save_invstd / coef_fwd / running stats and 1/N_group (inv_count[1])
void bn_nhwc_stats_merge(const float* gathered, int world, int c, const float* w, const float* b, float eps,
                         float momentum, float* running_mean, float* running_var, float* save_mean, float* save_invstd,
                         float* coef_fwd, float* inv_count, hipStream_t s);
// backward: bn_nhwc_bwd_reduce(..., group_payload) writes [sum_dy | sum_dy_xmu] (2C) and the LOCAL
// grad_w / grad_b instead of coef_bwd; after the exchange, coef_bwd from the group's sums (`rows`
// payload rows summed in order: world after a peer all-gather, 1 after an all-reduce)
void bn_nhwc_bwd_coef_group(const float* sums, int rows, int c, const float* inv_count, const float* save_mean,
                            const float* save_invstd, const float* w, float* coef_bwd, hipStream_t s);
// group backward from externally computed partials [2][gy][C] (sum_dy | sum_dy_xmu rows, e.g. a
// convolution epilogue's): the exchange payload [2C] and the LOCAL grad_w / grad_b
void bn_nhwc_bwd_local(const float* part, int gy, int c, const float* save_invstd, float* grad_w, float* grad_b,
                       float* payload, hipStream_t s);

// dx = A * dy' + B * x + K   (dy' masked in registers when relu && !dy_is_masked)
void bn_nhwc_bwd_apply(const void* dy, bool dy_is_masked, const void* x, int x_t, const void* z,
                       const float* coef_fwd, bool relu, const float* coef_bwd, void* dx, int64_t m, int c, int cus,
                       hipStream_t s);

}  // namespace apex_amd
