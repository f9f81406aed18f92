// RNN-T transducer joint / loss kernels (host interface).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

struct JointArgs {
  const void* f;  // [B, T, H]
  const void* g;  // [B, U, H]
  const int* f_len;
  const int* g_len;
  const int64_t* batch_offset;  // packed: inclusive cumsum of f_len * g_len
  void* out;                    // [B, T, U, H] or packed [sum, H]
  uint8_t* mask;                // same shape as out (relu / dropout) or nullptr
  int B, T, U, H;
  bool packed, relu, dropout;
  float p_drop;
  uint64_t seed, offset;
  int dtype;
};

struct LossArgs {
  const void* x;  // log-probs [B, T, U, V] (U = max label len + 1) or packed [sum, V]
  const int* label;  // [B, U - 1]
  const int* f_len;
  const int* y_len;
  const int64_t* batch_offset;  // packed: inclusive cumsum of f_len * (y_len + 1)
  float* alpha;  // [B, T, U]
  float* beta;   // [B, T, U]
  float* loss;   // [B]
  int B, T, U;
  int64_t V;
  int blank;
  bool packed;
  int dtype;
};

void transducer_joint_fwd(const JointArgs& a, hipStream_t s);
void transducer_joint_bwd(const JointArgs& a, const void* grad, void* f_grad, void* g_grad, float scale,
                          hipStream_t s);
void transducer_loss_fwd(const LossArgs& a, hipStream_t s);
void transducer_loss_bwd(const LossArgs& a, const float* loss_grad, void* x_grad, bool fused, hipStream_t s);

}  // namespace apex_amd
