// Torch-free launchers for the fused scale/mask/softmax kernels (csrc/softmax/softmax.hip).
//
// Reference: csrc/megatron/scaled_masked_softmax.h (padding mask, uint8, masked -> -10000),
// csrc/megatron/scaled_upper_triang_masked_softmax.h (causal).  The reference limits the key
// length to 2048 (one warp row, register tile); here rows of up to 16384 keys stay register
// resident (1, 4 or 8 wave64s per row) and longer rows use a generic kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

enum SoftmaxMask : int { kMaskNone = 0, kMaskPad = 1, kMaskCausal = 2 };

struct SoftmaxFwdArgs {
  const void* x;        // [rows, sk]
  const uint8_t* mask;  // kMaskPad: [pad_batches, 1, sq, sk]; 1 = masked
  void* y;              // [rows, sk]
  int64_t rows;         // b * np * sq (or attn_batches * sq)
  int sq, sk;
  int heads;            // np (pad mask batch stride)
  int pad_batches;      // 1 => mask broadcast over the batch
  float scale;
  int mode;             // SoftmaxMask
  int dtype;            // kF16 / kBF16 / kF32
};

struct SoftmaxBwdArgs {
  const void* dy;       // [rows, sk]
  const void* y;        // [rows, sk] softmax output
  void* dx;             // [rows, sk] (may alias dy)
  int64_t rows;
  int sk;
  float scale;
  int dtype;
};

void softmax_fwd(const SoftmaxFwdArgs& a, hipStream_t s);
void softmax_bwd(const SoftmaxBwdArgs& a, hipStream_t s);

}  // namespace apex_amd
