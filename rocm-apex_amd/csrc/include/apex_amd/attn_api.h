// Fused (flash-style) multi-head attention on gfx950 MFMA: host interface.
//
// Tensors are addressed as [batch][seq][head][d] with arbitrary element strides for batch / seq /
// head and d contiguous, so every layout of the reference's callers maps onto the same kernel
// without a copy: the multihead_attn fast path's interleaved [s][b*h][3][d] QKV
// (apex/contrib/multihead_attn/self_multihead_attn_func.py:43-47), the FMHA packed varlen
// [total][3][h][d] with cu_seqlens (apex/contrib/fmha/fmha.py:33-55), and plain [b][s][h][d].
// Varlen: when cu_q / cu_k are given, token t of sequence b lives at row cu[b] + t (batch
// stride ignored) and the per-sequence length is cu[b+1] - cu[b].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

struct AttnTensor {
  void* p;
  int64_t sb, ss, sh;  // element strides of batch, sequence, head
};

struct AttnArgs {
  AttnTensor q, k, v, o;
  const int* cu_q;  // [b + 1] or nullptr
  const int* cu_k;
  int b, h, h_k;    // query heads, key/value heads (h % h_k == 0)
  int sq, sk;       // (max) sequence lengths
  int d;            // head dim: 32, 64 or 128
  int rows_q;       // token rows of the q-side fp32 side buffers (lse, delta, dq accum)
  float scale;
  bool causal;      // key j visible to query i iff j <= i
  const float* bias;  // additive fp32 bias/mask, broadcast by zero strides (or nullptr)
  int64_t bias_sb, bias_sh, bias_sq, bias_sk;
  float p_drop;     // attention-probability dropout
  uint64_t seed, offset;
  // optional device-resident RNG step (int64[1], graph-safe dropout): the effective offset is
  // offset + (step << 32), read by the kernel, so a hipGraph replay draws fresh masks once the
  // step counter has been advanced on the device
  const int64_t* rng_step;
  float* lse;       // [h][rows_q] natural-log sum-exp of the scaled scores (+inf: empty row)
  int dtype;        // kF16 / kBF16
};

struct AttnBwdArgs {
  AttnArgs f;       // forward arguments (o, lse as produced by the forward)
  AttnTensor dout, dq, dk, dv;
  float* dq_acc;    // fp32 [rows_q][h][d], zeroed by attn_bwd
  float* delta;     // fp32 [h][rows_q]
};

bool attn_supported(int d, int dtype);
void attn_fwd(const AttnArgs& a, hipStream_t s);
void attn_bwd(const AttnBwdArgs& a, hipStream_t s);

}  // namespace apex_amd
