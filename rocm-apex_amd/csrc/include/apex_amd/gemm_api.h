// Torch-free launcher for the gfx950 MFMA GEMM with fused epilogues (csrc/gemm/gemm_mfma.hip),
// the engine behind apex.fused_dense (FusedDense, FusedDenseGeluDense) and apex.mlp.
//
// C[M][N] = A(M x K) * B(K x N), bf16/fp16 in, fp32 accumulate, bf16/fp16 out.
//   A "k-major": A(m, k) = A[m * lda + k]    (e.g. activations X[M][K])
//   A "m-major": A(m, k) = A[k * lda + m]    (e.g. dY^T for the weight gradient)
//   B "k-major": B(k, n) = B[n * ldb + k]    (e.g. torch Linear weight W[N][K] in forward)
//   B "n-major": B(k, n) = B[k * ldb + n]    (e.g. W[N'][K'] in the input-gradient GEMM, X in wgrad)
// The LDS staging keeps the global image; m/n-major operands are read back with the gfx950
// hardware transpose read (ds_read_b64_tr_b16), so no transpose kernel runs in any of the
// three GEMMs of a Linear layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

enum GemmEpilogue : int {
  kEpiNone = 0,      // C = acc + bias
  kEpiGelu = 1,      // aux_out = acc + bias ; C = gelu_tanh(aux_out)
  kEpiRelu = 2,      // C = relu(acc + bias)
  kEpiSigmoid = 3,   // C = sigmoid(acc + bias)
  kEpiDGelu = 4,     // C = acc * gelu_tanh'(aux_in)            (aux_in = pre-activation)
  kEpiDRelu = 5,     // C = acc * (aux_in > 0)                  (aux_in = relu output)
  kEpiDSigmoid = 6,  // C = acc * aux_in * (1 - aux_in)         (aux_in = sigmoid output)
};

struct GemmArgs {
  const void* a;
  const void* b;
  void* c;
  int64_t lda, ldb, ldc;
  int m, n, k;
  bool a_kmajor, b_kmajor;
  int dtype;            // kF16 / kBF16 (A, B, C, bias, aux)
  int epilogue;         // GemmEpilogue
  const void* bias;     // [N] or null
  const void* aux_in;   // [M][ldc] or null
  void* aux_out;        // [M][ldc] or null
  float* splitk_ws;     // fp32 split-K partials (gemm_splitk_workspace_floats) or null = no split
  // fp32 [ceil(m / 256)][n] column sums of the stored C per 256-row tile, or null (the bias
  // gradient of an activation-gradient GEMM: DGELU_BGRAD; gemm_colsum_fusable shapes only),
  // summed by column_sum_finalize
  float* colpart = nullptr;
};

// true when the shape / alignment / dtype is supported by the MFMA kernel
bool gemm_supported(const GemmArgs& g);
// true when g runs on the 256-tile kernel unsplit, which takes GemmArgs::colpart
bool gemm_colsum_fusable(const GemmArgs& g, int cus);
// out[n] = sum over p rows of part[p][n] (fixed order), written in out_dtype
void column_sum_finalize(const float* part, int p, int n, void* out, int out_dtype, hipStream_t s);
void gemm_mfma(const GemmArgs& g, int cus, hipStream_t s);
// fp32 workspace a split-K launch of g needs (0: the shape runs unsplit).  Split-K is used for
// no-epilogue GEMMs whose output has too few 256x256 tiles to fill the chip but whose K is long
// (weight gradients over many tokens): K is cut into chunks of >= 1024, each (tile, chunk)
// workgroup writes an fp32 partial tile, and a reduce pass sums the chunks and adds the bias.
int64_t gemm_splitk_workspace_floats(const GemmArgs& g, int cus);

// out[n] = sum_m x[m][n]  (fp32 accumulate, deterministic; used for bias gradients)
void column_sum(const void* x, int dtype, int64_t m, int n, int64_t ldx, void* out, int out_dtype, float* ws, int cus,
                hipStream_t s);
int64_t column_sum_workspace_floats(int64_t m, int n, int cus);
// dz = dy * gelu_tanh'(aux) and out = column sums of dz, one pass (workspace as column_sum)
// y = gelu_tanh(z) elementwise (numel % 8 == 0, 16-byte aligned), full-bandwidth vector pass
void gelu_tanh_forward(const void* z, void* y, int dtype, int64_t numel, int cus, hipStream_t s);
void dgelu_column_sum(const void* dy, const void* aux, void* dz, int dtype, int64_t m, int n, void* out, int out_dtype,
                      float* ws, int cus, hipStream_t s);

}  // namespace apex_amd
