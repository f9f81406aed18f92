// pybind surface of the fused attention kernels:
//   _C.attn.fwd / _C.attn.bwd      generic strided / varlen flash attention (apex.ops.attention)
//   _C.fmhalib.fwd / bwd (+ _nl)   the reference contrib FMHA module (apex/contrib/fmha/fmha.py:33-55):
//                                  packed qkv [total, 3, h, d] with cu_seqlens
#include <cmath>

#include "common.h"
#include "apex_amd/attn_api.h"

namespace apex_amd {

namespace {

using OT = c10::optional<at::Tensor>;
bool has(const OT& t) { return t.has_value() && t->defined(); }

// q-like tensor: [B, S, H, D] (padded) or [T, H, D] (varlen); d contiguous
AttnTensor view_of(const at::Tensor& t, bool varlen, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, ": GPU tensor expected");
  TORCH_CHECK(t.stride(-1) == 1, name, ": last (head) dim must be contiguous");
  AttnTensor v{};
  v.p = t.data_ptr();
  if (varlen) {
    TORCH_CHECK(t.dim() == 3, name, ": varlen tensors are [total, heads, d]");
    v.sb = 0;
    v.ss = t.stride(0);
    v.sh = t.stride(1);
  } else {
    TORCH_CHECK(t.dim() == 4, name, ": tensors are [batch, seq, heads, d]");
    v.sb = t.stride(0);
    v.ss = t.stride(1);
    v.sh = t.stride(2);
  }
  TORCH_CHECK(v.ss % 8 == 0 && v.sh % 8 == 0 && v.sb % 8 == 0 && ((uintptr_t)v.p & 15u) == 0, name,
              ": strides must be multiples of 8 elements and the base 16-byte aligned");
  return v;
}

struct Common {
  AttnArgs a{};
  at::Tensor cu_q_c, cu_k_c, bias_c;
};

void fill_common(Common& c, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const OT& cu_q,
                 const OT& cu_k, int64_t max_sq, int64_t max_sk, double scale, bool causal, const OT& bias,
                 double p_drop, int64_t seed, int64_t offset, const OT& rng_step = c10::nullopt) {
  const bool varlen = has(cu_q);
  TORCH_CHECK(varlen == has(cu_k), "attn: cu_seqlens_q and cu_seqlens_k go together");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(), "attn: dtype mismatch");
  // the forward's softmax takes the row max of the RAW scores and scales afterwards (valid for a
  // positive scale only), and folds the bias in as bias / scale
  TORCH_CHECK(scale > 0.0 && std::isfinite(scale), "attn: softmax scale must be positive and finite, got ", scale);
  AttnArgs& a = c.a;
  a.q = view_of(q, varlen, "q");
  a.k = view_of(k, varlen, "k");
  a.v = view_of(v, varlen, "v");
  a.d = (int)q.size(-1);
  TORCH_CHECK(k.size(-1) == a.d && v.size(-1) == a.d, "attn: head dims must match");
  a.dtype = dtype_code(q.scalar_type());
  TORCH_CHECK(attn_supported(a.d, a.dtype), "attn: head dim must be 32, 64 or 128 and dtype fp16/bf16");
  if (varlen) {
    c.cu_q_c = cu_q->to(at::kInt).contiguous();
    c.cu_k_c = cu_k->to(at::kInt).contiguous();
    a.cu_q = c.cu_q_c.data_ptr<int>();
    a.cu_k = c.cu_k_c.data_ptr<int>();
    a.b = (int)c.cu_q_c.numel() - 1;
    a.h = (int)q.size(1);
    a.h_k = (int)k.size(1);
    a.sq = (int)max_sq;
    a.sk = (int)max_sk;
    a.rows_q = (int)q.size(0);
  } else {
    a.b = (int)q.size(0);
    a.sq = (int)q.size(1);
    a.h = (int)q.size(2);
    a.sk = (int)k.size(1);
    a.h_k = (int)k.size(2);
    TORCH_CHECK(k.size(0) == a.b && v.size(0) == a.b, "attn: batch mismatch");
    a.rows_q = a.b * a.sq;
  }
  TORCH_CHECK(a.h_k > 0 && a.h % a.h_k == 0, "attn: query heads must be a multiple of key/value heads");
  a.scale = (float)scale;
  a.causal = causal;
  if (has(bias)) {
    TORCH_CHECK(bias->dim() == 4 && bias->scalar_type() == at::kFloat && bias->is_cuda(),
                "attn: bias must be a 4-D fp32 GPU tensor broadcastable to [b, h, sq, sk]");
    c.bias_c = *bias;
    a.bias = c.bias_c.data_ptr<float>();
    auto st = [&](int i) { return c.bias_c.size(i) == 1 ? (int64_t)0 : c.bias_c.stride(i); };
    a.bias_sb = st(0);
    a.bias_sh = st(1);
    a.bias_sq = st(2);
    a.bias_sk = st(3);
  }
  a.p_drop = (float)p_drop;
  a.seed = (uint64_t)seed;
  a.offset = (uint64_t)offset;
  a.rng_step = nullptr;
  if (has(rng_step)) {
    TORCH_CHECK(rng_step->is_cuda() && rng_step->scalar_type() == at::kLong && rng_step->numel() >= 1,
                "attn: rng_step must be an int64 GPU tensor");
    a.rng_step = rng_step->data_ptr<int64_t>();
  }
}

std::tuple<at::Tensor, at::Tensor> fwd(at::Tensor q, at::Tensor k, at::Tensor v, OT cu_q, OT cu_k, int64_t max_sq,
                                       int64_t max_sk, double scale, bool causal, OT bias, double p_drop, int64_t seed,
                                       int64_t offset, OT out, OT rng_step) {
  const c10::hip::HIPGuard guard(q.get_device());
  Common c;
  fill_common(c, q, k, v, cu_q, cu_k, max_sq, max_sk, scale, causal, bias, p_drop, seed, offset, rng_step);
  at::Tensor o = has(out) ? *out : at::empty(q.sizes(), q.options());
  c.a.o = view_of(o, has(cu_q), "out");
  at::Tensor lse = at::empty({c.a.h, c.a.rows_q}, q.options().dtype(at::kFloat));
  c.a.lse = lse.data_ptr<float>();
  attn_fwd(c.a, cur_stream());
  return {o, lse};
}

std::vector<at::Tensor> bwd(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor out, at::Tensor lse,
                            OT cu_q, OT cu_k, int64_t max_sq, int64_t max_sk, double scale, bool causal, OT bias,
                            double p_drop, int64_t seed, int64_t offset, OT dq_out, OT dk_out, OT dv_out,
                            OT rng_step) {
  const c10::hip::HIPGuard guard(q.get_device());
  Common c;
  fill_common(c, q, k, v, cu_q, cu_k, max_sq, max_sk, scale, causal, bias, p_drop, seed, offset, rng_step);
  const bool varlen = has(cu_q);
  AttnBwdArgs ba{};
  ba.f = c.a;
  ba.f.o = view_of(out, varlen, "out");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == (int64_t)c.a.h * c.a.rows_q,
              "attn bwd: lse must be the forward's [h, rows] fp32 tensor");
  ba.f.lse = lse.data_ptr<float>();
  at::Tensor g = dout;
  if (g.stride(-1) != 1 || g.stride(-2) % 8) g = g.contiguous();
  ba.dout = view_of(g, varlen, "dout");
  at::Tensor dq = has(dq_out) ? *dq_out : at::empty(q.sizes(), q.options());
  at::Tensor dk = has(dk_out) ? *dk_out : at::empty(k.sizes(), k.options());
  at::Tensor dv = has(dv_out) ? *dv_out : at::empty(v.sizes(), v.options());
  ba.dq = view_of(dq, varlen, "dq");
  ba.dk = view_of(dk, varlen, "dk");
  ba.dv = view_of(dv, varlen, "dv");
  // default: split atomic-free dK/dV + dQ kernels (1.1-3x the fused dQ-atomic kernel at every
  // head dim once their element loops are branch-free: profiles/kernels_attn_r01e.jsonl);
  // APEX_ATTN_BWD=atomic selects the fused kernel (kept for A/B timing)
  const char* mode = std::getenv("APEX_ATTN_BWD");
  const bool atomic = mode != nullptr && std::string(mode) == "atomic";
  at::Tensor dq_acc;
  if (atomic) dq_acc = at::empty({(int64_t)c.a.rows_q * c.a.h * c.a.d}, q.options().dtype(at::kFloat));
  at::Tensor delta = at::empty({(int64_t)c.a.h * c.a.rows_q}, q.options().dtype(at::kFloat));
  ba.dq_acc = atomic ? dq_acc.data_ptr<float>() : nullptr;
  ba.delta = delta.data_ptr<float>();
  attn_bwd(ba, cur_stream());
  return {dq, dk, dv};
}

// ---- contrib FMHA surface (qkv [total, 3, h, d]) ----
// seed / offset come from the python caller's torch generator (the reference passes a
// c10 Generator, apex/contrib/fmha/fmha.py:38)
std::vector<at::Tensor> fmha_fwd(at::Tensor qkv, at::Tensor cu_seqlens, double p_dropout, int64_t max_s,
                                 bool is_training, int64_t seed, int64_t offset) {
  TORCH_CHECK(qkv.dim() == 4 && qkv.size(1) == 3, "fmha: qkv must be [total, 3, heads, d]");
  const double p = is_training ? p_dropout : 0.0;
  const int64_t d = qkv.size(3);
  auto q = qkv.select(1, 0), k = qkv.select(1, 1), v = qkv.select(1, 2);
  auto r = fwd(q, k, v, cu_seqlens, cu_seqlens, max_s, max_s, 1.0 / std::sqrt((double)d), false, c10::nullopt, p, seed,
               offset, c10::nullopt, c10::nullopt);
  // "S_dmask" slot carries what the backward needs: lse + the dropout seed/offset
  auto meta = at::empty({2}, qkv.options().dtype(at::kLong).device(at::kCPU));
  meta[0] = seed;
  meta[1] = offset;
  return {std::get<0>(r), std::get<1>(r), meta};
}

std::vector<at::Tensor> fmha_bwd(at::Tensor dout, at::Tensor qkv, at::Tensor out, at::Tensor lse, at::Tensor meta,
                                 at::Tensor cu_seqlens, double p_dropout, int64_t max_s) {
  const int64_t d = qkv.size(3);
  auto dqkv = at::empty_like(qkv);
  auto q = qkv.select(1, 0), k = qkv.select(1, 1), v = qkv.select(1, 2);
  bwd(dout, q, k, v, out, lse, cu_seqlens, cu_seqlens, max_s, max_s, 1.0 / std::sqrt((double)d), false, c10::nullopt,
      p_dropout, meta[0].item<int64_t>(), meta[1].item<int64_t>(), dqkv.select(1, 0), dqkv.select(1, 1),
      dqkv.select(1, 2), c10::nullopt);
  return {dqkv};
}

}  // namespace

void bind_attn(pybind11::module_& root) {
  namespace py = pybind11;
  auto m = root.def_submodule("attn", "gfx950 flash attention (MFMA, in-register online softmax)");
  m.def("fwd", &fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("cu_seqlens_q") = c10::nullopt,
        py::arg("cu_seqlens_k") = c10::nullopt, py::arg("max_seqlen_q") = 0, py::arg("max_seqlen_k") = 0,
        py::arg("scale"), py::arg("causal") = false, py::arg("bias") = c10::nullopt, py::arg("dropout_p") = 0.0,
        py::arg("seed") = 0, py::arg("offset") = 0, py::arg("out") = c10::nullopt, py::arg("rng_step") = c10::nullopt);
  m.def("bwd", &bwd, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("out"), py::arg("lse"),
        py::arg("cu_seqlens_q") = c10::nullopt, py::arg("cu_seqlens_k") = c10::nullopt,
        py::arg("max_seqlen_q") = 0, py::arg("max_seqlen_k") = 0, py::arg("scale"), py::arg("causal") = false,
        py::arg("bias") = c10::nullopt, py::arg("dropout_p") = 0.0, py::arg("seed") = 0, py::arg("offset") = 0,
        py::arg("dq") = c10::nullopt, py::arg("dk") = c10::nullopt, py::arg("dv") = c10::nullopt,
        py::arg("rng_step") = c10::nullopt);
  m.def("supported", [](int64_t d, at::ScalarType t) {
    return (t == at::kHalf || t == at::kBFloat16) && attn_supported((int)d, dtype_code(t));
  });

  auto f = root.def_submodule("fmhalib", "contrib FMHA (packed varlen qkv) on the gfx950 flash kernels");
  f.def("fwd", &fmha_fwd);
  f.def("fwd_nl", &fmha_fwd);
  f.def("bwd", &fmha_bwd);
  f.def("bwd_nl", &fmha_bwd);
}

}  // namespace apex_amd
