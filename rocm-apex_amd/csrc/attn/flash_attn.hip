// Flash-style fused attention, forward and backward, for gfx950 (wave64, v_mfma_f32_32x32x16).
//
// Replaces the reference's three separate attention paths with one kernel family:
//   * contrib multihead_attn "fast" impl: QKV GEMM -> strided-batched QK^T -> masked softmax +
//     dropout -> strided-batched PV (apex/contrib/csrc/multihead_attn/self_multihead_attn_cuda.cu,
//     materialises the [b*h, sq, sk] score and probability tensors in HBM),
//   * contrib fmha (sm80-only CUTLASS kernels, head dim 64, seq <= 512;
//     apex/contrib/csrc/fmha/src/fmha_fprop_fp16_kernel.sm80.cu),
//   * the masked softmax of apex.transformer.functional.FusedScaleMaskSoftmax when the caller
//     wants the whole attention.
// Nothing of size sq x sk ever reaches HBM.
//
// Forward (one workgroup = 4 waves = 128 query rows of one (batch, head); 64-key tiles):
//   * "swapped" S^T = K Q^T: K tile rows are the MFMA A operand (row reads from LDS), each wave's
//     32 query rows live in registers as the B operand.  The accumulator then holds, per lane,
//     ONE query and 16 keys per 32-key tile, so the online-softmax row max / row sum are 31
//     in-register ops plus one lane^32 exchange.
//   * P stays in registers: accumulator registers 8s..8s+7 are the B operand of O^T += V^T P^T
//     (k permuted by crow(), V^T read with ds_read_b64_tr_b16 at the matching rows).
//   * K/V tiles double-buffered in LDS with register staging (issue next tile's loads before the
//     MFMAs, write them after), one barrier per tile; K rows padded to D+8 (conflict-free
//     ds_read_b128), V rows to a 64/192-B bank offset for the transposed reads.
//   * masks: key padding (varlen lengths), causal, additive fp32 bias with broadcast strides;
//     dropout by a counter-based hash of (seed, offset, batch*head, query, key) — regenerated
//     bit-exactly by the backward pass.
// Backward (FlashAttention-2 order; one workgroup = 4 waves = 128 keys of one (batch, kv head)):
//   * per 32-query slice: S and dP with the key on the lane (K, V of the wave's 32 keys in
//     registers), P = exp2(c S - lse2), dS = P (dP - delta); dV^T += dO^T P and dK^T += Q^T dS
//     with P / dS fed from registers (same crow() trick), Q / dO read transposed from one LDS
//     image each; dS crosses LDS once for dQ = dS K, which is summed over key blocks with
//     no-return global_atomic_add_f32 into an fp32 buffer (full 128-B segments per instruction).
//   * GQA: the workgroup sweeps every query head of its kv group, so dK / dV need no cross-
//     workgroup sum.
#include "apex_amd/attn_api.h"
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"
#include "apex_amd/mfma.h"

namespace apex_amd {
namespace attn {

using namespace mfma;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

template <int D>
struct Geo {
  static constexpr int KSTR = D + 8;                 // row-read images (16-B slot shift per row)
  static constexpr int TSTR = (D == 32) ? 96 : D + 32;  // transposed-read images (64/192-B bank offset per row)
  static constexpr int NKK = D / 16;                 // 16-deep k steps over d
  static constexpr int NDT = D / 32;                 // 32-wide d tiles
};

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// Counter-based dropout decision; mirrored in python (apex.ops.attention.dropout_keep_mask).
// One 32-bit hash per (batch*head, query, key pair k >> 1): the even key of the pair tests the low
// 16 bits against t16 = p * 65536, the odd key the high 16 bits.  A hash per pair instead of per
// element halves the integer work (two quarter-rate v_mul_lo_u32 per mix32), which set the cost
// of dropout in every attention kernel: the (bh, q) prefix is per row, and the two keys of a pair
// sit in one lane (forward, dQ: key across the accumulator registers) or in lanes l, l ^ 1 (dK/dV:
// key on the lane; each lane hashes half the rows and swaps them with its neighbour by DPP).
__device__ __forceinline__ uint32_t drop_row(uint32_t seed_mix, uint32_t bh, uint32_t q) {
  return mix32(mix32(seed_mix ^ (bh * 0x9E3779B9u)) ^ (q * 0x85EBCA6Bu));
}
__device__ __forceinline__ uint32_t drop_pair(uint32_t row, uint32_t k) {
  return mix32(row ^ ((k >> 1) * 0xC2B2AE35u));
}
__device__ __forceinline__ uint32_t drop_bits(uint32_t h, uint32_t k) { return (k & 1u) ? (h >> 16) : (h & 0xFFFFu); }
__device__ __forceinline__ uint32_t drop_t16(float p) { return (uint32_t)fminf(p * 65536.f, 65536.f); }
// 1 / keep rate of the quantised test: exactly (65536 - t16) / 65536 of the 16-bit values survive,
// so scaling by 1 / (1 - p) would bias the expected activation by (1 - p) 65536 / (65536 - t16)
__device__ __forceinline__ float drop_inv_keep(float p) {
  const uint32_t t = drop_t16(p);
  return t < 65536u ? 65536.f / (float)(65536u - t) : 0.f;
}
// neighbour lane's value (lanes l, l ^ 1: DPP quad_perm [1, 0, 3, 2])
__device__ __forceinline__ uint32_t swap_pair_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
__host__ __device__ inline uint32_t seed_mix_of(uint64_t seed, uint64_t offset) {
  uint32_t x = (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x27d4eb2du) ^ ((uint32_t)offset * 0x165667b1u) ^
               ((uint32_t)(offset >> 32) * 0xd3a2646cu);
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// host offset + the device RNG step (graph-safe dropout, AttnArgs::rng_step)
__device__ __forceinline__ uint64_t drop_offset(const AttnArgs& a) {
  return a.offset + (a.rng_step ? ((uint64_t)(*a.rng_step) << 32) : 0ull);
}

// v_exp_f32 directly (inputs here are <= 0 or -inf; no denormal range reduction needed)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// reductions over the lane pair (l, l ^ 32) of a 32x32 accumulator column: v_permlane32_swap
// exchanges the two wave halves in the VALU (no LDS round trip as with ds_bpermute); both lanes of
// a pair combine the same two values in the same order, so they agree bitwise
__device__ __forceinline__ float swap32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float swap32_add(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

struct Seq {
  int64_t qrow0, krow0;  // token-space base row (side buffers)
  int64_t qoff, koff;    // element offset of the sequence start for the batch stride / varlen row
  int lq, lk;
};

__device__ __forceinline__ void seq_of(const AttnArgs& a, int b, int64_t q_sb, int64_t q_ss, int64_t k_sb,
                                       int64_t k_ss, Seq& s) {
  if (a.cu_q != nullptr) {
    const int c0 = a.cu_q[b];
    s.qrow0 = c0;
    s.lq = a.cu_q[b + 1] - c0;
    s.qoff = (int64_t)c0 * q_ss;
  } else {
    s.qrow0 = (int64_t)b * a.sq;
    s.lq = a.sq;
    s.qoff = (int64_t)b * q_sb;
  }
  if (a.cu_k != nullptr) {
    const int c0 = a.cu_k[b];
    s.krow0 = c0;
    s.lk = a.cu_k[b + 1] - c0;
    s.koff = (int64_t)c0 * k_ss;
  } else {
    s.krow0 = (int64_t)b * a.sk;
    s.lk = a.sk;
    s.koff = (int64_t)b * k_sb;
  }
}

__device__ __forceinline__ int64_t tensor_off(const AttnTensor& t, const Seq& s, bool is_q, bool varlen, int b) {
  // offset of the (batch, seq=0, head=0) element for tensor t sharing the q- or k-side sequence map
  if (varlen) return (is_q ? s.qrow0 : s.krow0) * t.ss;
  return (int64_t)b * t.sb;
}

// XCD-aware workgroup order: the hardware deals consecutive workgroups round-robin over the 8
// XCDs (private L2 each); remapping the linear id so every XCD gets a contiguous chunk keeps the
// query blocks of one (batch, head) — which all read the same K / V (or the key blocks that all
// read the same Q / dO) — on one L2 (bijective for any grid size).
__device__ __forceinline__ void xcd_remap(int& bx, int& by, int& bz) {
  const int gx = gridDim.x, gy = gridDim.y;
  const int n = gx * gy * gridDim.z;
  const int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int xcd = lin & 7, i = lin >> 3, q = n >> 3, r = n & 7;
  const int nl = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + i;
  bx = nl % gx;
  by = (nl / gx) % gy;
  bz = nl / (gx * gy);
}

// =============================================================================================
// forward
// =============================================================================================
// QF query fragments (32 queries each) per wave: a block covers 128 * QF queries.  QF = 2 feeds
// every K / V fragment read from LDS into two MFMAs (half the LDS traffic per FLOP) at the cost
// of one wave per SIMD for d = 128.
// LO = true: one resident block less than the default (more registers per lane, no spills)
template <int D, int MODE, int QF, bool LO>
constexpr int fwd_occupancy() {
  constexpr bool PLAIN = MODE == 0;
  constexpr int base = QF == 2 ? (D == 128 ? 1 : 2)
                               : ((D == 128 && !PLAIN) ? 1 : ((D <= 64 && MODE <= 1) ? 3 : 2));
  return LO && base > 1 ? base - 1 : base;
}

// MODE: 0 = PLAIN (no bias, no dropout), 1 = dropout without bias, 2 = bias (+ dropout); the
// variants compile out what they do not use (register pressure of the element loops)
template <typename T, int D, int MODE, int QF, bool LO>
__global__ void __launch_bounds__(256, (fwd_occupancy<D, MODE, QF, LO>())) fwd_kernel(const AttnArgs a) {
  int bx, by, bz;
  xcd_remap(bx, by, bz);
  using G = Geo<D>;
  constexpr int BN = 64, KSTR = G::KSTR, VSTR = G::TSTR, NKK = G::NKK, NDT = G::NDT;
  constexpr int KT = BN * KSTR, VT = BN * VSTR;
  constexpr int CPR = D / 8;                 // 16-B chunks per row
  constexpr int CPT = BN * CPR / 256;        // chunks per thread per tensor (D >= 32 -> >= 1)
  constexpr int QB = 128 * QF;               // queries per block
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  auto kbuf = [&](int i) { return lds + i * (KT + VT); };
  auto vbuf = [&](int i) { return lds + i * (KT + VT) + KT; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h2 = lane >> 5, ql = lane & 31;
  const int hq = by, b = bz;
  const int hk = hq / (a.h / a.h_k);
  Seq sq;
  seq_of(a, b, a.q.sb, a.q.ss, a.k.sb, a.k.ss, sq);
  // causal: workgroup x also runs block n-1-x (work per block grows / shrinks linearly with x), so
  // every workgroup does the same number of tiles
  const int nblk = (a.sq + QB - 1) / QB;
  for (int pass = 0; pass < (a.causal ? 2 : 1); ++pass) {
    const int blk = pass == 0 ? (int)bx : nblk - 1 - (int)bx;
    if (pass == 1 && blk <= (int)bx) break;
    const int q_start = blk * QB;
    if (q_start >= sq.lq) continue;  // uniform over the workgroup
    const bool varq = a.cu_q != nullptr, vark = a.cu_k != nullptr;
    const uint16_t* qp = (const uint16_t*)a.q.p + tensor_off(a.q, sq, true, varq, b) + (int64_t)hq * a.q.sh;
    const uint16_t* kp = (const uint16_t*)a.k.p + tensor_off(a.k, sq, false, vark, b) + (int64_t)hk * a.k.sh;
    const uint16_t* vp = (const uint16_t*)a.v.p + tensor_off(a.v, sq, false, vark, b) + (int64_t)hk * a.v.sh;
    T* op = (T*)a.o.p + tensor_off(a.o, sq, true, varq, b) + (int64_t)hq * a.o.sh;

    const int wq0 = q_start + wave * 32 * QF;  // first query of this wave
    int myq[QF];
    bool qvalid[QF];
    s16x8 qf[QF][NKK];
    #pragma unroll
    for (int f = 0; f < QF; ++f) {
      myq[f] = wq0 + 32 * f + ql;
      qvalid[f] = myq[f] < sq.lq;
      #pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        if (qvalid[f]) qf[f][kk] = *reinterpret_cast<const s16x8*>(qp + (int64_t)myq[f] * a.q.ss + kk * 16 + 8 * h2);
        else
          #pragma unroll
          for (int j = 0; j < 8; ++j) qf[f][kk][j] = 0;
      }
    }

    int k_end = sq.lk;
    if (a.causal) k_end = min(k_end, q_start + QB);
    const int nkb = (k_end + BN - 1) / BN;

    uint4 rk[CPT], rv[CPT];
    auto gload = [&](int kb0) {
      #pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int ch = tid + 256 * i, row = ch / CPR, col = (ch % CPR) * 8;
        const int key = kb0 + row;
        const bool ok = key < sq.lk;
        rk[i] = ok ? *reinterpret_cast<const uint4*>(kp + (int64_t)key * a.k.ss + col) : make_uint4(0, 0, 0, 0);
        rv[i] = ok ? *reinterpret_cast<const uint4*>(vp + (int64_t)key * a.v.ss + col) : make_uint4(0, 0, 0, 0);
      }
    };
    auto lstore = [&](int buf) {
      #pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int ch = tid + 256 * i, row = ch / CPR, col = (ch % CPR) * 8;
        *reinterpret_cast<uint4*>(kbuf(buf) + row * KSTR + col) = rk[i];
        *reinterpret_cast<uint4*>(vbuf(buf) + row * VSTR + col) = rv[i];
      }
    };

    f32x16 o[QF][NDT];
    float m_i[QF], l_i[QF];
    #pragma unroll
    for (int f = 0; f < QF; ++f) {
      m_i[f] = -INFINITY;
      l_i[f] = 0.f;
      #pragma unroll
      for (int i = 0; i < NDT; ++i) o[f][i] = zero16();
    }
    const float c = a.scale * kLog2e;
    const float inv_scale = 1.f / a.scale;
    const bool dropout = MODE >= 1 && a.p_drop > 0.f;  // MODE 0: no dropout (compiled out)
    const uint32_t thresh = drop_t16(a.p_drop);
    const float inv_keep = dropout ? drop_inv_keep(a.p_drop) : 1.f;
    const uint32_t smix = seed_mix_of(a.seed, drop_offset(a));
    const uint32_t bh = (uint32_t)(b * a.h + hq);
    uint32_t drow[QF];
    #pragma unroll
    for (int f = 0; f < QF; ++f) drow[f] = dropout ? drop_row(smix, bh, (uint32_t)myq[f]) : 0u;
    const float* biasb = (MODE == 2 && a.bias) ? a.bias + (int64_t)b * a.bias_sb + (int64_t)hq * a.bias_sh : nullptr;

    if (nkb > 0) {
      gload(0);
      lstore(0);
    }
    __syncthreads();
    for (int it = 0; it < nkb; ++it) {
      const int cur = it & 1, kb0 = it * BN;
      const bool more = it + 1 < nkb;
      if (more) gload(kb0 + BN);
      const uint16_t* Kl = kbuf(cur);
      const uint16_t* Vl = vbuf(cur);

      // S^T[key][q] = K Q^T: every K fragment read feeds QF MFMAs
      f32x16 sacc[QF][2];
      #pragma unroll
      for (int f = 0; f < QF; ++f) sacc[f][0] = sacc[f][1] = zero16();
      #pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const s16x8 a0 = frag_rows<KSTR>(Kl, 0, kk, lane);
        const s16x8 a1 = frag_rows<KSTR>(Kl, 32, kk, lane);
        #pragma unroll
        for (int f = 0; f < QF; ++f) {
          sacc[f][0] = mma<T>(a0, qf[f][kk], sacc[f][0]);
          sacc[f][1] = mma<T>(a1, qf[f][kk], sacc[f][1]);
        }
      }
      const bool need_mask = (kb0 + BN > sq.lk) || (a.causal && kb0 + BN - 1 > wq0) || biasb != nullptr;
      // probabilities are packed to 16-bit right away (P fragments), so the fp32 scores of one
      // query fragment are dead before the next fragment's softmax starts
      s16x8 pf[QF][2][2];
      #pragma unroll
      for (int f = 0; f < QF; ++f) {
        // scores stay in raw Q.K units until the exponent: max over the raw values (c > 0, so
        // fl(c * max) == max(fl(c * s))) and p = exp2(fma(s, c, -m)) — one VALU op per score
        // less than scaling first; the bias is added in raw units (bias / scale)
        float x[1][2][16];
        #pragma unroll
        for (int t = 0; t < 2; ++t)
          #pragma unroll
          for (int r = 0; r < 16; ++r) x[0][t][r] = sacc[f][t][r];
        if (need_mask) {
          // key-contiguous bias over a whole tile: the lane's 32 keys are 8 runs of 4 (crow), so 8
          // 16-byte loads instead of 32 scalar ones (BERT's key-padding mask: the forward ran 2.4x
          // the bias-free kernel, profiles/r06/pmc_attn_r06.md)
          const bool bvec = biasb != nullptr && a.bias_sk == 1 && kb0 + BN <= sq.lk &&
                            ((reinterpret_cast<uintptr_t>(biasb) | (uintptr_t)(a.bias_sq * 4)) & 15) == 0;
          const float* brow = bvec ? biasb + (int64_t)(qvalid[f] ? myq[f] : 0) * a.bias_sq + kb0 + 4 * h2 : nullptr;
          #pragma unroll
          for (int t = 0; t < 2; ++t)
            #pragma unroll
            for (int i = 0; i < 4; ++i) {
              // one 4-key run at a time: 4 live registers (all 32 values at once spilled)
              float4 q4 = make_float4(0.f, 0.f, 0.f, 0.f);
              if (bvec) q4 = *reinterpret_cast<const float4*>(brow + 32 * t + 8 * i);
              #pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int r = 4 * i + j;
                const int key = kb0 + 32 * t + crow(r, h2);
                const bool ok = key < sq.lk && (!a.causal || key <= myq[f]);
                float v = x[0][t][r];
                if (biasb != nullptr && ok && qvalid[f]) {
                  const float bvv = j == 0 ? q4.x : j == 1 ? q4.y : j == 2 ? q4.z : q4.w;
                  v += (bvec ? bvv : biasb[(int64_t)myq[f] * a.bias_sq + (int64_t)key * a.bias_sk]) * inv_scale;
                }
                x[0][t][r] = ok ? v : -INFINITY;
              }
            }
        }
        float mx = -INFINITY;
        #pragma unroll
        for (int t = 0; t < 2; ++t)
          #pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, x[0][t][r]);
        mx = swap32_max(mx) * c;
        const float m_new = fmaxf(m_i[f], mx);
        const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
        const float alpha = fast_exp2(m_i[f] - m_use);
        float ls = 0.f;
        #pragma unroll
        for (int t = 0; t < 2; ++t)
          #pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float pr = fast_exp2(__builtin_fmaf(x[0][t][r], c, -m_use));
            ls += pr;
            x[0][t][r] = pr;
          }
        ls = swap32_add(ls);
        l_i[f] = l_i[f] * alpha + ls;
        m_i[f] = m_new;
        // skip the O rescale when no lane's running max moved (after the first tiles it rarely does;
        // measured equal or faster at every head dim: profiles/kernels_attn_r01e.jsonl lazy0/lazy1)
        if (__any(alpha != 1.f)) {
          #pragma unroll
          for (int i = 0; i < NDT; ++i)
            #pragma unroll
            for (int r = 0; r < 16; ++r) o[f][i][r] *= alpha;
        }
        if (dropout) {
          // registers r, r + 1 (r even) hold keys k, k + 1 of one pair: one hash for both
          #pragma unroll
          for (int t = 0; t < 2; ++t)
            #pragma unroll
            for (int r = 0; r < 16; r += 2) {
              const uint32_t hp = drop_pair(drow[f], (uint32_t)(kb0 + 32 * t + crow(r, h2)));
              x[0][t][r] *= (hp & 0xFFFFu) >= thresh ? inv_keep : 0.f;
              x[0][t][r + 1] *= (hp >> 16) >= thresh ? inv_keep : 0.f;
            }
        }
        #pragma unroll
        for (int t = 0; t < 2; ++t)
          #pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) pf[f][t][s2] = pack8<T>(&x[0][t][8 * s2]);
      }
      // O^T[d][q] += V^T[d][key] P^T[key][q]: every V fragment read feeds QF MFMAs
      #pragma unroll
      for (int t = 0; t < 2; ++t)
        #pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int klo = 32 * t + 16 * s2 + 4 * h2;
          #pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const s16x8 vf = frag_tr<VSTR>(Vl, 32 * dt, klo, klo + 8, lane);
            #pragma unroll
            for (int f = 0; f < QF; ++f) o[f][dt] = mma<T>(vf, pf[f][t][s2], o[f][dt]);
          }
        }
      if (more) lstore(cur ^ 1);
      __syncthreads();
    }

    #pragma unroll
    for (int f = 0; f < QF; ++f) {
      if (!qvalid[f]) continue;
      const float inv_l = l_i[f] > 0.f ? 1.f / l_i[f] : 0.f;
      T* orow = op + (int64_t)myq[f] * a.o.ss;
      #pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
        #pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 32 * dt + 8 * g4 + 4 * h2;
          uint32_t w0 = (uint32_t)from_f<T>(o[f][dt][4 * g4] * inv_l).x |
                        ((uint32_t)from_f<T>(o[f][dt][4 * g4 + 1] * inv_l).x << 16);
          uint32_t w1 = (uint32_t)from_f<T>(o[f][dt][4 * g4 + 2] * inv_l).x |
                        ((uint32_t)from_f<T>(o[f][dt][4 * g4 + 3] * inv_l).x << 16);
          *reinterpret_cast<uint2*>(orow + d0) = make_uint2(w0, w1);
        }
      if (h2 == 0 && a.lse != nullptr)
        a.lse[(int64_t)hq * a.rows_q + sq.qrow0 + myq[f]] =
            l_i[f] > 0.f ? (m_i[f] + log2f(l_i[f])) * kLn2 : INFINITY;
    }
    __syncthreads();  // LDS is reused by the paired block
  }
}

// =============================================================================================
// backward
// =============================================================================================
// delta[h][row] = sum_d dO * O   (D/8 lanes per row)
template <typename T, int D>
__global__ void __launch_bounds__(256) bwd_delta_kernel(const AttnBwdArgs ba) {
  const AttnArgs& a = ba.f;
  constexpr int LPR = D / 8, RPB = 256 / LPR;
  const int hq = blockIdx.y, b = blockIdx.z;
  Seq sq;
  seq_of(a, b, a.q.sb, a.q.ss, a.k.sb, a.k.ss, sq);
  const int q = blockIdx.x * RPB + threadIdx.x / LPR, c8 = (threadIdx.x % LPR) * 8;
  float acc = 0.f;
  const bool varq = a.cu_q != nullptr;
  if (q < sq.lq) {
    const T* o = (const T*)a.o.p + tensor_off(a.o, sq, true, varq, b) + (int64_t)hq * a.o.sh + (int64_t)q * a.o.ss;
    const T* g = (const T*)ba.dout.p + tensor_off(ba.dout, sq, true, varq, b) + (int64_t)hq * ba.dout.sh +
                 (int64_t)q * ba.dout.ss;
    float ov[8], gv[8];
    Vec8<T>::load(ov, o + c8);
    Vec8<T>::load(gv, g + c8);
    #pragma unroll
    for (int e = 0; e < 8; ++e) acc += ov[e] * gv[e];
  }
  #pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (q < sq.lq && (threadIdx.x % LPR) == 0) ba.delta[(int64_t)hq * a.rows_q + sq.qrow0 + q] = acc;
}

template <typename T, int D, bool PLAIN>
__global__ void __launch_bounds__(256, 1) bwd_kernel(const AttnBwdArgs ba) {
  const AttnArgs& a = ba.f;
  using G = Geo<D>;
  constexpr int BK = 128, QB = 32, NKK = G::NKK, NDT = G::NDT;
  constexpr int KLSTR = G::TSTR;   // K image: transposed reads for dQ
  constexpr int QSTR = G::KSTR;    // Q / dO images: row reads (S, dP) and transposed reads (dK, dV)
  constexpr int DSSTR = BK + 8;    // dS image: row reads for dQ
  constexpr int CPR = D / 8;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* Kl = lds;
  uint16_t* Ql = Kl + BK * KLSTR;
  uint16_t* dOl = Ql + QB * QSTR;
  uint16_t* dSl = dOl + QB * QSTR;
  float* lse_l = reinterpret_cast<float*>(dSl + QB * DSSTR);
  float* del_l = lse_l + QB;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h2 = lane >> 5, ql = lane & 31;
  const int hk = blockIdx.y, b = blockIdx.z;
  Seq sq;
  seq_of(a, b, a.q.sb, a.q.ss, a.k.sb, a.k.ss, sq);
  const int k_start = blockIdx.x * BK;
  if (k_start >= sq.lk) return;
  const bool varq = a.cu_q != nullptr, vark = a.cu_k != nullptr;
  const uint16_t* kp = (const uint16_t*)a.k.p + tensor_off(a.k, sq, false, vark, b) + (int64_t)hk * a.k.sh;
  const uint16_t* vp = (const uint16_t*)a.v.p + tensor_off(a.v, sq, false, vark, b) + (int64_t)hk * a.v.sh;

  // K tile of the workgroup -> LDS (transposed reads for dQ); own 32 keys' K, V -> registers
  for (int ch = tid; ch < BK * CPR; ch += 256) {
    const int row = ch / CPR, col = (ch % CPR) * 8, key = k_start + row;
    *reinterpret_cast<uint4*>(Kl + row * KLSTR + col) =
        key < sq.lk ? *reinterpret_cast<const uint4*>(kp + (int64_t)key * a.k.ss + col) : make_uint4(0, 0, 0, 0);
  }
  const int mykey = k_start + wave * 32 + ql;
  const bool kvalid = mykey < sq.lk;
  s16x8 kf[NKK], vf[NKK];
  #pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    if (kvalid) {
      kf[kk] = *reinterpret_cast<const s16x8*>(kp + (int64_t)mykey * a.k.ss + kk * 16 + 8 * h2);
      vf[kk] = *reinterpret_cast<const s16x8*>(vp + (int64_t)mykey * a.v.ss + kk * 16 + 8 * h2);
    } else {
      #pragma unroll
      for (int j = 0; j < 8; ++j) kf[kk][j] = vf[kk][j] = 0;
    }
  }

  f32x16 dk[NDT], dv[NDT];
  #pragma unroll
  for (int i = 0; i < NDT; ++i) dk[i] = dv[i] = zero16();
  const float c = a.scale * kLog2e;
  const bool dropout = !PLAIN && a.p_drop > 0.f;  // PLAIN: no bias, no dropout (compiled out)
  const uint32_t thresh = drop_t16(a.p_drop);
  const float inv_keep = dropout ? drop_inv_keep(a.p_drop) : 1.f;
  const uint32_t smix = seed_mix_of(a.seed, drop_offset(a));
  const int group = a.h / a.h_k;
  // dQ tile ownership: d-tile dtq, key part kpart of kparts (NDT * kparts == 4 waves)
  constexpr int KPARTS = 4 / NDT, KPL = BK / KPARTS;
  const int dtq = wave % NDT, kpart = wave / NDT;

  for (int hq = hk * group; hq < (hk + 1) * group; ++hq) {
    const uint16_t* qp = (const uint16_t*)a.q.p + tensor_off(a.q, sq, true, varq, b) + (int64_t)hq * a.q.sh;
    const uint16_t* gp =
        (const uint16_t*)ba.dout.p + tensor_off(ba.dout, sq, true, varq, b) + (int64_t)hq * ba.dout.sh;
    const float* lse_h = a.lse + (int64_t)hq * a.rows_q + sq.qrow0;
    const float* del_h = ba.delta + (int64_t)hq * a.rows_q + sq.qrow0;
    float* dq_h = ba.dq_acc + (sq.qrow0 * a.h + hq) * D;
    const uint32_t bh = (uint32_t)(b * a.h + hq);
    const float* biash = (!PLAIN && a.bias) ? a.bias + (int64_t)b * a.bias_sb + (int64_t)hq * a.bias_sh : nullptr;
    const int q_begin = a.causal ? (k_start / QB) * QB : 0;
    // next Q / dO slice is fetched into registers under the current slice's MFMAs and written
    // to LDS after the dQ phase (issue-early / write-late), so no global latency is exposed
    constexpr int QCH = QB * CPR, QCPT = (QCH + 255) / 256;
    uint4 pq[QCPT], pg[QCPT];
    float plse = INFINITY, pdel = 0.f;
    auto fetch = [&](int q0n) {
      #pragma unroll
      for (int i = 0; i < QCPT; ++i) {
        const int ch = tid + 256 * i;
        if (ch < QCH) {
          const int row = ch / CPR, col = (ch % CPR) * 8, q = q0n + row;
          const bool ok = q < sq.lq;
          pq[i] = ok ? *reinterpret_cast<const uint4*>(qp + (int64_t)q * a.q.ss + col) : make_uint4(0, 0, 0, 0);
          pg[i] = ok ? *reinterpret_cast<const uint4*>(gp + (int64_t)q * ba.dout.ss + col) : make_uint4(0, 0, 0, 0);
        }
      }
      if (tid < QB) {
        const int q = q0n + tid;
        plse = q < sq.lq ? lse_h[q] : INFINITY;
        pdel = q < sq.lq ? del_h[q] : 0.f;
      }
    };
    auto commit = [&]() {
      #pragma unroll
      for (int i = 0; i < QCPT; ++i) {
        const int ch = tid + 256 * i;
        if (ch < QCH) {
          const int row = ch / CPR, col = (ch % CPR) * 8;
          *reinterpret_cast<uint4*>(Ql + row * QSTR + col) = pq[i];
          *reinterpret_cast<uint4*>(dOl + row * QSTR + col) = pg[i];
        }
      }
      if (tid < QB) {
        lse_l[tid] = plse;
        del_l[tid] = pdel;
      }
    };
    fetch(q_begin);
    commit();
    __syncthreads();
    for (int q0 = q_begin; q0 < sq.lq; q0 += QB) {
      const bool more = q0 + QB < sq.lq;
      if (more) fetch(q0 + QB);

      // S[q][key] and dP[q][key] with the key on the lane
      f32x16 sacc = zero16(), dpacc = zero16();
      #pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const s16x8 aq = frag_rows<QSTR>(Ql, 0, kk, lane);
        sacc = mma<T>(aq, kf[kk], sacc);
        const s16x8 ag = frag_rows<QSTR>(dOl, 0, kk, lane);
        dpacc = mma<T>(ag, vf[kk], dpacc);
      }
      float p[16], ds[16];
      const bool edge = !kvalid || q0 + QB > sq.lq || (a.causal && q0 < k_start + wave * 32 + 32) ||
                        biash != nullptr;
      #pragma unroll
      for (int r = 0; r < 16; ++r) p[r] = sacc[r] * c - lse_l[crow(r, h2)] * kLog2e;
      if (edge) {  // wave-uniform: interior slices run the element loop branch-free
        #pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int q = q0 + crow(r, h2);
          const bool ok = kvalid && q < sq.lq && (!a.causal || mykey <= q);
          float xv = p[r];
          if (biash != nullptr && ok) xv += biash[(int64_t)q * a.bias_sq + (int64_t)mykey * a.bias_sk] * kLog2e;
          p[r] = ok ? xv : -INFINITY;
        }
      }
      #pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = crow(r, h2), q = q0 + qr;
        const float pv = fast_exp2(p[r]);
        float dpv = dpacc[r];
        float pd = pv;
        if (dropout) {
          const float mk =
              drop_bits(drop_pair(drop_row(smix, bh, (uint32_t)q), (uint32_t)mykey), (uint32_t)mykey) >= thresh
                  ? inv_keep : 0.f;
          pd = pv * mk;
          dpv *= mk;
        }
        p[r] = pd;
        ds[r] = pv * (dpv - del_l[qr]);
      }
      // dV^T += dO^T P,  dK^T += Q^T dS   (P / dS straight from registers)
      #pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const s16x8 pf = pack8<T>(&p[8 * s2]);
        const s16x8 dsf = pack8<T>(&ds[8 * s2]);
        const int klo = 16 * s2 + 4 * h2;
        #pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const s16x8 gt = frag_tr<QSTR>(dOl, 32 * dt, klo, klo + 8, lane);
          dv[dt] = mma<T>(gt, pf, dv[dt]);
          const s16x8 qt = frag_tr<QSTR>(Ql, 32 * dt, klo, klo + 8, lane);
          dk[dt] = mma<T>(qt, dsf, dk[dt]);
        }
      }
      // dS -> LDS [q][key]
      #pragma unroll
      for (int r = 0; r < 16; ++r) dSl[crow(r, h2) * DSSTR + wave * 32 + ql] = from_f<T>(ds[r]).x;
      __syncthreads();
      // dQ[q][d] += dS[q][keys] K[keys][d] for this wave's (d tile, key part)
      f32x16 dq = zero16();
      #pragma unroll
      for (int kk = 0; kk < KPL / 16; ++kk) {
        const int kb = kpart * KPL + 16 * kk;
        const s16x8 af = frag_rows<DSSTR>(dSl, 0, kb / 16, lane);
        const s16x8 bf = frag_tr<KLSTR>(Kl, 32 * dtq, kb + 8 * h2, kb + 8 * h2 + 4, lane);
        dq = mma<T>(af, bf, dq);
      }
      #pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = q0 + crow(r, h2);
        if (q < sq.lq) unsafeAtomicAdd(dq_h + (int64_t)q * a.h * D + 32 * dtq + ql, dq[r] * a.scale);
      }
      if (more) commit();
      __syncthreads();
    }
  }

  if (kvalid) {
    T* dkp = (T*)ba.dk.p + tensor_off(ba.dk, sq, false, vark, b) + (int64_t)hk * ba.dk.sh + (int64_t)mykey * ba.dk.ss;
    T* dvp = (T*)ba.dv.p + tensor_off(ba.dv, sq, false, vark, b) + (int64_t)hk * ba.dv.sh + (int64_t)mykey * ba.dv.ss;
    #pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
      #pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * h2;
        const float s = a.scale;
        uint32_t k0 = (uint32_t)from_f<T>(dk[dt][4 * g4] * s).x | ((uint32_t)from_f<T>(dk[dt][4 * g4 + 1] * s).x << 16);
        uint32_t k1 = (uint32_t)from_f<T>(dk[dt][4 * g4 + 2] * s).x | ((uint32_t)from_f<T>(dk[dt][4 * g4 + 3] * s).x << 16);
        *reinterpret_cast<uint2*>(dkp + d0) = make_uint2(k0, k1);
        uint32_t v0 = (uint32_t)from_f<T>(dv[dt][4 * g4]).x | ((uint32_t)from_f<T>(dv[dt][4 * g4 + 1]).x << 16);
        uint32_t v1 = (uint32_t)from_f<T>(dv[dt][4 * g4 + 2]).x | ((uint32_t)from_f<T>(dv[dt][4 * g4 + 3]).x << 16);
        *reinterpret_cast<uint2*>(dvp + d0) = make_uint2(v0, v1);
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Split backward (default): dK/dV and dQ in two atomic-free kernels.
//
// The fused kernel above sums dQ over key blocks with fp32 global atomics: (sk / 128) * sq * h * d
// * 4 B of atomic traffic (2 GB at b8 h16 s2048 d128), and the chip retires atomics at only
// ~1.3 TB/s of added bytes (MI355X_MICROARCH.md, atomics price list) — that, not the MFMAs, set
// its time.  Recomputing S and dP once more in a query-major kernel costs 2 extra s^2 d GEMMs
// (7 instead of 5) but removes every atomic, the fp32 dQ buffer, its memset and the convert pass.
// ---------------------------------------------------------------------------------------------

// XOR-swizzled Q / dO slice images of the dK/dV kernel (head dim 64 / 128): rows are D elements
// long with no padding, and 16-byte chunk c of row r is stored at chunk c ^ swz(r).  The padded
// (D + 8) layout kept the 32-row fragment reads conflict-free but put two of the four rows a
// 16-lane ds_read_b64_tr_b16 touches on the same banks (22 % LDS bank-conflict cycles,
// profiles/pmc_kernels_r03.md); the swizzle gives both the row reads (16 rows, one chunk) and the
// transposed reads (4 rows x 4 chunks per 32 lanes) 16 distinct 16-byte bank slots.
//   D = 128 (one row per 256-B bank line): swz(r) = ((r & 3) << 2) | ((r >> 2) & 3)
//   D =  64 (two rows per line):           swz(r) = f((r >> 1) & 7), f(j) = ((j & 1) << 2) | (j >> 1)
template <int D>
__device__ __forceinline__ int qswz(int r) {
  if constexpr (D == 128) return ((r & 3) << 2) | ((r >> 2) & 3);
  else {
    const int j = (r >> 1) & 7;
    return ((j & 1) << 2) | (j >> 1);
  }
}

template <int D>
__device__ __forceinline__ s16x8 frag_rows_sw(const uint16_t* lds, int kk, int lane) {
  const int row = lane & 31;
  const int c = (2 * kk + (lane >> 5)) ^ qswz<D>(row);
  return *reinterpret_cast<const s16x8*>(lds + row * D + 8 * c);
}

template <int D>
__device__ __forceinline__ s16x8 frag_tr_sw(const uint16_t* lds, int colbase, int klo, int khi, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int col = colbase + 16 * (g & 1) + 4 * p;
  const int ck = col >> 3, off = col & 7;
  const int r0 = klo + q, r1 = khi + q;
  const s16x4 lo = tr_read(lds + r0 * D + ((ck ^ qswz<D>(r0)) << 3) + off);
  const s16x4 hi = tr_read(lds + r1 * D + ((ck ^ qswz<D>(r1)) << 3) + off);
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int D>
constexpr bool dkdv_swz() {
  return D == 64 || D == 128;
}

// dK, dV: one workgroup = 4 waves = 128 keys (K, V of the wave's 32 keys in registers); 32-query
// slices of Q / dO (+ lse, delta) double-buffered in LDS, one barrier per slice.
template <typename T, int D, int MODE, int QS>
__global__ void __launch_bounds__(256, (D == 128 ? 1 : 2)) bwd_dkdv_kernel(const AttnBwdArgs ba) {
  int bx, by, bz;
  xcd_remap(bx, by, bz);
  const AttnArgs& a = ba.f;
  using G = Geo<D>;
  constexpr int BK = 128, QB = QS, NKK = G::NKK, NDT = G::NDT;  // QB queries per LDS slice
  constexpr bool SW = dkdv_swz<D>();
  constexpr int QSTR = SW ? D : G::KSTR;  // row reads (S, dP) and transposed reads (dK, dV)
  constexpr int CPR = D / 8;
  // Q, dO images + lse, delta (fp32) + per-row dropout hash prefix (u32), in 16-bit units
  constexpr int SLICE = 2 * QB * QSTR + 6 * QB;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  auto Ql = [&](int i) { return lds + i * SLICE; };
  auto dOl = [&](int i) { return lds + i * SLICE + QB * QSTR; };
  auto lse_l = [&](int i) { return reinterpret_cast<float*>(lds + i * SLICE + 2 * QB * QSTR); };
  auto del_l = [&](int i) { return lse_l(i) + QB; };
  auto hq_l = [&](int i) { return reinterpret_cast<uint32_t*>(del_l(i) + QB); };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h2 = lane >> 5, ql = lane & 31;
  const int hk = by, b = bz;
  Seq sq;
  seq_of(a, b, a.q.sb, a.q.ss, a.k.sb, a.k.ss, sq);
  // causal: workgroup x also runs block n-1-x (work per block grows / shrinks linearly with x), so
  // every workgroup does the same number of tiles
  const int nblk = (a.sk + BK - 1) / BK;
  for (int pass = 0; pass < (a.causal ? 2 : 1); ++pass) {
    const int blk = pass == 0 ? (int)bx : nblk - 1 - (int)bx;
    if (pass == 1 && blk <= (int)bx) break;
    const int k_start = blk * BK;
    if (k_start >= sq.lk) continue;  // uniform over the workgroup
    const bool varq = a.cu_q != nullptr, vark = a.cu_k != nullptr;
    const uint16_t* kp = (const uint16_t*)a.k.p + tensor_off(a.k, sq, false, vark, b) + (int64_t)hk * a.k.sh;
    const uint16_t* vp = (const uint16_t*)a.v.p + tensor_off(a.v, sq, false, vark, b) + (int64_t)hk * a.v.sh;
    const int mykey = k_start + wave * 32 + ql;
    const bool kvalid = mykey < sq.lk;
    s16x8 kf[NKK], vf[NKK];
    #pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      if (kvalid) {
        kf[kk] = *reinterpret_cast<const s16x8*>(kp + (int64_t)mykey * a.k.ss + kk * 16 + 8 * h2);
        vf[kk] = *reinterpret_cast<const s16x8*>(vp + (int64_t)mykey * a.v.ss + kk * 16 + 8 * h2);
      } else {
        #pragma unroll
        for (int j = 0; j < 8; ++j) kf[kk][j] = vf[kk][j] = 0;
      }
    }
    f32x16 dk[NDT], dv[NDT];
    #pragma unroll
    for (int i = 0; i < NDT; ++i) dk[i] = dv[i] = zero16();
    const float c = a.scale * kLog2e;
    const bool dropout = MODE >= 1 && a.p_drop > 0.f;  // MODE 0: no dropout (compiled out)
    const uint32_t thresh = drop_t16(a.p_drop);
    const float inv_keep = dropout ? drop_inv_keep(a.p_drop) : 1.f;
    const uint32_t smix = seed_mix_of(a.seed, drop_offset(a));
    const int group = a.h / a.h_k;
    constexpr int QCH = QB * CPR, QCPT = (QCH + 255) / 256;

    for (int hq = hk * group; hq < (hk + 1) * group; ++hq) {
      const uint16_t* qp = (const uint16_t*)a.q.p + tensor_off(a.q, sq, true, varq, b) + (int64_t)hq * a.q.sh;
      const uint16_t* gp =
          (const uint16_t*)ba.dout.p + tensor_off(ba.dout, sq, true, varq, b) + (int64_t)hq * ba.dout.sh;
      const float* lse_h = a.lse + (int64_t)hq * a.rows_q + sq.qrow0;
      const float* del_h = ba.delta + (int64_t)hq * a.rows_q + sq.qrow0;
      const uint32_t bh = (uint32_t)(b * a.h + hq);
      const float* biash = (MODE == 2 && a.bias) ? a.bias + (int64_t)b * a.bias_sb + (int64_t)hq * a.bias_sh : nullptr;
      // a key-only bias (bias_sq 0: key padding) is one value per lane (its key) for the whole head
      const bool bkey_ok = biash != nullptr && a.bias_sq == 0 && kvalid;
      const float bkey = bkey_ok ? biash[(int64_t)mykey * a.bias_sk] * kLog2e : 0.f;
      const int q_begin = a.causal ? (k_start / QB) * QB : 0;
      uint4 pq[QCPT], pg[QCPT];
      float plse = INFINITY, pdel = 0.f;
      uint32_t phq = 0;
      const uint32_t hbh = mix32(smix ^ (bh * 0x9E3779B9u));
      auto fetch = [&](int q0n) {
        #pragma unroll
        for (int i = 0; i < QCPT; ++i) {
          const int ch = tid + 256 * i;
          if (ch < QCH) {
            const int row = ch / CPR, col = (ch % CPR) * 8, q = q0n + row;
            const bool ok = q < sq.lq;
            pq[i] = ok ? *reinterpret_cast<const uint4*>(qp + (int64_t)q * a.q.ss + col) : make_uint4(0, 0, 0, 0);
            pg[i] = ok ? *reinterpret_cast<const uint4*>(gp + (int64_t)q * ba.dout.ss + col) : make_uint4(0, 0, 0, 0);
          }
        }
        if (tid < QB) {
          const int q = q0n + tid;
          plse = q < sq.lq ? lse_h[q] : INFINITY;
          pdel = q < sq.lq ? del_h[q] : 0.f;
          // the (bh, q) part of drop_hash, once per row instead of once per element
          if (dropout) phq = mix32(hbh ^ ((uint32_t)q * 0x85EBCA6Bu));
        }
      };
      auto commit = [&](int buf) {
        #pragma unroll
        for (int i = 0; i < QCPT; ++i) {
          const int ch = tid + 256 * i;
          if (ch < QCH) {
            const int row = ch / CPR;
            // 32-row sub-slices restart the swizzle pattern: row index within the sub-slice
            const int col = SW ? ((ch % CPR) ^ qswz<D>(row & 31)) * 8 : (ch % CPR) * 8;
            *reinterpret_cast<uint4*>(Ql(buf) + row * QSTR + col) = pq[i];
            *reinterpret_cast<uint4*>(dOl(buf) + row * QSTR + col) = pg[i];
          }
        }
        if (tid < QB) {
          lse_l(buf)[tid] = plse * kLog2e;
          del_l(buf)[tid] = pdel;
          if (dropout) hq_l(buf)[tid] = phq;
        }
      };
      // the previous head's last slice ended with a barrier: both buffers are free
      fetch(q_begin);
      commit(0);
      __syncthreads();
      int buf = 0;
      for (int q0 = q_begin; q0 < sq.lq; q0 += QB, buf ^= 1) {
        const bool more = q0 + QB < sq.lq;
        if (more) fetch(q0 + QB);
        // 32-query sub-slices of the LDS slice (QB = 64 halves the barriers / commits per query)
        #pragma unroll
        for (int sub = 0; sub < QB / 32; ++sub) {
        const int q0s = q0 + 32 * sub;
        if (q0s >= sq.lq) break;  // uniform over the workgroup
        const uint16_t* Qb = Ql(buf) + 32 * sub * QSTR;
        const uint16_t* Gb = dOl(buf) + 32 * sub * QSTR;
        const float* lb = lse_l(buf) + 32 * sub;
        const float* db = del_l(buf) + 32 * sub;
        const uint32_t* hb = hq_l(buf) + 32 * sub;
        f32x16 sacc = zero16(), dpacc = zero16();
        #pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          if constexpr (SW) {
            sacc = mma<T>(frag_rows_sw<D>(Qb, kk, lane), kf[kk], sacc);
            dpacc = mma<T>(frag_rows_sw<D>(Gb, kk, lane), vf[kk], dpacc);
          } else {
            sacc = mma<T>(frag_rows<QSTR>(Qb, 0, kk, lane), kf[kk], sacc);
            dpacc = mma<T>(frag_rows<QSTR>(Gb, 0, kk, lane), vf[kk], dpacc);
          }
        }
        float p[16], ds[16];
        const bool edge = !kvalid || q0s + 32 > sq.lq || (a.causal && q0s < k_start + wave * 32 + 32) ||
                          biash != nullptr;
        #pragma unroll
        for (int r = 0; r < 16; ++r) p[r] = sacc[r] * c - lb[crow(r, h2)];
        if (edge) {  // wave-uniform: interior slices run the element loop branch-free
          #pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int q = q0s + crow(r, h2);
            const bool ok = kvalid && q < sq.lq && (!a.causal || mykey <= q);
            float xv = p[r];
            if (biash != nullptr && ok)
              xv += bkey_ok ? bkey : biash[(int64_t)q * a.bias_sq + (int64_t)mykey * a.bias_sk] * kLog2e;
            p[r] = ok ? xv : -INFINITY;
          }
        }
        // dropout: lanes l, l ^ 1 hold keys k, k ^ 1 of one pair and need the same 16 row hashes;
        // each hashes the rows of its own parity (the (bh, q) prefix read from LDS) and takes the
        // other half from its neighbour
        const uint32_t par = (uint32_t)ql & 1u;
        #pragma unroll
        for (int r = 0; r < 16; r += 2) {
          float pv[2], dpv[2], mk[2] = {1.f, 1.f};
          if (dropout) {
            const uint32_t mine = drop_pair(hb[crow(r, h2) + par], (uint32_t)mykey);
            const uint32_t other = swap_pair_lane(mine);
            mk[0] = drop_bits(par ? other : mine, (uint32_t)mykey) >= thresh ? inv_keep : 0.f;
            mk[1] = drop_bits(par ? mine : other, (uint32_t)mykey) >= thresh ? inv_keep : 0.f;
          }
          #pragma unroll
          for (int j = 0; j < 2; ++j) {
            pv[j] = fast_exp2(p[r + j]);
            dpv[j] = dpacc[r + j] * mk[j];
            p[r + j] = pv[j] * mk[j];
            ds[r + j] = pv[j] * (dpv[j] - db[crow(r + j, h2)]);
          }
        }
        #pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const s16x8 pf = pack8<T>(&p[8 * s2]);
          const s16x8 dsf = pack8<T>(&ds[8 * s2]);
          const int klo = 16 * s2 + 4 * h2;
          #pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            if constexpr (SW) {
              dv[dt] = mma<T>(frag_tr_sw<D>(Gb, 32 * dt, klo, klo + 8, lane), pf, dv[dt]);
              dk[dt] = mma<T>(frag_tr_sw<D>(Qb, 32 * dt, klo, klo + 8, lane), dsf, dk[dt]);
            } else {
              dv[dt] = mma<T>(frag_tr<QSTR>(Gb, 32 * dt, klo, klo + 8, lane), pf, dv[dt]);
              dk[dt] = mma<T>(frag_tr<QSTR>(Qb, 32 * dt, klo, klo + 8, lane), dsf, dk[dt]);
            }
          }
        }
        }
        if (more) commit(buf ^ 1);
        __syncthreads();
      }
    }

    if (kvalid) {
      T* dkp = (T*)ba.dk.p + tensor_off(ba.dk, sq, false, vark, b) + (int64_t)hk * ba.dk.sh + (int64_t)mykey * ba.dk.ss;
      T* dvp = (T*)ba.dv.p + tensor_off(ba.dv, sq, false, vark, b) + (int64_t)hk * ba.dv.sh + (int64_t)mykey * ba.dv.ss;
      #pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
        #pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 32 * dt + 8 * g4 + 4 * h2;
          const float s = a.scale;
          uint32_t k0 = (uint32_t)from_f<T>(dk[dt][4 * g4] * s).x | ((uint32_t)from_f<T>(dk[dt][4 * g4 + 1] * s).x << 16);
          uint32_t k1 = (uint32_t)from_f<T>(dk[dt][4 * g4 + 2] * s).x | ((uint32_t)from_f<T>(dk[dt][4 * g4 + 3] * s).x << 16);
          *reinterpret_cast<uint2*>(dkp + d0) = make_uint2(k0, k1);
          uint32_t v0 = (uint32_t)from_f<T>(dv[dt][4 * g4]).x | ((uint32_t)from_f<T>(dv[dt][4 * g4 + 1]).x << 16);
          uint32_t v1 = (uint32_t)from_f<T>(dv[dt][4 * g4 + 2]).x | ((uint32_t)from_f<T>(dv[dt][4 * g4 + 3]).x << 16);
          *reinterpret_cast<uint2*>(dvp + d0) = make_uint2(v0, v1);
        }
    }
    __syncthreads();  // LDS is reused by the paired block
  }
}

// dQ: the forward's structure (one workgroup = 4 waves = 128 queries, 64-key tiles of K / V
// double-buffered in LDS through registers), with Q and dO of the wave's 32 queries in
// registers.  Per tile: S^T = K Q^T and dP^T = V dO^T (query on the lane), P from the saved lse,
// dS = P (dP - delta), then dQ^T += K^T dS^T with dS fed from registers (crow() k order).  K is
// kept as two LDS images: row-read (S) and transposed-read (dQ) paddings differ.
template <typename T, int D, int MODE>
__global__ void __launch_bounds__(256, (D == 128 ? 1 : 2)) bwd_dq_kernel(const AttnBwdArgs ba) {
  int bx, by, bz;
  xcd_remap(bx, by, bz);
  const AttnArgs& a = ba.f;
  using G = Geo<D>;
  constexpr int BN = 64, RSTR = G::KSTR, TSTR = G::TSTR, NKK = G::NKK, NDT = G::NDT;
  constexpr int KT = BN * RSTR, KTT = BN * TSTR, VT = BN * RSTR, TILE = KT + KTT + VT;
  constexpr int CPR = D / 8;
  constexpr int CPT = BN * CPR / 256;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  auto krow = [&](int i) { return lds + i * TILE; };
  auto ktr = [&](int i) { return lds + i * TILE + KT; };
  auto vrow = [&](int i) { return lds + i * TILE + KT + KTT; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h2 = lane >> 5, ql = lane & 31;
  const int hq = by, b = bz;
  const int hk = hq / (a.h / a.h_k);
  Seq sq;
  seq_of(a, b, a.q.sb, a.q.ss, a.k.sb, a.k.ss, sq);
  // causal: heaviest query blocks first (the tail then ends on light blocks); the pairing used by
  // the other kernels would push this one past 256 VGPRs (spills) in its dropout variant
  const int nblk = (a.sq + 127) / 128;
  {
    const int blk = a.causal ? nblk - 1 - (int)bx : (int)bx;
    const int q_start = blk * 128;
    if (q_start >= sq.lq) return;  // uniform over the workgroup
    const bool varq = a.cu_q != nullptr, vark = a.cu_k != nullptr;
    const uint16_t* qp = (const uint16_t*)a.q.p + tensor_off(a.q, sq, true, varq, b) + (int64_t)hq * a.q.sh;
    const uint16_t* gp = (const uint16_t*)ba.dout.p + tensor_off(ba.dout, sq, true, varq, b) + (int64_t)hq * ba.dout.sh;
    const uint16_t* kp = (const uint16_t*)a.k.p + tensor_off(a.k, sq, false, vark, b) + (int64_t)hk * a.k.sh;
    const uint16_t* vp = (const uint16_t*)a.v.p + tensor_off(a.v, sq, false, vark, b) + (int64_t)hk * a.v.sh;
    T* dqp = (T*)ba.dq.p + tensor_off(ba.dq, sq, true, varq, b) + (int64_t)hq * ba.dq.sh;

    const int myq = q_start + wave * 32 + ql;
    const bool qvalid = myq < sq.lq;
    s16x8 qf[NKK], gf[NKK];
    #pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      if (qvalid) {
        qf[kk] = *reinterpret_cast<const s16x8*>(qp + (int64_t)myq * a.q.ss + kk * 16 + 8 * h2);
        gf[kk] = *reinterpret_cast<const s16x8*>(gp + (int64_t)myq * ba.dout.ss + kk * 16 + 8 * h2);
      } else {
        #pragma unroll
        for (int j = 0; j < 8; ++j) qf[kk][j] = gf[kk][j] = 0;
      }
    }
    const float lse2 = qvalid ? a.lse[(int64_t)hq * a.rows_q + sq.qrow0 + myq] * kLog2e : INFINITY;
    const float dlt = qvalid ? ba.delta[(int64_t)hq * a.rows_q + sq.qrow0 + myq] : 0.f;

    int k_end = sq.lk;
    if (a.causal) k_end = min(k_end, q_start + 128);
    const int nkb = (k_end + BN - 1) / BN;

    uint4 rk[CPT], rv[CPT];
    auto gload = [&](int kb0) {
      #pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int ch = tid + 256 * i, row = ch / CPR, col = (ch % CPR) * 8;
        const int key = kb0 + row;
        const bool ok = key < sq.lk;
        rk[i] = ok ? *reinterpret_cast<const uint4*>(kp + (int64_t)key * a.k.ss + col) : make_uint4(0, 0, 0, 0);
        rv[i] = ok ? *reinterpret_cast<const uint4*>(vp + (int64_t)key * a.v.ss + col) : make_uint4(0, 0, 0, 0);
      }
    };
    auto lstore = [&](int buf) {
      #pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int ch = tid + 256 * i, row = ch / CPR, col = (ch % CPR) * 8;
        *reinterpret_cast<uint4*>(krow(buf) + row * RSTR + col) = rk[i];
        *reinterpret_cast<uint4*>(ktr(buf) + row * TSTR + col) = rk[i];
        *reinterpret_cast<uint4*>(vrow(buf) + row * RSTR + col) = rv[i];
      }
    };

    f32x16 dq[NDT];
    #pragma unroll
    for (int i = 0; i < NDT; ++i) dq[i] = zero16();
    const float c = a.scale * kLog2e;
    const bool dropout = MODE >= 1 && a.p_drop > 0.f;  // MODE 0: no dropout (compiled out)
    const uint32_t thresh = drop_t16(a.p_drop);
    const float inv_keep = dropout ? drop_inv_keep(a.p_drop) : 1.f;
    const uint32_t smix = seed_mix_of(a.seed, drop_offset(a));
    const uint32_t bh = (uint32_t)(b * a.h + hq);
    const uint32_t drow = dropout ? drop_row(smix, bh, (uint32_t)myq) : 0u;
    const float* biasp = (MODE == 2 && a.bias) ? a.bias + (int64_t)b * a.bias_sb + (int64_t)hq * a.bias_sh + (int64_t)myq * a.bias_sq
                                : nullptr;

    if (nkb > 0) {
      gload(0);
      lstore(0);
    }
    __syncthreads();
    for (int it = 0; it < nkb; ++it) {
      const int cur = it & 1, kb0 = it * BN;
      const bool more = it + 1 < nkb;
      if (more) gload(kb0 + BN);
      const uint16_t* Kr = krow(cur);
      const uint16_t* Kt = ktr(cur);
      const uint16_t* Vr = vrow(cur);

      f32x16 s[2] = {zero16(), zero16()}, dp[2] = {zero16(), zero16()};
      #pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        s[0] = mma<T>(frag_rows<RSTR>(Kr, 0, kk, lane), qf[kk], s[0]);
        s[1] = mma<T>(frag_rows<RSTR>(Kr, 32, kk, lane), qf[kk], s[1]);
        dp[0] = mma<T>(frag_rows<RSTR>(Vr, 0, kk, lane), gf[kk], dp[0]);
        dp[1] = mma<T>(frag_rows<RSTR>(Vr, 32, kk, lane), gf[kk], dp[1]);
      }
      const bool need_mask = !qvalid || (kb0 + BN > sq.lk) || (a.causal && kb0 + BN - 1 > q_start + wave * 32) ||
                             biasp != nullptr;
      float ds[2][16];
      #pragma unroll
      for (int t = 0; t < 2; ++t)
        #pragma unroll
        for (int r = 0; r < 16; ++r) ds[t][r] = s[t][r] * c - lse2;
      if (need_mask) {  // wave-uniform: the interior tiles run the element loop branch-free
        // key-contiguous bias over a whole tile: one 16-byte run of 4 keys at a time (see the forward)
        const bool bvec = biasp != nullptr && a.bias_sk == 1 && kb0 + BN <= sq.lk && qvalid &&
                          (reinterpret_cast<uintptr_t>(biasp) & 15) == 0;
        #pragma unroll
        for (int t = 0; t < 2; ++t)
          #pragma unroll
          for (int i = 0; i < 4; ++i) {
            float4 q4 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (bvec) q4 = *reinterpret_cast<const float4*>(biasp + kb0 + 4 * h2 + 32 * t + 8 * i);
            #pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = 4 * i + j;
              const int key = kb0 + 32 * t + crow(r, h2);
              const bool ok = qvalid && key < sq.lk && (!a.causal || key <= myq);
              float xv = ds[t][r];
              if (biasp != nullptr && ok) {
                const float bvv = j == 0 ? q4.x : j == 1 ? q4.y : j == 2 ? q4.z : q4.w;
                xv += (bvec ? bvv : biasp[(int64_t)key * a.bias_sk]) * kLog2e;
              }
              ds[t][r] = ok ? xv : -INFINITY;
            }
          }
      }
      #pragma unroll
      for (int t = 0; t < 2; ++t)
        #pragma unroll
        for (int r = 0; r < 16; r += 2) {
          float dpv0 = dp[t][r], dpv1 = dp[t][r + 1];
          if (dropout) {  // registers r, r + 1 hold the two keys of one pair
            const uint32_t hp = drop_pair(drow, (uint32_t)(kb0 + 32 * t + crow(r, h2)));
            dpv0 *= (hp & 0xFFFFu) >= thresh ? inv_keep : 0.f;
            dpv1 *= (hp >> 16) >= thresh ? inv_keep : 0.f;
          }
          ds[t][r] = fast_exp2(ds[t][r]) * (dpv0 - dlt);
          ds[t][r + 1] = fast_exp2(ds[t][r + 1]) * (dpv1 - dlt);
        }
      // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
      #pragma unroll
      for (int t = 0; t < 2; ++t)
        #pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const s16x8 dsf = pack8<T>(&ds[t][8 * s2]);
          const int klo = 32 * t + 16 * s2 + 4 * h2;
          #pragma unroll
          for (int dt = 0; dt < NDT; ++dt) dq[dt] = mma<T>(frag_tr<TSTR>(Kt, 32 * dt, klo, klo + 8, lane), dsf, dq[dt]);
        }
      if (more) lstore(cur ^ 1);
      __syncthreads();
    }

    if (qvalid) {
      T* row = dqp + (int64_t)myq * ba.dq.ss;
      const float s = a.scale;
      #pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
        #pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 32 * dt + 8 * g4 + 4 * h2;
          uint32_t w0 = (uint32_t)from_f<T>(dq[dt][4 * g4] * s).x | ((uint32_t)from_f<T>(dq[dt][4 * g4 + 1] * s).x << 16);
          uint32_t w1 = (uint32_t)from_f<T>(dq[dt][4 * g4 + 2] * s).x | ((uint32_t)from_f<T>(dq[dt][4 * g4 + 3] * s).x << 16);
          *reinterpret_cast<uint2*>(row + d0) = make_uint2(w0, w1);
        }
    }
  }
}

// dQ (fp32 accumulator [rows][h][D]) -> output dtype with the caller's strides
template <typename T, int D>
__global__ void __launch_bounds__(256) dq_convert_kernel(const AttnBwdArgs ba) {
  const AttnArgs& a = ba.f;
  constexpr int LPR = D / 8, RPB = 256 / LPR;
  const int hq = blockIdx.y, b = blockIdx.z;
  Seq sq;
  seq_of(a, b, a.q.sb, a.q.ss, a.k.sb, a.k.ss, sq);
  const int q = blockIdx.x * RPB + threadIdx.x / LPR, c8 = (threadIdx.x % LPR) * 8;
  if (q >= sq.lq) return;
  float v[8];
  Vec8<float>::load(v, ba.dq_acc + ((sq.qrow0 + q) * a.h + hq) * D + c8);
  T* dst = (T*)ba.dq.p + tensor_off(ba.dq, sq, true, a.cu_q != nullptr, b) + (int64_t)hq * ba.dq.sh +
           (int64_t)q * ba.dq.ss + c8;
  Vec8<T>::store(dst, v);
}

template <int D>
constexpr size_t fwd_lds() {
  return (size_t)2 * (64 * Geo<D>::KSTR + 64 * Geo<D>::TSTR) * 2;
}
template <int D>
constexpr size_t bwd_lds() {
  return (size_t)(128 * Geo<D>::TSTR + 2 * 32 * Geo<D>::KSTR + 32 * (128 + 8)) * 2 + 2 * 32 * 4;
}

// query fragments per wave: APEX_ATTN_FWD_QF=1|2 forces one; default 2 for the bias (+ dropout)
// mode at d <= 64 (its 1-fragment form spills 46 VGPRs; BERT-large +1.8 % same box) and 1 otherwise
// (GPT-2 medium's causal dropout mode: 2 fragments -2 %; profiles/r06/ab_attn_fwd_qf_r06x.txt)
inline int fwd_qf(const AttnArgs& a, int d) {
  const char* e = std::getenv("APEX_ATTN_FWD_QF");
  if (e != nullptr && (e[0] == '1' || e[0] == '2')) return e[0] - '0';
  return (a.bias != nullptr && d <= 64) ? 2 : 1;
}

// occupancy: APEX_ATTN_FWD_OCC=lo (A/B; default the per-shape rule in fwd_occupancy)
inline bool fwd_lo() {
  const char* e = std::getenv("APEX_ATTN_FWD_OCC");
  return e != nullptr && e[0] == 'l';
}

template <typename T, int D, int QF, bool LO>
void launch_fwd_qf(const AttnArgs& a, hipStream_t s) {
  const int nqb = (a.sq + 128 * QF - 1) / (128 * QF);
  const dim3 grid(a.causal ? (nqb + 1) / 2 : nqb, a.h, a.b);
  if (a.bias == nullptr && !(a.p_drop > 0.f))
    hipLaunchKernelGGL((fwd_kernel<T, D, 0, QF, LO>), grid, dim3(256), fwd_lds<D>(), s, a);
  else if (a.bias == nullptr) hipLaunchKernelGGL((fwd_kernel<T, D, 1, QF, LO>), grid, dim3(256), fwd_lds<D>(), s, a);
  else hipLaunchKernelGGL((fwd_kernel<T, D, 2, QF, LO>), grid, dim3(256), fwd_lds<D>(), s, a);
}

template <typename T, int D>
void launch_fwd(const AttnArgs& a, hipStream_t s) {
  if (fwd_qf(a, D) == 2) launch_fwd_qf<T, D, 2, false>(a, s);
  else if (fwd_lo()) launch_fwd_qf<T, D, 1, true>(a, s);
  else launch_fwd_qf<T, D, 1, false>(a, s);
}

template <int D, int QS>
constexpr size_t dkdv_lds() {
  return (size_t)2 * (2 * QS * (dkdv_swz<D>() ? D : Geo<D>::KSTR) + 6 * QS) * 2;
}

// dK/dV LDS slice depth in queries (APEX_ATTN_DKDV_QS=32|64 overrides, A/B).  Measured on MI355X
// (profiles/attn_dkdv_qs_r02.jsonl): at head dim 128 (one wave per SIMD) 64-query slices halve
// the per-slice commit + barrier stalls, bwd 1.94 -> 1.39 ms (b8 s2048 h16), 1.17-1.23x causal; at
// head dim <= 64 (two waves per SIMD hide them already) 32 stays 1-5 % faster
template <int D>
inline int dkdv_qs() {
  const char* e = std::getenv("APEX_ATTN_DKDV_QS");
  if (e != nullptr) return e[0] == '3' ? 32 : 64;
  return D == 128 ? 64 : 32;
}
template <int D>
constexpr size_t dq_lds() {
  return (size_t)2 * 64 * (2 * Geo<D>::KSTR + Geo<D>::TSTR) * 2;
}

template <typename T, int D, int MODE>
void launch_bwd_v(const AttnBwdArgs& ba, hipStream_t s) {
  constexpr bool PLAIN = MODE == 0;
  const AttnArgs& a = ba.f;
  constexpr int RPB = 256 / (D / 8);
  hipLaunchKernelGGL((bwd_delta_kernel<T, D>), dim3((a.sq + RPB - 1) / RPB, a.h, a.b), dim3(256), 0, s, ba);
  if (ba.dq_acc == nullptr) {  // split, atomic-free path
    const int nkb = (a.sk + 127) / 128, nqb = (a.sq + 127) / 128;
    const dim3 grid(a.causal ? (nkb + 1) / 2 : nkb, a.h_k, a.b);
    if (dkdv_qs<D>() == 64) hipLaunchKernelGGL((bwd_dkdv_kernel<T, D, MODE, 64>), grid, dim3(256), (dkdv_lds<D, 64>()), s, ba);
    else hipLaunchKernelGGL((bwd_dkdv_kernel<T, D, MODE, 32>), grid, dim3(256), (dkdv_lds<D, 32>()), s, ba);
    hipLaunchKernelGGL((bwd_dq_kernel<T, D, MODE>), dim3(nqb, a.h, a.b), dim3(256), dq_lds<D>(), s, ba);
    return;
  }
  (void)hipMemsetAsync(ba.dq_acc, 0, (size_t)a.rows_q * a.h * D * sizeof(float), s);
  hipLaunchKernelGGL((bwd_kernel<T, D, PLAIN>), dim3((a.sk + 127) / 128, a.h_k, a.b), dim3(256), bwd_lds<D>(), s, ba);
  hipLaunchKernelGGL((dq_convert_kernel<T, D>), dim3((a.sq + RPB - 1) / RPB, a.h, a.b), dim3(256), 0, s, ba);
}

template <typename T, int D>
void launch_bwd(const AttnBwdArgs& ba, hipStream_t s) {
  if (ba.f.bias == nullptr && !(ba.f.p_drop > 0.f)) launch_bwd_v<T, D, 0>(ba, s);
  else if (ba.f.bias == nullptr) launch_bwd_v<T, D, 1>(ba, s);
  else launch_bwd_v<T, D, 2>(ba, s);
}

}  // namespace attn

bool attn_supported(int d, int dtype) { return (d == 32 || d == 64 || d == 128) && (dtype == kF16 || dtype == kBF16); }

void attn_fwd(const AttnArgs& a, hipStream_t s) {
  if (!attn_supported(a.d, a.dtype)) throw std::runtime_error("attn_fwd: unsupported head dim / dtype");
  if (a.h_k <= 0 || a.h % a.h_k) throw std::runtime_error("attn_fwd: h must be a multiple of h_k");
  dispatch_16(a.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    switch (a.d) {
      case 32: attn::launch_fwd<T, 32>(a, s); break;
      case 64: attn::launch_fwd<T, 64>(a, s); break;
      default: attn::launch_fwd<T, 128>(a, s); break;
    }
  }, "attn_fwd");
  check_launch("attn_fwd");
}

void attn_bwd(const AttnBwdArgs& a, hipStream_t s) {
  if (!attn_supported(a.f.d, a.f.dtype)) throw std::runtime_error("attn_bwd: unsupported head dim / dtype");
  dispatch_16(a.f.dtype, [&](auto tag) {
    using T = typename decltype(tag)::type;
    switch (a.f.d) {
      case 32: attn::launch_bwd<T, 32>(a, s); break;
      case 64: attn::launch_bwd<T, 64>(a, s); break;
      default: attn::launch_bwd<T, 128>(a, s); break;
    }
  }, "attn_bwd");
  check_launch("attn_bwd");
}

}  // namespace apex_amd
