// Multi-tensor-apply (MTA) engine for gfx950.
//
// What it replaces: the reference packs <=110 tensor addresses and <=320 (tensor, chunk) pairs
// into the kernel-argument struct and relaunches every 320 chunks
// (reference csrc/multi_tensor_apply.cuh:16-147).  Here the whole work list lives in a
// device-resident table that the host builds once per distinct tensor list and caches
// (bindings/mta_host.cpp), so an optimizer step over ANY number of tensors is ONE launch of a
// persistent, grid-strided kernel sized to the 256 CUs, and it is capturable in a hipGraph
// (no per-call H2D copy once the table is cached).
#pragma once
#include "apex_amd/device.h"

namespace apex_amd {

constexpr int kMtaBlock = 256;  // 4 waves per block; up to 8 blocks/CU resident
constexpr int kVec = 8;         // elements per lane per step

struct MtaMeta {
  const int64_t* sizes;   // [ntensors] numel
  const uint64_t* ptrs;   // [depth][ntensors] base addresses
  const int2* chunks;     // [nchunks] {tensor index, chunk index within tensor}
  const int* first_chunk; // [ntensors + 1] prefix of chunk counts (chunks of a tensor are contiguous)
  uint64_t* partials;     // [2 * nchunks] tagged per-chunk partials: (launch tag << 32) | float bits
  float* stage;           // [2 * nchunks] the finalizing block's validated per-chunk sums of the partials
  unsigned* ticket;       // arrival counter for single-pass grid reductions (reset by last block)
  unsigned* epoch;        // tag of the previous launch over this table (bumped by the last block)
  int ntensors;
  int nchunks;
  int chunk_size;
  int depth;
  int aligned;            // every base pointer 32-byte aligned -> vector path legal
  int split;              // elementwise (no-reduction) launches: work items per chunk (mta_split)
};

// Elementwise launches split each chunk into `split` work items of chunk_size / split elements.
// The API's chunk (the reference's 2048 * 32 = 64k elements) gives a 100M-parameter step only 6
// blocks per CU, too few loads in flight for HBM3E; 16k-element items raise that to the 8-block cap
// with a grid-strided tail: +4-5 % on Adam / SGD (tools/mta_bench.py, profiles/r05/mta_split_r05.jsonl).
// Reductions stay one item per chunk: split items cost each block a drain + block reduction per
// item, which measured 85 -> 117 us on a 100M-element L2 norm.
inline int mta_split(int chunk_size, int item) {
  return (item > 0 && chunk_size > item && chunk_size % item == 0 && item % kVec == 0) ? chunk_size / item : 1;
}

template <typename T>
__device__ __forceinline__ T* mta_ptr(const MtaMeta& m, int d, int t, int64_t start) {
  // the table holds plain addresses; going through a global (addrspace 1) pointer lets the
  // compiler's address-space inference emit global_load/store instead of flat_* (flat ops also
  // count against lgkmcnt, which serialises them with LDS traffic)
  using GT = __attribute__((address_space(1))) T;
  GT* g = (GT*)(m.ptrs[(size_t)d * m.ntensors + t]);
  return (T*)(g + start);
}

// ---------------------------------------------------------------------------------------------
// Generic elementwise driver. `Op` provides:
//   static constexpr unsigned kRead, kWrite;   // bitmask over list depth
//   static constexpr bool kSkipOnNoop;         // early-exit when *noop != 0 at kernel start
//   struct TS; __device__ TS tensor_state(int tensor) const;   // per-tensor scalars
//   template<int N> __device__ void operator()(float (&r)[D][N], const TS&, bool& bad) const;
// Ts... are the storage types of each list (float / f16_t / bf16_t).
// ---------------------------------------------------------------------------------------------
template <int I, typename... Ts> struct TypeAt;
template <typename T0, typename... Ts> struct TypeAt<0, T0, Ts...> { using type = T0; };
template <int I, typename T0, typename... Ts> struct TypeAt<I, T0, Ts...> {
  using type = typename TypeAt<I - 1, Ts...>::type;
};

// Streaming IO for the multi-tensor ops.  APEX_MTA_NT=1 (variant build) issues the loads /
// stores as nontemporal (the data is touched once per step); the default is plain vector IO.
#ifndef APEX_MTA_NT
#define APEX_MTA_NT 0
#endif
#ifndef APEX_MTA_ILP
#define APEX_MTA_ILP 1
#endif
#ifndef APEX_MTA_RED_UNROLL
#define APEX_MTA_RED_UNROLL 4
#endif
typedef unsigned mta_u4 __attribute__((ext_vector_type(4)));
typedef unsigned mta_u2 __attribute__((ext_vector_type(2)));

template <typename T>
struct MtaIO {
  static constexpr int kBytes = (int)sizeof(T) * kVec;
  static __device__ __forceinline__ void load(float (&r)[kVec], const T* p) {
    if constexpr (!APEX_MTA_NT) {
      Vec8<T>::load(r, p);
    } else if constexpr (kBytes >= 16) {
      mta_u4 buf[kBytes / 16];
#pragma unroll
      for (int i = 0; i < kBytes / 16; ++i) buf[i] = __builtin_nontemporal_load(reinterpret_cast<const mta_u4*>(p) + i);
      Vec8<T>::load(r, reinterpret_cast<const T*>(buf));
    } else {
      mta_u2 buf = __builtin_nontemporal_load(reinterpret_cast<const mta_u2*>(p));
      Vec8<T>::load(r, reinterpret_cast<const T*>(&buf));
    }
  }
  static __device__ __forceinline__ void store(T* p, const float (&r)[kVec]) {
    if constexpr (!APEX_MTA_NT) {
      Vec8<T>::store(p, r);
    } else if constexpr (kBytes >= 16) {
      mta_u4 buf[kBytes / 16];
      Vec8<T>::store(reinterpret_cast<T*>(buf), r);
#pragma unroll
      for (int i = 0; i < kBytes / 16; ++i) __builtin_nontemporal_store(buf[i], reinterpret_cast<mta_u4*>(p) + i);
    } else {
      mta_u2 buf;
      Vec8<T>::store(reinterpret_cast<T*>(&buf), r);
      __builtin_nontemporal_store(buf, reinterpret_cast<mta_u2*>(p));
    }
  }
};

template <typename Op, int D, int I, typename... Ts>
struct ListIO {
  using T = typename TypeAt<I, Ts...>::type;
  static __device__ __forceinline__ void load_vec(float (&r)[D][kVec], void* const (&base)[D], int i) {
    if constexpr ((Op::kRead >> I) & 1u) MtaIO<T>::load(r[I], reinterpret_cast<const T*>(base[I]) + i);
    else {
#pragma unroll
      for (int k = 0; k < kVec; ++k) r[I][k] = 0.f;
    }
    if constexpr (I + 1 < D) ListIO<Op, D, I + 1, Ts...>::load_vec(r, base, i);
  }
  static __device__ __forceinline__ void store_vec(const float (&r)[D][kVec], void* const (&base)[D], int i) {
    if constexpr ((Op::kWrite >> I) & 1u) MtaIO<T>::store(reinterpret_cast<T*>(base[I]) + i, r[I]);
    if constexpr (I + 1 < D) ListIO<Op, D, I + 1, Ts...>::store_vec(r, base, i);
  }
  static __device__ __forceinline__ void load_one(float (&r)[D][1], void* const (&base)[D], int i) {
    if constexpr ((Op::kRead >> I) & 1u) r[I][0] = to_f(reinterpret_cast<const T*>(base[I])[i]);
    else r[I][0] = 0.f;
    if constexpr (I + 1 < D) ListIO<Op, D, I + 1, Ts...>::load_one(r, base, i);
  }
  static __device__ __forceinline__ void store_one(const float (&r)[D][1], void* const (&base)[D], int i) {
    if constexpr ((Op::kWrite >> I) & 1u) reinterpret_cast<T*>(base[I])[i] = from_f<T>(r[I][0]);
    if constexpr (I + 1 < D) ListIO<Op, D, I + 1, Ts...>::store_one(r, base, i);
  }
  static __device__ __forceinline__ void set_base(void* (&base)[D], const MtaMeta& m, int t, int64_t start) {
    base[I] = mta_ptr<T>(m, I, t, start);
    if constexpr (I + 1 < D) ListIO<Op, D, I + 1, Ts...>::set_base(base, m, t, start);
  }
};

// ---------------------------------------------------------------------------------------------
// Single-pass grid reduction support: every block writes its partial(s) as tagged agent-scope
// atomics, takes a ticket, and the last arriving block finalizes (mta_tensor_reduce below).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool mta_last_block(unsigned* ticket, int* smem_flag);
__device__ __forceinline__ void mta_put_partial(uint64_t* p, float v, unsigned tag);
__device__ __forceinline__ void mta_collect_partials(const MtaMeta& m, int num_acc, unsigned tag);

// The last-arriving block of a reduction launch: either the real finalize over the collected
// partials, or (the skip flag is set: this step is skipped anyway) the op's skipped result.
// Both reset the ticket and advance the epoch, so the next launch's partials carry a fresh tag.
template <typename Op>
__device__ __forceinline__ void mta_finish(const MtaMeta& meta, const Op& op, unsigned tag, bool skipped) {
  if (skipped) {
    op.finalize_skipped(meta);
  } else {
    mta_collect_partials(meta, Op::kNumAcc, tag);
    op.finalize(meta, tag);
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(meta.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(meta.epoch, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// bytes each lane loads per kVec-element step (the lists the op reads)
template <unsigned Mask, typename... Ts>
constexpr int mta_read_bytes() {
  int b = 0, i = 0;
  ((b += ((Mask >> i++) & 1u) ? (int)sizeof(Ts) * kVec : 0), ...);
  return b;
}

// Ops with kNumAcc > 0 accumulate per-element sums (or maxima when Op::kAccMax) which are
// reduced per chunk into meta.partials; the last block then calls op.finalize(meta, smem).
template <typename Op, typename... Ts>
__global__ void __launch_bounds__(kMtaBlock) mta_elementwise_kernel(MtaMeta meta, int* noop, Op op) {
  constexpr int D = sizeof...(Ts);
  constexpr int NA = Op::kNumAcc;
  __shared__ float smem[kMtaBlock / 64 * 2 + 2];
  const int split = NA == 0 ? meta.split : 1;
  const int item = meta.chunk_size / split;
  const int nwork = meta.nchunks * split;
  if constexpr (Op::kSkipOnNoop) {
    // uniform early exit; a reduction op still has to take part in the ticket protocol.  The
    // flag can also be raised DURING this launch (kCheckPartial ops set it on a non-finite
    // chunk), so a skipping block still publishes tagged (zero) partials for its chunks: a
    // finalizer that did not skip then never waits on a slot nobody writes.
    if (__hip_atomic_load(noop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
      if constexpr (NA == 0) return;
      else {
        const unsigned tag = __hip_atomic_load(meta.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        for (int w = blockIdx.x; w < nwork; w += gridDim.x)
          if (threadIdx.x < NA) mta_put_partial(meta.partials + (size_t)threadIdx.x * nwork + w, 0.f, tag);
        if (mta_last_block(meta.ticket, reinterpret_cast<int*>(&smem[kMtaBlock / 64 * 2])))
          mta_finish(meta, op, tag, true);
        return;
      }
    }
  }
  bool bad = false;
  unsigned tag = 0;
  if constexpr (NA > 0) tag = __hip_atomic_load(meta.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  for (int w = blockIdx.x; w < nwork; w += gridDim.x) {
    const int c = split == 1 ? w : w / split;
    const int2 tc = meta.chunks[c];
    const int64_t start = (int64_t)tc.y * meta.chunk_size + (int64_t)(w - c * split) * item;
    const int64_t rem = meta.sizes[tc.x] - start;
    if (rem <= 0) continue;  // a split item past the end of its tensor's last chunk
    const int len = rem < item ? (int)rem : item;
    void* base[D];
    ListIO<Op, D, 0, Ts...>::set_base(base, meta, tc.x, start);
    const auto ts = op.tensor_state(tc.x);
    float acc[NA > 0 ? NA : 1];
#pragma unroll
    for (int a = 0; a < (NA > 0 ? NA : 1); ++a) acc[a] = 0.f;
    const int nvec = meta.aligned ? (len / kVec) : 0;
    int v = threadIdx.x;
    // light streams (<= 32 B loaded per lane per step, e.g. a bf16 -> fp32 scale) keep two steps
    // loads in flight per lane; heavier ones (Adam: 128 B) have enough with one
    if constexpr (Op::kWrite != 0 && (APEX_MTA_ILP > 1 || mta_read_bytes<Op::kRead, Ts...>() <= 32)) {
      // two vectors per thread per trip: both loads are in flight before either is stored
      for (; v + kMtaBlock < nvec; v += 2 * kMtaBlock) {
        float r0[D][kVec], r1[D][kVec];
        ListIO<Op, D, 0, Ts...>::load_vec(r0, base, v * kVec);
        ListIO<Op, D, 0, Ts...>::load_vec(r1, base, (v + kMtaBlock) * kVec);
        op.template apply<kVec>(r0, ts, bad, acc);
        op.template apply<kVec>(r1, ts, bad, acc);
        ListIO<Op, D, 0, Ts...>::store_vec(r0, base, v * kVec);
        ListIO<Op, D, 0, Ts...>::store_vec(r1, base, (v + kMtaBlock) * kVec);
      }
    }
    if constexpr (Op::kWrite == 0 && APEX_MTA_RED_UNROLL > 1) {
      // read-only ops (norms, finite checks): several independent loads in flight per lane
      constexpr int U = APEX_MTA_RED_UNROLL;
      for (; v + (U - 1) * kMtaBlock < nvec; v += U * kMtaBlock) {
        float r[U][D][kVec];
#pragma unroll
        for (int u = 0; u < U; ++u) ListIO<Op, D, 0, Ts...>::load_vec(r[u], base, (v + u * kMtaBlock) * kVec);
#pragma unroll
        for (int u = 0; u < U; ++u) op.template apply<kVec>(r[u], ts, bad, acc);
      }
    }
    for (; v < nvec; v += kMtaBlock) {
      float r[D][kVec];
      ListIO<Op, D, 0, Ts...>::load_vec(r, base, v * kVec);
      op.template apply<kVec>(r, ts, bad, acc);
      ListIO<Op, D, 0, Ts...>::store_vec(r, base, v * kVec);
    }
    for (int i = nvec * kVec + threadIdx.x; i < len; i += kMtaBlock) {
      float r[D][1];
      ListIO<Op, D, 0, Ts...>::load_one(r, base, i);
      op.template apply<1>(r, ts, bad, acc);
      ListIO<Op, D, 0, Ts...>::store_one(r, base, i);
    }
    if constexpr (NA > 0) {
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        float s = op.acc_is_max() ? block_max(acc[a], smem + a * (kMtaBlock / 64))
                                  : block_sum(acc[a], smem + a * (kMtaBlock / 64));
        if (threadIdx.x == 0) {
          mta_put_partial(meta.partials + (size_t)a * nwork + w, s, tag);
          if (Op::kCheckPartial && !is_finite(s)) bad = true;
        }
      }
    }
  }
  // benign race (every writer stores the same value); an agent-scope (write-through) store so
  // the finalizing block's agent-scope re-read below sees it on any XCD
  if (bad) __hip_atomic_store(noop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if constexpr (NA > 0) {
    if (mta_last_block(meta.ticket, reinterpret_cast<int*>(&smem[kMtaBlock / 64 * 2]))) {
      bool skipped = false;
      if constexpr (Op::kSkipOnNoop)
        skipped = __hip_atomic_load(noop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
      mta_finish(meta, op, tag, skipped);
    }
  }
}

inline int mta_grid(int nchunks, int max_blocks) { return nchunks < max_blocks ? (nchunks > 0 ? nchunks : 1) : max_blocks; }
// one block per work item, up to the resident-block cap (grid-strided beyond it); reductions
// (kNumAcc > 0) pass split = false
inline int mta_grid_work(const MtaMeta& m, int max_blocks, bool split = true) {
  const int64_t n = (int64_t)m.nchunks * (split ? m.split : 1);
  return mta_grid(n < max_blocks ? (int)n : max_blocks, max_blocks);
}

// Base class for ops without reductions / per-tensor state.
struct MtaOpBase {
  static constexpr int kNumAcc = 0;
  static constexpr bool kAccMax = false;
  static constexpr bool kCheckPartial = false;
  struct TS {};
  __device__ __forceinline__ TS tensor_state(int) const { return {}; }
  __device__ __forceinline__ bool acc_is_max() const { return false; }
  __device__ __forceinline__ void finalize(const MtaMeta&, unsigned) const {}
  __device__ __forceinline__ void finalize_skipped(const MtaMeta&) const {}
};

// Sum (or max) partial slot `a` over the chunks of tensor t, in chunk order (deterministic).
// Cross-XCD hand-off of the per-chunk partials without an L2 writeback: every partial is ONE
// 64-bit agent-scope atomic word carrying its value and the launch tag, so it is self-validating
// (no ordering between different locations is needed).  The finalizing block reads each word
// with an agent-scope atomic load and re-reads until the tag matches this launch — normally
// immediately, since every block's stores were acknowledged before it took its ticket.  An
// agent-scope release fence instead writes back the whole XCD L2 per block (measured ~30 us on
// a 1.5k-block norm).
__device__ __forceinline__ void mta_put_partial(uint64_t* p, float v, unsigned tag) {
  const uint64_t w = ((uint64_t)tag << 32) | (uint64_t)__float_as_uint(v);
  __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float mta_get_partial(const uint64_t* p, unsigned tag) {
  uint64_t w = __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int spin = 0; (unsigned)(w >> 32) != tag && spin < (1 << 22); ++spin) {
    __builtin_amdgcn_s_sleep(1);
    w = __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return __uint_as_float((unsigned)(w & 0xffffffffu));
}

// Finalizing block, all threads: validate every tagged partial and stage the values for the
// per-tensor sums (read back by this same block after the barrier).  Each thread issues its
// partials in batches of 8 independent atomic loads (one round trip per batch instead of one per
// partial), then checks the tags and re-reads only a word that is not yet this launch's.
__device__ __forceinline__ void mta_collect_partials(const MtaMeta& m, int num_acc, unsigned tag) {
  constexpr int B = 8;
  const int n = num_acc * m.nchunks;
  for (int i0 = threadIdx.x; i0 < n; i0 += B * blockDim.x) {
    uint64_t w[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int i = i0 + b * blockDim.x;
      w[b] = i < n ? __hip_atomic_load(m.partials + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int i = i0 + b * blockDim.x;
      if (i < n)
        m.stage[i] = (unsigned)(w[b] >> 32) == tag ? __uint_as_float((unsigned)(w[b] & 0xffffffffu))
                                                   : mta_get_partial(m.partials + i, tag);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ float mta_tensor_reduce(const MtaMeta& m, int a, int t, bool is_max, unsigned) {
  const float* p = m.stage + (size_t)a * m.nchunks;
  float s = 0.f;
  for (int c = m.first_chunk[t]; c < m.first_chunk[t + 1]; ++c) s = is_max ? fmaxf(s, p[c]) : s + p[c];
  return s;
}

__device__ __forceinline__ bool mta_last_block(unsigned* ticket, int* smem_flag) {
  // every storing wave drains its stores (the tagged partials are acknowledged) before the ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    // the partials are self-validating tagged atomics (mta_get_partial), so no fence here
    unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = (prev == gridDim.x - 1);
    *smem_flag = last;
  }
  __syncthreads();
  return *smem_flag != 0;
}

}  // namespace apex_amd
