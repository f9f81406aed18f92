// Host side of the multi-tensor-apply engine: builds the device work table for a tensor
// list-of-lists and caches it, keyed by (device, STREAM, depth, chunk_size, addresses, sizes).
//
// The table also holds the scratch of the single-pass reductions (per-chunk partials + the
// last-block ticket).  Keying by the launching stream gives every stream its own scratch, so two
// reductions over the same tensor list that are in flight on different streams (e.g. a norm on a
// side stream beside one on the compute stream) never share a ticket; launches on one stream are
// ordered, so they can share one.
//
// An optimizer steps the same parameter/state tensors every iteration, so after the first step
// every multi-tensor launch finds its table resident on the device: no per-step H2D traffic and
// no kernel-argument packing (the reference repacks <=110 addresses per launch on the host,
// csrc/multi_tensor_apply.cuh:84-146).  Gradients set to None between steps come back at new
// addresses: a list whose STRUCTURE (device, stream, depth, chunk size, sizes) matches a cached
// table gets that table's changed address rows patched in place (one small upload, ordered on
// the stream after the launches that read the old rows) instead of a full rebuild — unless the
// table may be replayed by a captured graph.
#include "common.h"
#include <algorithm>
#include <list>
#include <mutex>
#include <unordered_map>

namespace apex_amd {
namespace {

struct Entry {
  std::vector<uint64_t> key;
  at::Tensor dev;   // the table
  MtaMeta meta;
  bool pinned_forever = false;
  std::list<uint64_t>::iterator lru_it;
  uint64_t shash = 0;    // hash of the structural part of the key
  size_t off_ptrs = 0;   // byte offset of the [depth][nt] address rows in the table
};

std::mutex g_mu;
std::unordered_map<uint64_t, Entry> g_cache;
std::list<uint64_t> g_lru;
constexpr size_t kMaxEntries = 1024;

inline uint64_t mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  return h * 0xff51afd7ed558ccdull;
}

inline size_t align8(size_t x) { return (x + 7) & ~size_t(7); }

}  // namespace

MtaMeta mta_meta(const std::vector<std::vector<at::Tensor>>& lists, int chunk_size) {
  TORCH_CHECK(!lists.empty(), "multi_tensor_apply: empty tensor_lists");
  TORCH_CHECK(chunk_size > 0 && chunk_size % kVec == 0, "chunk_size must be a positive multiple of ", kVec);
  const int depth = (int)lists.size();
  const int nt = (int)lists[0].size();
  TORCH_CHECK(nt > 0, "multi_tensor_apply: empty tensor list");
  for (int d = 0; d < depth; ++d)
    TORCH_CHECK((int)lists[d].size() == nt, "multi_tensor_apply: list ", d, " has ", lists[d].size(),
                " tensors, expected ", nt);
  const auto dev = lists[0][0].device();
  TORCH_CHECK(dev.is_cuda(), "multi_tensor_apply: tensors must be on a GPU");

  std::vector<uint64_t> key;
  key.reserve(4 + (size_t)nt * (depth + 1));
  key.push_back((uint64_t)dev.index());
  key.push_back((uint64_t)(uintptr_t)cur_stream());
  key.push_back((uint64_t)depth);
  key.push_back((uint64_t)chunk_size);
  key.push_back((uint64_t)nt);
  bool aligned = true;
  for (int t = 0; t < nt; ++t) {
    const auto& t0 = lists[0][t];
    const int64_t n = t0.numel();
    key.push_back((uint64_t)n);
    for (int d = 0; d < depth; ++d) {
      const auto& x = lists[d][t];
      TORCH_CHECK(x.device() == dev, "multi_tensor_apply: all tensors must be on the same device");
      TORCH_CHECK(x.numel() == n, "multi_tensor_apply: size mismatch at list ", d, " tensor ", t);
      TORCH_CHECK(x.is_non_overlapping_and_dense(), "multi_tensor_apply: tensor ", t, " of list ", d,
                  " is not dense");
      TORCH_CHECK(x.scalar_type() == lists[d][0].scalar_type(), "multi_tensor_apply: list ", d,
                  " mixes dtypes (", lists[d][0].scalar_type(), " vs ", x.scalar_type(), " at tensor ", t,
                  "); split lists by dtype");
      // elementwise over raw storage: every list must walk the same physical element order
      if (d > 0 && !(x.is_contiguous() && t0.is_contiguous()))
        TORCH_CHECK(x.strides() == t0.strides(), "multi_tensor_apply: memory layout mismatch at tensor ", t,
                    " of list ", d);
      const uint64_t p = (uint64_t)x.data_ptr();
      aligned = aligned && (p % 32 == 0);
      key.push_back(p);
    }
  }
  uint64_t h = 0x1234567ull;
  for (auto v : key) h = mix(h, v);
  // structural hash: every key word but the addresses
  uint64_t sh = 0x7654321ull;
  for (int i = 0; i < 5; ++i) sh = mix(sh, key[i]);
  for (int t = 0; t < nt; ++t) sh = mix(sh, key[5 + (size_t)t * (depth + 1)]);

  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_cache.find(h);
  hipStreamCaptureStatus cap0 = hipStreamCaptureStatusNone;
  hipStreamIsCapturing(cur_stream(), &cap0);
  if (it != g_cache.end() && it->second.key == key) {
    g_lru.splice(g_lru.begin(), g_lru, it->second.lru_it);
    // a table first built eagerly (e.g. by warm-up steps on the capture stream) and now recorded
    // into a graph: the graph replays it, so it must never be address-patched or evicted again
    if (cap0 != hipStreamCaptureStatusNone) it->second.pinned_forever = true;
    return it->second.meta;
  }
  if (cap0 == hipStreamCaptureStatusNone && (it == g_cache.end() || !it->second.pinned_forever)) {
    // the structurally identical table with the most matching addresses (recently used first)
    auto best = g_cache.end();
    size_t best_match = 0;
    for (uint64_t lh : g_lru) {
      auto c = g_cache.find(lh);
      if (c == g_cache.end() || c->second.pinned_forever || c->second.shash != sh || c->second.key.size() != key.size())
        continue;
      bool same = true;
      size_t match = 0;
      for (size_t i = 0; i < key.size() && same; ++i) {
        const bool is_ptr = i >= 5 && (i - 5) % (size_t)(depth + 1) != 0;
        if (is_ptr) match += c->second.key[i] == key[i];
        else same = c->second.key[i] == key[i];
      }
      if (same && (best == g_cache.end() || match > best_match)) {
        best = c;
        best_match = match;
      }
    }
    if (best != g_cache.end()) {
      Entry e = std::move(best->second);
      g_lru.erase(e.lru_it);
      g_cache.erase(best);
      auto clash = g_cache.find(h);  // the new hash held by a different (unpinned) key: drop it
      if (clash != g_cache.end()) {
        g_lru.erase(clash->second.lru_it);
        g_cache.erase(clash);
      }
      // patch the span of address rows that changed ([depth][nt] layout in the table)
      std::vector<uint64_t> rows((size_t)depth * nt);
      for (int t = 0; t < nt; ++t)
        for (int d = 0; d < depth; ++d) rows[(size_t)d * nt + t] = key[5 + (size_t)t * (depth + 1) + 1 + d];
      size_t lo = rows.size(), hi = 0;
      for (int t = 0; t < nt; ++t)
        for (int d = 0; d < depth; ++d) {
          const size_t r = (size_t)d * nt + t;
          if (e.key[5 + (size_t)t * (depth + 1) + 1 + d] != rows[r]) {
            lo = std::min(lo, r);
            hi = std::max(hi, r + 1);
          }
        }
      const c10::hip::HIPGuard guard(dev.index());
      if (lo < hi)
        mta_upload_bytes(e.dev.data_ptr<uint8_t>() + e.off_ptrs + lo * sizeof(uint64_t), rows.data() + lo,
                         (hi - lo) * sizeof(uint64_t), cur_stream());
      e.meta.aligned = aligned ? 1 : 0;
      e.key = std::move(key);
      g_lru.push_front(h);
      e.lru_it = g_lru.begin();
      MtaMeta m = e.meta;
      g_cache[h] = std::move(e);
      return m;
    }
  }
  if (it != g_cache.end()) {  // hash collision with a different key: drop the old one
    if (!it->second.pinned_forever) {
      g_lru.erase(it->second.lru_it);
      g_cache.erase(it);
    } else {
      TORCH_CHECK(false, "multi_tensor_apply: table hash collision with a graph-captured table");
    }
  }

  // ---- build the table on the host ----
  std::vector<int> first(nt + 1, 0);
  int nchunks = 0;
  for (int t = 0; t < nt; ++t) {
    first[t] = nchunks;
    const int64_t n = lists[0][t].numel();
    const int64_t c = (n + chunk_size - 1) / chunk_size;
    TORCH_CHECK(nchunks + c < (1ll << 31), "multi_tensor_apply: too many chunks");
    nchunks += (int)c;
  }
  first[nt] = nchunks;
  static const int item = [] {
    const char* e = std::getenv("APEX_AMD_MTA_ITEM");  // A/B knob: elements per work item
    return e ? std::atoi(e) : 16384;
  }();
  const int split = mta_split(chunk_size, item);
  TORCH_CHECK((int64_t)nchunks * split < (1ll << 31), "multi_tensor_apply: too many work items");

  const size_t off_sizes = 0;
  const size_t off_ptrs = align8(off_sizes + sizeof(int64_t) * nt);
  const size_t off_chunks = align8(off_ptrs + sizeof(uint64_t) * (size_t)depth * nt);
  const size_t off_first = align8(off_chunks + sizeof(int2) * (size_t)std::max(nchunks, 1));
  const size_t off_part = align8(off_first + sizeof(int) * (size_t)(nt + 1));
  const size_t off_stage = align8(off_part + sizeof(uint64_t) * 2 * (size_t)std::max(nchunks, 1));
  const size_t off_ticket = align8(off_stage + sizeof(float) * 2 * (size_t)std::max(nchunks, 1));
  const size_t bytes = off_ticket + 64;

  std::vector<uint8_t> host(bytes, 0);
  uint8_t* hb = host.data();
  auto* sizes = reinterpret_cast<int64_t*>(hb + off_sizes);
  auto* ptrs = reinterpret_cast<uint64_t*>(hb + off_ptrs);
  auto* chunks = reinterpret_cast<int2*>(hb + off_chunks);
  auto* fc = reinterpret_cast<int*>(hb + off_first);
  for (int t = 0; t < nt; ++t) {
    sizes[t] = lists[0][t].numel();
    for (int d = 0; d < depth; ++d) ptrs[(size_t)d * nt + t] = (uint64_t)lists[d][t].data_ptr();
    for (int c = first[t]; c < first[t + 1]; ++c) chunks[c] = make_int2(t, c - first[t]);
  }
  for (int t = 0; t <= nt; ++t) fc[t] = first[t];

  const c10::hip::HIPGuard guard(dev.index());
  auto devbuf = at::empty({(int64_t)bytes}, at::TensorOptions().dtype(at::kByte).device(dev));
  // through kernel arguments: no pinned staging buffer whose allocator events would break
  // hipGraph capture, and nothing to keep alive for replays
  mta_upload_bytes(devbuf.data_ptr(), hb, bytes, cur_stream());

  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  hipStreamIsCapturing(cur_stream(), &cap);

  uint8_t* db = devbuf.data_ptr<uint8_t>();
  MtaMeta m;
  m.sizes = reinterpret_cast<const int64_t*>(db + off_sizes);
  m.ptrs = reinterpret_cast<const uint64_t*>(db + off_ptrs);
  m.chunks = reinterpret_cast<const int2*>(db + off_chunks);
  m.first_chunk = reinterpret_cast<const int*>(db + off_first);
  m.partials = reinterpret_cast<uint64_t*>(db + off_part);
  m.stage = reinterpret_cast<float*>(db + off_stage);
  m.ticket = reinterpret_cast<unsigned*>(db + off_ticket);
  m.epoch = reinterpret_cast<unsigned*>(db + off_ticket + 4);
  m.ntensors = nt;
  m.nchunks = nchunks;
  m.chunk_size = chunk_size;
  m.depth = depth;
  m.aligned = aligned ? 1 : 0;
  m.split = split;

  // LRU eviction (never evict tables a captured graph may replay)
  while (g_cache.size() >= kMaxEntries && !g_lru.empty()) {
    auto victim = std::prev(g_lru.end());
    bool evicted = false;
    for (auto v = victim;; --v) {
      auto vit = g_cache.find(*v);
      if (vit != g_cache.end() && !vit->second.pinned_forever) {
        g_cache.erase(vit);
        g_lru.erase(v);
        evicted = true;
        break;
      }
      if (v == g_lru.begin()) break;
    }
    if (!evicted) break;
  }

  g_lru.push_front(h);
  Entry e;
  e.key = std::move(key);
  e.dev = devbuf;
  e.meta = m;
  e.shash = sh;
  e.off_ptrs = off_ptrs;
  e.lru_it = g_lru.begin();
  if (cap != hipStreamCaptureStatusNone) e.pinned_forever = true;
  g_cache[h] = std::move(e);
  return m;
}

void mta_cache_clear() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto it = g_cache.begin(); it != g_cache.end();) {
    if (!it->second.pinned_forever) {
      g_lru.erase(it->second.lru_it);
      it = g_cache.erase(it);
    } else {
      ++it;
    }
  }
}

int64_t mta_cache_size() {
  std::lock_guard<std::mutex> lk(g_mu);
  return (int64_t)g_cache.size();
}

}  // namespace apex_amd
