// Peer-memory (hipIpc over xGMI) exchange for tiny, latency-bound collectives inside one node —
// the per-layer batch-norm statistics of SyncBatchNorm / BatchNorm2d_NHWC(bn_group > 1)
// (reference: apex/contrib/csrc/groupbn/ipc.cu + nhwc_batch_norm_kernel.h:595-730, a CUDA-IPC
// butterfly compiled out on HIP; SURVEY §5.8: RCCL's all_gather costs a launch + protocol
// round trip per layer for ~16 KB).
//
// Every rank owns one exchange buffer in device memory, exported with hipIpcGetMemHandle and
// opened by the other members of its group.  Layout: [2 parities][group][slot], slot = 16-byte
// header (epoch flag) + nmax fp32 payload.  One call (one 256-thread workgroup):
//   1. push: write the local payload into slot `me` of EVERY member's buffer (remote stores go
//      straight over xGMI), system-scope release fence, then store the epoch into each header;
//   2. wait: spin (bounded, with s_sleep) until all `group` headers of this parity in the LOCAL
//      buffer carry the epoch (system-scope ACQUIRE loads of the flags, then a system acquire
//      fence for the whole workgroup);
//   3. read: copy the `group` payloads into the output [group][n].
// The exchange buffers are allocated UNCACHED (hipExtMallocWithFlags(hipDeviceMallocUncached),
// the allocation RCCL uses for its cross-GPU flags): coarse-grained device memory is only coherent
// at kernel boundaries, while these slots are written by remote GPUs over xGMI and polled by a
// running kernel.  If the driver refuses an uncached (or fine-grained) IPC-exportable buffer the
// allocation falls back to plain device memory and reports it (peer_alloc_kind); the Python side
// then validates the protocol with a short handshake before trusting it (PeerExchange).
// Parity = epoch & 1 double-buffers the slots: a rank can only reach epoch e+2 after every member
// published e+1, which each member does only after it finished reading epoch e.
//
// Failure handling: the wait is bounded in WALL time (kTimeoutTicks of the 100 MHz real-time
// counter, 30 s by default: far above any legitimate skew between ranks such as a first-step convolution
// search or a rank-0 checkpoint, so the kernel always terminates even if a member died).  A wait
// that runs out never hands back stale slots: the whole output is POISONED with NaN and *err is
// incremented.  NaN statistics propagate into the loss and the gradients, so the dynamic loss
// scaler skips that step instead of training on garbage, and PeerExchange polls *err without a
// device sync and raises.
#include "apex_amd/device.h"
#include "apex_amd/dispatch.h"

#include <cstring>
#include <stdexcept>
#include <string>

namespace apex_amd {
namespace peer {

constexpr int kHeaderFloats = 4;
constexpr int kMaxGroup = 8;
constexpr uint64_t kTicksPerSecond = 100000000ull;  // the 100 MHz real-time counter (wall_clock64)

struct Ptrs {
  float* buf[kMaxGroup];
};

__global__ void __launch_bounds__(256) allgather_kernel(const float* __restrict__ local, int n, int nmax, Ptrs bufs,
                                                        int me, int group, uint32_t epoch, float* __restrict__ out,
                                                        int* __restrict__ err, uint64_t timeout_ticks) {
  const int tid = threadIdx.x;
  const int slot = nmax + kHeaderFloats;
  const int parity = (int)(epoch & 1u);
  // 1. push
  for (int j = 0; j < group; ++j) {
    float* dst = bufs.buf[j] + (int64_t)(parity * group + me) * slot + kHeaderFloats;
    for (int i = tid; i < n; i += 256) dst[i] = local[i];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: remote payload stores performed
  __syncthreads();
  if (tid < group) {
    uint32_t* flag = reinterpret_cast<uint32_t*>(bufs.buf[tid] + (int64_t)(parity * group + me) * slot);
    __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 2. wait for every member's slot in the local buffer
  __shared__ int timed_out;
  if (tid == 0) timed_out = 0;
  __syncthreads();
  if (tid < group) {
    uint32_t* flag = reinterpret_cast<uint32_t*>(bufs.buf[me] + (int64_t)(parity * group + tid) * slot);
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      if (wall_clock64() - t0 > timeout_ticks) {
        timed_out = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: no stale L1 / L2 lines of the slots
  if (timed_out) {
    const float qnan = __builtin_nanf("");
    for (int i = tid; i < group * n; i += 256) out[i] = qnan;
    if (tid == 0) atomicAdd(err, 1);
    return;
  }
  // 3. read
  for (int j = 0; j < group; ++j) {
    const float* src = bufs.buf[me] + (int64_t)(parity * group + j) * slot + kHeaderFloats;
    for (int i = tid; i < n; i += 256) out[(int64_t)j * n + i] = src[i];
  }
}

}  // namespace peer

// kind: 2 = uncached, 1 = fine-grained, 0 = plain coarse-grained device memory.  A kind is only
// accepted when the buffer can also be exported for IPC (hipIpcGetMemHandle succeeds on it).
void* peer_alloc(size_t bytes, int* kind) {
  const unsigned flags[2] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
  void* p = nullptr;
  int k = -1;
  for (int i = 0; i < 2 && k < 0; ++i) {
    if (hipExtMallocWithFlags(&p, bytes, flags[i]) != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      continue;
    }
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, p) == hipSuccess) {
      k = 2 - i;
    } else {
      (void)hipGetLastError();
      (void)hipFree(p);
      p = nullptr;
    }
  }
  if (k < 0) {
    if (hipMalloc(&p, bytes) != hipSuccess) throw std::runtime_error("peer_alloc: hipMalloc failed");
    k = 0;
  }
  if (hipMemset(p, 0, bytes) != hipSuccess) throw std::runtime_error("peer_alloc: hipMemset failed");
  if (hipDeviceSynchronize() != hipSuccess) throw std::runtime_error("peer_alloc: sync failed");
  if (kind) *kind = k;
  return p;
}

void peer_free(void* p) { (void)hipFree(p); }

std::string peer_handle(void* p) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) throw std::runtime_error("peer_handle: hipIpcGetMemHandle failed");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void* peer_open(const std::string& handle) {
  if (handle.size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("peer_open: bad handle size");
  hipIpcMemHandle_t h;
  memcpy(&h, handle.data(), sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
    throw std::runtime_error("peer_open: hipIpcOpenMemHandle failed");
  return p;
}

void peer_close(void* p) { (void)hipIpcCloseMemHandle(p); }

int peer_max_group() { return peer::kMaxGroup; }

void peer_allgather(const float* local, int n, int nmax, float* const* bufs, int me, int group, uint32_t epoch,
                    float* out, int* err, double timeout_s, hipStream_t s) {
  if (!(timeout_s > 0.0) || timeout_s > 600.0) throw std::runtime_error("peer_allgather: timeout must be in (0, 600] s");
  const uint64_t ticks = (uint64_t)(timeout_s * (double)peer::kTicksPerSecond);
  if (group < 1 || group > peer::kMaxGroup || me < 0 || me >= group || n > nmax)
    throw std::runtime_error("peer_allgather: bad group / size");
  peer::Ptrs p{};
  for (int j = 0; j < group; ++j) p.buf[j] = bufs[j];
  hipLaunchKernelGGL(peer::allgather_kernel, dim3(1), dim3(256), 0, s, local, n, nmax, p, me, group, epoch, out, err,
                     ticks);
  check_launch("peer_allgather");
}

}  // namespace apex_amd
