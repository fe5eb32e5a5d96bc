// Stream-ordered IPC exchange (gmt_ipc_exchange, gmt/kernels.h), gfx950.
//
// The halo transport "ipc" (csrc/comm/transport_mpi.cpp) runs every
// exchange as ONE launch on the caller's stream — no host synchronisation,
// no MPI token rounds, so the exchange can be captured into a hipGraph.
// Send channels and receive channels are workgroups of the same grid (at
// most 128 per role, looping over 16 KB chunks, so spinning workgroups never
// occupy the GPU that the peer processes' kernels need):
//   send:    wait until the receiver has finished reading the staging slot
//            about to be overwritten (flag >= e - 2), copy the caller's send
//            buffer into slot e & 1; the last send workgroup publishes "data
//            ready" (flag = e) in every receiver's memory;
//   receive: wait for "data ready" (flag >= e), pull the sender's slot into
//            the caller's receive buffer; the last receive workgroup tells
//            every sender "slot consumed" (flag = e);
//   the last workgroup of all advances the local epoch to e.
// Pulling (not pushing) keeps the coherence one-sided: the sender's
// system-scope release writes its L2 back before the flag store, and the
// receiver's system-scope acquire invalidates its caches before it reads
// remote memory; nothing writes into another device's cached memory.
// gmt_signal_wait (below) is the same kind of stream-ordered wait for a
// completion signal raised inside another stream's kernel (gmt_tb_opts).
//
// The epoch lives in device memory (read at the start, advanced by the last
// workgroup of the recv step), so replayed graphs stay in step.
//
// Flags are GMT_SPACE_FLAGS memory (uncached); loads and stores of them are
// vector atomics at system scope.  Every wait gives up after ~2^22 sleeps
// (about a second) and sets *err, so a lost peer cannot hang the GPU.
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {
namespace ipc {

constexpr int64_t kBlockBytes = 16 * 1024;  // bytes per chunk: 4 x 16 B per lane
constexpr int64_t kMaxRoleBlocks = 128;     // workgroups per role: spinning groups never fill the GPU
constexpr unsigned kSpinLimit = 1u << 22;

struct Args {
  gmt_ipc_chan c[2 * GMT_IPC_MAX_CHAN];     // sends, then receives
  int64_t cstart[2 * GMT_IPC_MAX_CHAN + 1];  // prefix sum of chunks per channel (sends, then receives)
  int ns, nr;
  int64_t sb, rb;  // workgroups of the send role, then of the receive role
  uint64_t* epoch;
  unsigned* counter;  // [0] send role, [1] receive role, [2] all
  unsigned* err;
};

__device__ __forceinline__ uint64_t load_sys(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the last of `total` arrivals on *c (thread 0 of each workgroup) resets it
__device__ __forceinline__ bool last_arrival(unsigned* c, unsigned total) {
  if (__hip_atomic_fetch_add(c, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) != total - 1) return false;
  __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

__global__ __launch_bounds__(kBlock) void ipc_exchange_kernel(Args a) {
  const bool send = blockIdx.x < a.sb;
  const int64_t rb = send ? blockIdx.x : blockIdx.x - a.sb;  // workgroup within the role
  const int64_t nrb = send ? a.sb : a.rb;
  const int k0 = send ? 0 : a.ns, k1 = send ? a.ns : a.ns + a.nr;  // the role's channels
  const int64_t c0 = a.cstart[k0], c1 = a.cstart[k1];
  const uint64_t e = __hip_atomic_load(a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  // send channels wait until the receiver has consumed the slot they are
  // about to overwrite (exchange e - 2); receive channels wait for "ready"
  const uint64_t lag = send ? 2 : 0;
  int k = k0;
  for (int64_t c = c0 + rb; c < c1; c += nrb) {
    while (k + 1 < k1 && c >= a.cstart[k + 1]) ++k;
    const gmt_ipc_chan& ch = a.c[k];
    if (threadIdx.x == 0 && ch.wait != nullptr && e > lag) {
      unsigned it = 0;
      while (load_sys(ch.wait) < e - lag) {
        __builtin_amdgcn_s_sleep(2);
        if (++it == kSpinLimit) {
          __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
    __syncthreads();
    const char* src = static_cast<const char*>(ch.src) + (e & 1) * ch.src_stride;
    char* dst = static_cast<char*>(ch.dst) + (e & 1) * ch.dst_stride;
    const int64_t lo = (c - a.cstart[k]) * kBlockBytes;
    const int64_t hi = lo + kBlockBytes < ch.bytes ? lo + kBlockBytes : ch.bytes;
    if ((((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) && ((hi - lo) & 15) == 0) {
      d2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = lo + 16 * (threadIdx.x + u * kBlock);
        if (o < hi) v[u] = *reinterpret_cast<const d2*>(src + o);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = lo + 16 * (threadIdx.x + u * kBlock);
        if (o < hi) *reinterpret_cast<d2*>(dst + o) = v[u];
      }
    } else {
      for (int64_t o = lo + threadIdx.x; o < hi; o += kBlock) dst[o] = src[o];
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    // each role signals on its own: a rank's "ready" must not wait for its
    // own receives (those wait for the peers' "ready")
    if (last_arrival(a.counter + (send ? 0 : 1), static_cast<unsigned>(nrb))) {
      for (int j = k0; j < k1; ++j)
        if (a.c[j].signal) __hip_atomic_store(a.c[j].signal, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (last_arrival(a.counter + 2, static_cast<unsigned>(a.sb + a.rb)))
      __hip_atomic_store(a.epoch, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// gmt_signal_wait: thread 0 polls the signal (uncached memory) with sleeps
__global__ __launch_bounds__(kWave) void signal_wait_kernel(const uint64_t* signal, uint64_t* seen, unsigned* err) {
  if (threadIdx.x != 0) return;
  const uint64_t want = __hip_atomic_load(seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  unsigned it = 0;
  while (__hip_atomic_load(const_cast<uint64_t*>(signal), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want) {
    __builtin_amdgcn_s_sleep(2);
    if (++it == kSpinLimit) {
      __hip_atomic_fetch_or(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
  __hip_atomic_store(seen, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace ipc
}  // namespace gmt

extern "C" int gmt_signal_wait(const uint64_t* signal, uint64_t* seen, unsigned* err, void* stream) {
  using namespace gmt;
  if (!signal || !seen || !err) return static_cast<int>(hipErrorInvalidValue);
  ipc::signal_wait_kernel<<<1, kWave, 0, static_cast<hipStream_t>(stream)>>>(signal, seen, err);
  GMT_RET_LAUNCH();
}

extern "C" int gmt_ipc_exchange(int n_send, const gmt_ipc_chan* sends, int n_recv, const gmt_ipc_chan* recvs,
                                uint64_t* epoch, unsigned* counters, unsigned* err, void* stream) {
  using namespace gmt;
  if (n_send < 0 || n_recv < 0 || n_send > GMT_IPC_MAX_CHAN || n_recv > GMT_IPC_MAX_CHAN || n_send + n_recv < 1 ||
      !epoch || !counters || !err)
    return static_cast<int>(hipErrorInvalidValue);
  ipc::Args a{};
  a.ns = n_send;
  a.nr = n_recv;
  a.epoch = epoch;
  a.counter = counters;
  a.err = err;
  a.cstart[0] = 0;
  for (int k = 0; k < n_send + n_recv; ++k) {
    const gmt_ipc_chan& c = k < n_send ? sends[k] : recvs[k - n_send];
    if (c.bytes < 0) return static_cast<int>(hipErrorInvalidValue);
    a.c[k] = c;
    // a zero-byte channel still takes one chunk: its wait and signal
    a.cstart[k + 1] = a.cstart[k] + (c.bytes > 0 ? (c.bytes + ipc::kBlockBytes - 1) / ipc::kBlockBytes : 1);
  }
  const int64_t sc = a.cstart[n_send], rc = a.cstart[n_send + n_recv] - sc;
  a.sb = sc < ipc::kMaxRoleBlocks ? sc : ipc::kMaxRoleBlocks;
  a.rb = rc < ipc::kMaxRoleBlocks ? rc : ipc::kMaxRoleBlocks;
  ipc::ipc_exchange_kernel<<<grid_1d(a.sb + a.rb), kBlock, 0, static_cast<hipStream_t>(stream)>>>(a);
  GMT_RET_LAUNCH();
}
