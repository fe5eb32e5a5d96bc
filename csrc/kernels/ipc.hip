// Stream-ordered IPC exchange (gmt_ipc_exchange, gmt/kernels.h), gfx950.
//
// The halo transport "ipc" (csrc/comm/transport_ipc.cpp) runs every
// exchange as ONE launch on the caller's stream — no host synchronisation,
// no control-plane rounds, so the exchange can be captured into a hipGraph.
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
// The channel table lives in device memory (gmt_ipc_plan_init), so a plan
// has any number of channels (an all-gather over 63 peers is 126) and the
// launch arguments stay a few words — the same bytes in a replayed graph.
// The epoch lives in device memory too (read at the start, advanced by the
// last workgroup), so replayed graphs stay in step.
//
// Flags are GMT_SPACE_FLAGS memory (uncached); loads and stores of them are
// vector atomics at system scope.  Every wait is bounded by the device wall
// clock (GMT_WAIT_TIMEOUT_MS, default 10 s): a wait that expires stores
// 1 + its channel index into the plan's error word (host-visible pinned
// memory, read by the host after each synchronisation) and gives up, so a
// lost peer can neither hang the GPU nor pass unnoticed.
#include <cstdlib>

#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {
namespace ipc {

constexpr int64_t kBlockBytes = 16 * 1024;  // bytes per chunk: 4 x 16 B per lane
constexpr int64_t kMaxRoleBlocks = 128;     // workgroups per role: spinning groups never fill the GPU

struct Args {
  const gmt_ipc_chan* chan;  // sends, then receives (device memory)
  const int64_t* cstart;     // prefix sum of chunks per channel, n_send + n_recv + 1 entries
  int ns, nr;
  int64_t sb, rb;  // workgroups of the send role, then of the receive role
  uint64_t* epoch;
  unsigned* counter;  // [0] send role, [1] receive role, [2] all
  unsigned* err;
  uint64_t timeout_ticks;  // device wall-clock ticks per wait
};


// the last of `total` arrivals on *c (thread 0 of each workgroup) resets it
__device__ __forceinline__ bool last_arrival(unsigned* c, unsigned total) {
  if (__hip_atomic_fetch_add(c, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) != total - 1) return false;
  __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// Poll *flag until it reaches `want` or the wall clock runs out; on timeout
// record `code` in *err (a plain system-scope store: any non-zero is an error).
// Once an exchange of the plan has failed, later ones do not wait again (the
// host aborts at its next synchronisation; queued exchanges drain quickly).
// (relaxed polls of the uncached flag, one system-scope acquire after the
// flag is seen: an acquire per poll would invalidate the caches every time)
__device__ __forceinline__ void bounded_wait(const uint64_t* flag, uint64_t want, uint64_t ticks, unsigned* err,
                                             unsigned code) {
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(const_cast<uint64_t*>(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > ticks) {
      __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // system scope: the peer's data is read after this
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
    const gmt_ipc_chan ch = a.chan[k];
    if (threadIdx.x == 0 && ch.wait != nullptr && e > lag)
      bounded_wait(ch.wait, e - lag, a.timeout_ticks, a.err, static_cast<unsigned>(k + 1));
    __syncthreads();
    const char* src = static_cast<const char*>(ch.src) + (e & 1) * ch.src_stride;
    char* dst = static_cast<char*>(ch.dst) + (e & 1) * ch.dst_stride;
    const int64_t lo = (c - a.cstart[k]) * kBlockBytes;
    const int64_t hi = lo + kBlockBytes < ch.bytes ? lo + kBlockBytes : ch.bytes;
    // a strided side maps message byte o to run o / run_bytes at o % run_bytes
    // (faces are far below 4 GiB: 32-bit division)
    auto at = [](int64_t o, int64_t run, int64_t ld) -> int64_t {
      if (run == 0) return o;
      const uint32_t q = static_cast<uint32_t>(o) / static_cast<uint32_t>(run);
      return static_cast<int64_t>(q) * ld + (o - static_cast<int64_t>(q) * run);
    };
    const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) |
                         static_cast<uintptr_t>(ch.src_run | ch.src_ld | ch.dst_run | ch.dst_ld);
    if ((al & 15) == 0 && ((hi - lo) & 15) == 0) {
      d2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = lo + 16 * (threadIdx.x + u * kBlock);
        if (o < hi) v[u] = *reinterpret_cast<const d2*>(src + at(o, ch.src_run, ch.src_ld));
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = lo + 16 * (threadIdx.x + u * kBlock);
        if (o < hi) *reinterpret_cast<d2*>(dst + at(o, ch.dst_run, ch.dst_ld)) = v[u];
      }
    } else {
      for (int64_t o = lo + threadIdx.x; o < hi; o += kBlock)
        dst[at(o, ch.dst_run, ch.dst_ld)] = src[at(o, ch.src_run, ch.src_ld)];
    }
  }
  // every wave's copies complete (the barrier waits for them), then ONE
  // system-scope release for the workgroup: the L2 writeback it implies
  // covers every wave's stores, four of them cost four writebacks
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    // each role signals on its own: a rank's "ready" must not wait for its
    // own receives (those wait for the peers' "ready")
    if (last_arrival(a.counter + (send ? 0 : 1), static_cast<unsigned>(nrb))) {
      // the other workgroups' data reached this one through their fence ->
      // counter RMW -> this acquire; one system-scope release here makes the
      // chain a formal release sequence for the peer's acquire of the
      // signal (one thread, once per exchange)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      for (int j = k0; j < k1; ++j) {
        uint64_t* sig = a.chan[j].signal;
        if (sig) __hip_atomic_store(sig, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (last_arrival(a.counter + 2, static_cast<unsigned>(a.sb + a.rb)))
      __hip_atomic_store(a.epoch, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// gmt_signal_wait: thread 0 polls the signal (uncached memory) with sleeps
__global__ __launch_bounds__(kWave) void signal_wait_kernel(const uint64_t* signal, uint64_t* seen, unsigned* err,
                                                           uint64_t ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t want = __hip_atomic_load(seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(const_cast<uint64_t*>(signal), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want) {
    __builtin_amdgcn_s_sleep(4);
    if (wall_clock64() - t0 > ticks) {
      __hip_atomic_fetch_or(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
  __hip_atomic_store(seen, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// gmt_push_sync: the hand-over between two inline-halo passes (the pass
// kernel stored its output faces straight into the neighbours' ghost cells,
// gmt_tb_opts.push).  One workgroup per XCD (workgroups are dealt to the 8
// XCDs round robin): workgroup 0 tells every neighbour that this rank's
// pass, faces included, is complete; every workgroup then waits for every
// neighbour's word and acquires at system scope, so no XCD's L2 keeps a
// stale copy of the ghost cells the neighbours just wrote.  Why push and
// not pull: a strided W / E face would need its own exchange launch between
// the passes (pack or copy kernel, the 9-10% of round 4); written by the
// pass itself it costs a few store instructions and this launch.
//
// Which mechanism makes the pushed cells visible to the next pass: the
// writer's system-scope release (above) and, on this side, an acquire on
// every XCD's L2.  Two acquires cover that: the system-scope fence at the
// end of this kernel, run by one workgroup on each XCD — the dispatcher
// deals the workgroups of a launch to the XCDs round robin, starting where
// the previous launch left off (workgroup i on XCD (x0 + i) mod 8), so the 8
// workgroups of this launch cover the 8 XCDs whatever x0;
// tests/test_kernels_gpu.py::test_workgroups_round_robin_over_xcds asserts
// it with gmt_xcd_of_workgroups — and the acquire fence of the next kernel's
// dispatch packet.
struct PushSyncArgs {
  const uint64_t* local;
  uint64_t* remote[8];
  uint64_t epoch;
  unsigned* err;
  unsigned* stop;
  uint64_t ticks;
  int mask;
};

__global__ __launch_bounds__(kWave) void push_sync_kernel(PushSyncArgs a) {
  const int d = threadIdx.x;
  // stopped (an earlier wait expired): no signal, no wait — the passes
  // return at entry and the host aborts at its next synchronisation
  if (a.stop && __hip_atomic_load(a.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  const bool mine = d < 8 && ((a.mask >> d) & 1);
  if (blockIdx.x == 0 && mine) {
    // the pass's face stores are complete: its waves drained vmcnt and the
    // pass finished before this launch (stream order)
    __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope
    __hip_atomic_store(a.remote[d], a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (mine) {
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(const_cast<uint64_t*>(a.local + d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) <
           a.epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > a.ticks) {
        __hip_atomic_fetch_or(a.err, 1u << d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (a.stop) __hip_atomic_fetch_or(a.stop, 1u << d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // system scope, on this workgroup's XCD
}

// per-wait bound in device wall-clock ticks (GMT_WAIT_TIMEOUT_MS, default 10 s)
uint64_t timeout_ticks() {
  static int dev_cached = -1;
  static uint64_t ticks = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (dev != dev_cached) {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
      khz = 100000;  // 100 MHz, the CDNA constant clock
    const char* e = std::getenv("GMT_WAIT_TIMEOUT_MS");
    const long ms = e && std::atol(e) > 0 ? std::atol(e) : 10000;
    ticks = static_cast<uint64_t>(ms) * static_cast<uint64_t>(khz);
    dev_cached = dev;
  }
  return ticks;
}

}  // namespace ipc
}  // namespace gmt

extern "C" int gmt_signal_wait(const uint64_t* signal, uint64_t* seen, unsigned* err, void* stream) {
  using namespace gmt;
  if (!signal || !seen || !err) return static_cast<int>(hipErrorInvalidValue);
  ipc::signal_wait_kernel<<<1, kWave, 0, static_cast<hipStream_t>(stream)>>>(signal, seen, err,
                                                                           ipc::timeout_ticks());
  GMT_RET_LAUNCH();
}

extern "C" int64_t gmt_ipc_table_bytes(int n_chan) {
  if (n_chan < 0) return 0;
  return static_cast<int64_t>(n_chan) * static_cast<int64_t>(sizeof(gmt_ipc_chan)) +
         (static_cast<int64_t>(n_chan) + 1) * static_cast<int64_t>(sizeof(int64_t));
}

extern "C" int gmt_ipc_plan_init(gmt_ipc_plan* p, int n_send, const gmt_ipc_chan* sends, int n_recv,
                                 const gmt_ipc_chan* recvs) {
  using namespace gmt;
  if (!p || !p->table || n_send < 0 || n_recv < 0 || n_send + n_recv < 1) return static_cast<int>(hipErrorInvalidValue);
  const int n = n_send + n_recv;
  char* host = static_cast<char*>(std::malloc(static_cast<size_t>(gmt_ipc_table_bytes(n))));
  if (!host) return static_cast<int>(hipErrorOutOfMemory);
  auto* c = reinterpret_cast<gmt_ipc_chan*>(host);
  auto* cs = reinterpret_cast<int64_t*>(host + static_cast<size_t>(n) * sizeof(gmt_ipc_chan));
  cs[0] = 0;
  for (int k = 0; k < n; ++k) {
    c[k] = k < n_send ? sends[k] : recvs[k - n_send];
    // strided sides: whole runs, a pitch no shorter than the run, offsets
    // that fit the kernel's 32-bit division
    auto bad_side = [&](int64_t run, int64_t ld) {
      return run < 0 || (run > 0 && (ld < run || c[k].bytes % run != 0 || c[k].bytes > 0xffffffffll));
    };
    if (c[k].bytes < 0 || bad_side(c[k].src_run, c[k].src_ld) || bad_side(c[k].dst_run, c[k].dst_ld)) {
      std::free(host);
      return static_cast<int>(hipErrorInvalidValue);
    }
    // a zero-byte channel still takes one chunk: its wait and signal
    cs[k + 1] = cs[k] + (c[k].bytes > 0 ? (c[k].bytes + ipc::kBlockBytes - 1) / ipc::kBlockBytes : 1);
  }
  p->n_send = n_send;
  p->n_recv = n_recv;
  p->send_chunks = cs[n_send];
  p->recv_chunks = cs[n] - cs[n_send];
  const hipError_t e = hipMemcpy(p->table, host, static_cast<size_t>(gmt_ipc_table_bytes(n)), hipMemcpyHostToDevice);
  std::free(host);
  return static_cast<int>(e);
}

extern "C" int gmt_ipc_exchange(const gmt_ipc_plan* p, void* stream) {
  using namespace gmt;
  if (!p || !p->table || !p->epoch || !p->counters || !p->err || p->n_send < 0 || p->n_recv < 0 ||
      p->n_send + p->n_recv < 1)
    return static_cast<int>(hipErrorInvalidValue);
  const int n = p->n_send + p->n_recv;
  ipc::Args a{};
  a.chan = static_cast<const gmt_ipc_chan*>(p->table);
  a.cstart = reinterpret_cast<const int64_t*>(static_cast<const char*>(p->table) + static_cast<size_t>(n) * sizeof(gmt_ipc_chan));
  a.ns = p->n_send;
  a.nr = p->n_recv;
  a.epoch = p->epoch;
  a.counter = p->counters;
  a.err = p->err;
  a.timeout_ticks = ipc::timeout_ticks();
  a.sb = p->send_chunks < ipc::kMaxRoleBlocks ? p->send_chunks : ipc::kMaxRoleBlocks;
  a.rb = p->recv_chunks < ipc::kMaxRoleBlocks ? p->recv_chunks : ipc::kMaxRoleBlocks;
  if (a.sb + a.rb < 1) return static_cast<int>(hipErrorInvalidValue);
  ipc::ipc_exchange_kernel<<<grid_1d(a.sb + a.rb), kBlock, 0, static_cast<hipStream_t>(stream)>>>(a);
  GMT_RET_LAUNCH();
}

extern "C" int gmt_push_sync(const uint64_t* local, uint64_t* const remote[8], int mask, uint64_t epoch, unsigned* err,
                             unsigned* stop, void* stream) {
  using namespace gmt;
  if (!local || !err || mask < 0 || mask > 255) return static_cast<int>(hipErrorInvalidValue);
  ipc::PushSyncArgs a{};
  a.local = local;
  for (int d = 0; d < 8; ++d) {
    a.remote[d] = remote ? remote[d] : nullptr;
    if (((mask >> d) & 1) && !a.remote[d]) return static_cast<int>(hipErrorInvalidValue);
  }
  a.epoch = epoch;
  a.err = err;
  a.stop = stop;
  a.ticks = ipc::timeout_ticks();
  a.mask = mask;
  if (mask == 0) return 0;
  ipc::push_sync_kernel<<<kNumXcd, kWave, 0, static_cast<hipStream_t>(stream)>>>(a);
  GMT_RET_LAUNCH();
}

namespace gmt {
namespace ipc {
__global__ __launch_bounds__(kWave) void xcd_probe_kernel(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xfu;  // XCC_ID
}
}  // namespace ipc
}  // namespace gmt

extern "C" int gmt_xcd_of_workgroups(int n, unsigned* out, void* stream) {
  using namespace gmt;
  if (n < 1 || n > 4096 || !out) return static_cast<int>(hipErrorInvalidValue);
  ipc::xcd_probe_kernel<<<n, kWave, 0, static_cast<hipStream_t>(stream)>>>(out);
  GMT_RET_LAUNCH();
}
