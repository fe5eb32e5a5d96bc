// Host (CPU) implementation of gmt/rt.h.
//
// "Device" and "managed" allocations are anonymous shared-memory files
// (memfd_create + mmap MAP_SHARED), so the HipIpc transport's
// export/open protocol has a faithful CPU analogue: another process on the
// node maps the same pages through /proc/<pid>/fd/<fd>.  Streams execute
// synchronously (every op is complete on return), events carry host
// timestamps, graphs are unsupported (callers fall back to eager launches).
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "gmt/numa_bind.hpp"
#include "gmt/rt.h"

namespace {

enum { kOk = 0, kInvalid = 1, kNoMem = 2, kUnsupported = 3, kNotReady = 4 };

struct Alloc {
  size_t bytes;
  int space;
  int fd;  // memfd for device/managed allocations, -1 otherwise
};

std::mutex g_mu;
std::map<uintptr_t, Alloc> g_allocs;   // base -> allocation
std::map<uintptr_t, size_t> g_opened;  // ipc-opened mappings
int g_device = 0;

struct IpcDesc {
  uint32_t magic;
  int32_t pid;
  int32_t fd;
  uint64_t bytes;
};
constexpr uint32_t kIpcMagic = 0x474d5448;  // "GMTH"

const Alloc* find_alloc(const void* p, uintptr_t* base) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  auto it = g_allocs.upper_bound(a);
  if (it == g_allocs.begin()) return nullptr;
  --it;
  if (a >= it->first && a < it->first + it->second.bytes) {
    if (base) *base = it->first;
    return &it->second;
  }
  return nullptr;
}

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

struct HostEvent {
  double t_ms = 0.0;
};

}  // namespace

extern "C" {

int gmt_rt_backend(void) { return GMT_BACKEND_HOST; }
const char* gmt_rt_backend_name(void) { return "host"; }
const char* gmt_rt_error_string(int err) {
  switch (err) {
    case kOk: return "success";
    case kInvalid: return "invalid value";
    case kNoMem: return "out of memory";
    case kUnsupported: return "not supported by the host backend";
    case kNotReady: return "not ready";
    default: return "unknown host-backend error";
  }
}

int gmt_rt_device_count(int* n) {
  *n = 1;
  return kOk;
}
int gmt_rt_set_device(int dev) {
  if (dev != 0) return kInvalid;
  g_device = dev;
  return kOk;
}
int gmt_rt_get_device(int* dev) {
  *dev = g_device;
  return kOk;
}

int gmt_rt_device_info(int dev, gmt_device_info* out) {
  if (dev != 0) return kInvalid;
  std::memset(out, 0, sizeof(*out));
  std::snprintf(out->name, sizeof(out->name), "host CPU (gmt host backend)");
  std::snprintf(out->arch, sizeof(out->arch), "host");
  const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGE_SIZE);
  out->total_mem = (pages > 0 && psz > 0) ? static_cast<size_t>(pages) * psz : 0;
  out->vendor_id = 0;
  out->compute_units = static_cast<int>(sysconf(_SC_NPROCESSORS_ONLN));
  out->managed_memory = 1;
  out->concurrent_managed_access = 1;
  return kOk;
}

int gmt_rt_mem_info(size_t* free_bytes, size_t* total_bytes) {
  const long pages = sysconf(_SC_PHYS_PAGES), avail = sysconf(_SC_AVPHYS_PAGES),
             psz = sysconf(_SC_PAGE_SIZE);
  *total_bytes = static_cast<size_t>(pages) * psz;
  *free_bytes = static_cast<size_t>(avail) * psz;
  return kOk;
}
int gmt_rt_device_synchronize(void) { return kOk; }
int gmt_rt_device_reset(void) { return kOk; }

int gmt_rt_malloc(void** p, size_t bytes, int space) {
  *p = nullptr;
  if (bytes == 0) bytes = 1;
  if (space == GMT_SPACE_DEVICE || space == GMT_SPACE_MANAGED || space == GMT_SPACE_FLAGS) {
    // memfd pages start zeroed (GMT_SPACE_FLAGS relies on it)
    const int fd = memfd_create("gmt_dev", MFD_CLOEXEC);
    if (fd < 0) return kNoMem;
    if (ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
      close(fd);
      return kNoMem;
    }
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) {
      close(fd);
      return kNoMem;
    }
    std::lock_guard<std::mutex> g(g_mu);
    g_allocs[reinterpret_cast<uintptr_t>(m)] = Alloc{bytes, space, fd};
    *p = m;
    return kOk;
  }
  if (space == GMT_SPACE_PINNED || space == GMT_SPACE_PINNED_COHERENT || space == GMT_SPACE_HOST) {
    if (posix_memalign(p, 64, bytes) != 0) return kNoMem;
    std::memset(*p, 0, bytes);
    if (space != GMT_SPACE_HOST) {
      std::lock_guard<std::mutex> g(g_mu);
      g_allocs[reinterpret_cast<uintptr_t>(*p)] = Alloc{bytes, space, -1};
    }
    return kOk;
  }
  return kInvalid;
}

int gmt_rt_free(void* p, int space) {
  if (!p) return kOk;
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_allocs.find(reinterpret_cast<uintptr_t>(p));
  if (space == GMT_SPACE_HOST) {
    free(p);
    return kOk;
  }
  if (it == g_allocs.end()) return kInvalid;
  if (it->second.fd >= 0) {
    munmap(p, it->second.bytes);
    close(it->second.fd);
  } else {
    free(p);
  }
  g_allocs.erase(it);
  return kOk;
}

int gmt_rt_memcpy(void* dst, const void* src, size_t bytes) {
  std::memmove(dst, src, bytes);
  return kOk;
}
int gmt_rt_memcpy_async(void* dst, const void* src, size_t bytes, gmt_stream_t) {
  std::memmove(dst, src, bytes);
  return kOk;
}
int gmt_rt_memcpy2d_async(void* dst, size_t dpitch, const void* src, size_t spitch,
                          size_t width_bytes, size_t height, gmt_stream_t) {
  for (size_t r = 0; r < height; ++r)
    std::memmove(static_cast<char*>(dst) + r * dpitch, static_cast<const char*>(src) + r * spitch,
                 width_bytes);
  return kOk;
}
int gmt_rt_memset_async(void* p, int value, size_t bytes, gmt_stream_t) {
  std::memset(p, value, bytes);
  return kOk;
}

int gmt_rt_pointer_space(const void* p, int* space) {
  std::lock_guard<std::mutex> g(g_mu);
  const Alloc* a = find_alloc(p, nullptr);
  *space = a ? a->space : GMT_SPACE_UNREGISTERED;
  return kOk;
}

int gmt_rt_mem_preferred_location(const void* p, size_t, int* location) {
  std::lock_guard<std::mutex> g(g_mu);
  const Alloc* a = find_alloc(p, nullptr);
  if (!a || a->space != GMT_SPACE_MANAGED) {
    *location = -2;
    return kInvalid;
  }
  *location = -1;  // host memory is the only location
  return kOk;
}
int gmt_rt_mem_prefetch_async(const void*, size_t, int, gmt_stream_t) { return kOk; }

int gmt_rt_stream_create(gmt_stream_t* s, int) {
  // distinct non-null handles; nothing to execute asynchronously
  *s = reinterpret_cast<gmt_stream_t>(new char[1]);
  return kOk;
}
int gmt_rt_stream_create_cumask(gmt_stream_t* s, int, const uint32_t*) { return gmt_rt_stream_create(s, 0); }
int gmt_rt_bind_numa(int, int* node) {
  *node = -1;
  return kOk;
}
// the CPU backend: off by default (the CPU test suite runs many jobs side by
// side; pinning every job's rank 0 to one core would serialise them)
int gmt_rt_pin_rank(int local_rank, int local_size, int, int* cpu) {
  *cpu = -1;
  if (!gmt::pin_enabled(false) || local_size < 1 || local_rank < 0 || local_rank >= local_size) return kOk;
  std::vector<int> rank_node(local_size, -1);
  *cpu = gmt::pin_rank_core(local_rank, local_size, rank_node.data());
  return kOk;
}
int gmt_rt_device_cu_count(int* n) {
  *n = 1;
  return kOk;
}
int gmt_rt_stream_destroy(gmt_stream_t s) {
  delete[] reinterpret_cast<char*>(s);
  return kOk;
}
int gmt_rt_stream_synchronize(gmt_stream_t) { return kOk; }
int gmt_rt_stream_wait_event(gmt_stream_t, gmt_event_t) { return kOk; }
int gmt_rt_event_create(gmt_event_t* e, int) {
  *e = reinterpret_cast<gmt_event_t>(new HostEvent());
  return kOk;
}
int gmt_rt_event_destroy(gmt_event_t e) {
  delete reinterpret_cast<HostEvent*>(e);
  return kOk;
}
int gmt_rt_event_record(gmt_event_t e, gmt_stream_t) {
  reinterpret_cast<HostEvent*>(e)->t_ms = now_ms();
  return kOk;
}
int gmt_rt_event_synchronize(gmt_event_t) { return kOk; }
int gmt_rt_event_query(gmt_event_t) { return kOk; }
int gmt_rt_stream_query(gmt_stream_t) { return kOk; }
int gmt_rt_event_elapsed_ms(float* ms, gmt_event_t a, gmt_event_t b) {
  *ms = static_cast<float>(reinterpret_cast<HostEvent*>(b)->t_ms -
                           reinterpret_cast<HostEvent*>(a)->t_ms);
  return kOk;
}
int gmt_rt_stream_begin_capture(gmt_stream_t) { return kUnsupported; }
int gmt_rt_stream_end_capture(gmt_stream_t, gmt_graph_t* g) {
  *g = nullptr;
  return kUnsupported;
}
int gmt_rt_graph_launch(gmt_graph_t, gmt_stream_t) { return kUnsupported; }
int gmt_rt_graph_destroy(gmt_graph_t) { return kOk; }

int gmt_rt_ipc_get_handle(gmt_ipc_handle* h, size_t* offset, void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  uintptr_t base = 0;
  const Alloc* a = find_alloc(p, &base);
  if (!a || a->fd < 0) return kInvalid;
  IpcDesc d{kIpcMagic, static_cast<int32_t>(getpid()), a->fd, a->bytes};
  std::memset(h, 0, sizeof(*h));
  std::memcpy(h->bytes, &d, sizeof(d));
  *offset = reinterpret_cast<uintptr_t>(p) - base;
  return kOk;
}

int gmt_rt_ipc_open(void** base, const gmt_ipc_handle* h) {
  IpcDesc d;
  std::memcpy(&d, h->bytes, sizeof(d));
  if (d.magic != kIpcMagic) return kInvalid;
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/fd/%d", d.pid, d.fd);
  const int fd = open(path, O_RDWR | O_CLOEXEC);
  if (fd < 0) return kInvalid;
  void* m = mmap(nullptr, d.bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return kNoMem;
  std::lock_guard<std::mutex> g(g_mu);
  g_opened[reinterpret_cast<uintptr_t>(m)] = d.bytes;
  *base = m;
  return kOk;
}

int gmt_rt_ipc_close(void* base) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_opened.find(reinterpret_cast<uintptr_t>(base));
  if (it == g_opened.end()) return kInvalid;
  munmap(base, it->second);
  g_opened.erase(it);
  return kOk;
}

int gmt_blas_daxpy(int64_t n, double a, const double* x, double* y, gmt_stream_t) {
  for (int64_t i = 0; i < n; ++i) y[i] += a * x[i];
  return kOk;
}

void gmt_trace_push(const char*) {}
void gmt_trace_pop(void) {}
void gmt_trace_mark(const char*) {}
void gmt_profiler_start(void) {}
void gmt_profiler_stop(void) {}

}  // extern "C"
