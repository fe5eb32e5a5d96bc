// HIP implementation of gmt/rt.h (gfx950 / ROCm 7.2).
//
// Maps the reference's CUDA runtime usage (cudaMalloc/cudaMallocHost/
// cudaMallocManaged, cudaMemcpy, cudaPointerGetAttributes,
// cudaMemRangeGetAttribute, cudaGetDeviceProperties — cuda_error.h:66-135,
// mpi_daxpy.cc:36-62, mpi_daxpy_nvtx.cc:177-205) and its cuBLAS DAXPY
// cross-check onto HIP, plus what the reference never had: high-priority
// streams for the halo path, IPC handles for peer/same-GPU direct copies and
// stream capture into hipGraphs for launch-bound loops.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "gmt/numa_bind.hpp"
#include "gmt/rt.h"

#define RT_RET(call) return static_cast<int>(call)

namespace {
inline hipStream_t S(gmt_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline hipEvent_t E(gmt_event_t e) { return reinterpret_cast<hipEvent_t>(e); }
}  // namespace

extern "C" {

int gmt_rt_backend(void) { return GMT_BACKEND_HIP; }
const char* gmt_rt_backend_name(void) { return "hip"; }
const char* gmt_rt_error_string(int err) { return hipGetErrorString(static_cast<hipError_t>(err)); }

int gmt_rt_device_count(int* n) { RT_RET(hipGetDeviceCount(n)); }
int gmt_rt_set_device(int dev) { RT_RET(hipSetDevice(dev)); }
int gmt_rt_get_device(int* dev) { RT_RET(hipGetDevice(dev)); }

int gmt_rt_device_info(int dev, gmt_device_info* out) {
  std::memset(out, 0, sizeof(*out));
  hipDeviceProp_t p;
  hipError_t e = hipGetDeviceProperties(&p, dev);
  if (e != hipSuccess) return static_cast<int>(e);
  std::snprintf(out->name, sizeof(out->name), "%s", p.name);
  if (out->name[0] == '\0') {  // some ROCm builds leave the marketing name empty
    char nm[256] = {0};
    if (hipDeviceGetName(nm, sizeof(nm), dev) != hipSuccess || nm[0] == '\0')
      std::snprintf(nm, sizeof(nm), "AMD GPU %.40s", p.gcnArchName);
    std::snprintf(out->name, sizeof(out->name), "%s", nm);
  }
  std::snprintf(out->arch, sizeof(out->arch), "%.63s", p.gcnArchName);
  out->total_mem = p.totalGlobalMem;
  out->vendor_id = 0x1002u;  // AMD PCI vendor id
  out->pci_domain = p.pciDomainID;
  out->pci_bus = p.pciBusID;
  out->pci_device = p.pciDeviceID;
  out->compute_units = p.multiProcessorCount;
  out->clock_khz = p.clockRate;
  out->l2_bytes = p.l2CacheSize;
  out->max_shared_per_block = static_cast<int>(p.sharedMemPerBlock);
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeManagedMemory, dev) == hipSuccess)
    out->managed_memory = v;
  v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeConcurrentManagedAccess, dev) == hipSuccess)
    out->concurrent_managed_access = v;
  out->xnack = std::strstr(p.gcnArchName, "xnack+") != nullptr;
  hipUUID u;
  if (hipDeviceGetUuid(&u, dev) == hipSuccess) {
    for (int i = 0; i < 16; ++i)
      std::snprintf(out->uuid + 2 * i, 3, "%02x", static_cast<unsigned char>(u.bytes[i]));
  }
  return 0;
}

int gmt_rt_mem_info(size_t* free_bytes, size_t* total_bytes) {
  RT_RET(hipMemGetInfo(free_bytes, total_bytes));
}
int gmt_rt_device_synchronize(void) { RT_RET(hipDeviceSynchronize()); }
int gmt_rt_device_reset(void) { RT_RET(hipDeviceReset()); }

int gmt_rt_malloc(void** p, size_t bytes, int space) {
  *p = nullptr;
  if (bytes == 0) bytes = 1;  // keep distinct non-null pointers for empty buffers
  switch (space) {
    case GMT_SPACE_DEVICE: RT_RET(hipMalloc(p, bytes));
    case GMT_SPACE_PINNED: RT_RET(hipHostMalloc(p, bytes, hipHostMallocDefault));
    case GMT_SPACE_PINNED_COHERENT: RT_RET(hipHostMalloc(p, bytes, hipHostMallocCoherent));
    case GMT_SPACE_MANAGED: RT_RET(hipMallocManaged(p, bytes, hipMemAttachGlobal));
    case GMT_SPACE_FLAGS: {
      hipError_t e = hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached);
      if (e == hipSuccess) e = hipMemset(*p, 0, bytes);
      RT_RET(e);
    }
    case GMT_SPACE_HOST: {
      // 64-B aligned so host staging buffers keep 16-B vector alignment
      if (posix_memalign(p, 64, bytes) != 0) return static_cast<int>(hipErrorOutOfMemory);
      return 0;
    }
    default: return static_cast<int>(hipErrorInvalidValue);
  }
}

int gmt_rt_free(void* p, int space) {
  if (!p) return 0;
  switch (space) {
    case GMT_SPACE_DEVICE:
    case GMT_SPACE_FLAGS:
    case GMT_SPACE_MANAGED: RT_RET(hipFree(p));
    case GMT_SPACE_PINNED:
    case GMT_SPACE_PINNED_COHERENT: RT_RET(hipHostFree(p));
    case GMT_SPACE_HOST: free(p); return 0;
    default: return static_cast<int>(hipErrorInvalidValue);
  }
}

int gmt_rt_memcpy(void* dst, const void* src, size_t bytes) {
  RT_RET(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
}
int gmt_rt_memcpy_async(void* dst, const void* src, size_t bytes, gmt_stream_t s) {
  RT_RET(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, S(s)));
}
int gmt_rt_memcpy2d_async(void* dst, size_t dpitch, const void* src, size_t spitch,
                          size_t width_bytes, size_t height, gmt_stream_t s) {
  RT_RET(hipMemcpy2DAsync(dst, dpitch, src, spitch, width_bytes, height, hipMemcpyDefault, S(s)));
}
int gmt_rt_memset_async(void* p, int value, size_t bytes, gmt_stream_t s) {
  RT_RET(hipMemsetAsync(p, value, bytes, S(s)));
}

int gmt_rt_pointer_space(const void* p, int* space) {
  *space = GMT_SPACE_UNREGISTERED;
  hipPointerAttribute_t a;
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky error of an unknown pointer
    return 0;
  }
  switch (a.type) {
    case hipMemoryTypeDevice: *space = GMT_SPACE_DEVICE; break;
    case hipMemoryTypeManaged: *space = GMT_SPACE_MANAGED; break;
    case hipMemoryTypeHost: *space = GMT_SPACE_PINNED; break;
    default: *space = GMT_SPACE_UNREGISTERED; break;
  }
  return 0;
}

int gmt_rt_mem_preferred_location(const void* p, size_t bytes, int* location) {
  int loc = -2;
  hipError_t e = hipMemRangeGetAttribute(&loc, sizeof(loc), hipMemRangeAttributePreferredLocation,
                                         p, bytes);
  *location = loc;
  RT_RET(e);
}

int gmt_rt_mem_prefetch_async(const void* p, size_t bytes, int device, gmt_stream_t s) {
  RT_RET(hipMemPrefetchAsync(p, bytes, device, S(s)));
}

int gmt_rt_stream_create(gmt_stream_t* s, int high_priority) {
  hipStream_t h = nullptr;
  hipError_t e;
  if (high_priority) {
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    e = hipStreamCreateWithPriority(&h, hipStreamNonBlocking, hi);
  } else {
    e = hipStreamCreateWithFlags(&h, hipStreamNonBlocking);
  }
  *s = reinterpret_cast<gmt_stream_t>(h);
  RT_RET(e);
}
int gmt_rt_stream_create_cumask(gmt_stream_t* s, int n_words, const uint32_t* mask) {
  hipStream_t h = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&h, static_cast<uint32_t>(n_words), mask);
  *s = reinterpret_cast<gmt_stream_t>(h);
  RT_RET(e);
}
int gmt_rt_bind_numa(int dev, int* node) {
  hipDeviceProp_t p;
  const hipError_t e = hipGetDeviceProperties(&p, dev);
  *node = e == hipSuccess ? gmt::bind_numa_near(p.pciDomainID, p.pciBusID, p.pciDeviceID) : -1;
  RT_RET(e);
}
int gmt_rt_pin_rank(int local_rank, int local_size, int ranks_per_device, int* cpu) {
  *cpu = -1;
  if (!gmt::pin_enabled(true) || local_size < 1 || local_rank < 0 || local_rank >= local_size) return 0;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev < 1) RT_RET(e);
  const int per = ranks_per_device > 0 ? ranks_per_device : 1;
  std::vector<int> dev_node(ndev, -1), rank_node(local_size, -1);
  for (int d = 0; d < ndev; ++d) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, d) == hipSuccess)
      dev_node[d] = gmt::pci_numa_node(p.pciDomainID, p.pciBusID, p.pciDeviceID);
  }
  for (int r = 0; r < local_size; ++r) rank_node[r] = dev_node[(r / per) % ndev];
  *cpu = gmt::pin_rank_core(local_rank, local_size, rank_node.data());
  return 0;
}
int gmt_rt_device_cu_count(int* n) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(n, hipDeviceAttributeMultiprocessorCount, dev);
  RT_RET(e);
}
int gmt_rt_stream_destroy(gmt_stream_t s) { RT_RET(s ? hipStreamDestroy(S(s)) : hipSuccess); }
int gmt_rt_stream_synchronize(gmt_stream_t s) { RT_RET(hipStreamSynchronize(S(s))); }
int gmt_rt_stream_wait_event(gmt_stream_t s, gmt_event_t e) {
  RT_RET(hipStreamWaitEvent(S(s), E(e), 0));
}
int gmt_rt_event_create(gmt_event_t* e, int enable_timing) {
  hipEvent_t h = nullptr;
  hipError_t r = hipEventCreateWithFlags(&h, enable_timing ? hipEventDefault : hipEventDisableTiming);
  *e = reinterpret_cast<gmt_event_t>(h);
  RT_RET(r);
}
int gmt_rt_event_destroy(gmt_event_t e) { RT_RET(e ? hipEventDestroy(E(e)) : hipSuccess); }
int gmt_rt_event_record(gmt_event_t e, gmt_stream_t s) { RT_RET(hipEventRecord(E(e), S(s))); }
int gmt_rt_event_synchronize(gmt_event_t e) { RT_RET(hipEventSynchronize(E(e))); }
int gmt_rt_event_query(gmt_event_t e) {
  hipError_t r = hipEventQuery(E(e));
  if (r == hipSuccess) return 0;
  if (r == hipErrorNotReady) return 1;
  return static_cast<int>(r);
}
int gmt_rt_stream_query(gmt_stream_t s) {
  hipError_t r = hipStreamQuery(S(s));
  if (r == hipSuccess) return 0;
  if (r == hipErrorNotReady) return 1;
  return static_cast<int>(r);
}
int gmt_rt_event_elapsed_ms(float* ms, gmt_event_t a, gmt_event_t b) {
  RT_RET(hipEventElapsedTime(ms, E(a), E(b)));
}

int gmt_rt_stream_begin_capture(gmt_stream_t s) {
  RT_RET(hipStreamBeginCapture(S(s), hipStreamCaptureModeThreadLocal));
}
int gmt_rt_stream_end_capture(gmt_stream_t s, gmt_graph_t* g) {
  hipGraph_t graph = nullptr;
  hipError_t e = hipStreamEndCapture(S(s), &graph);
  if (e != hipSuccess) return static_cast<int>(e);
  hipGraphExec_t exec = nullptr;
  e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  *g = reinterpret_cast<gmt_graph_t>(exec);
  RT_RET(e);
}
int gmt_rt_graph_launch(gmt_graph_t g, gmt_stream_t s) {
  RT_RET(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(g), S(s)));
}
int gmt_rt_graph_destroy(gmt_graph_t g) {
  RT_RET(g ? hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(g)) : hipSuccess);
}

int gmt_rt_ipc_get_handle(gmt_ipc_handle* h, size_t* offset, void* p) {
  static_assert(sizeof(hipIpcMemHandle_t) <= sizeof(gmt_ipc_handle), "ipc handle size");
  void* base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(reinterpret_cast<hipDeviceptr_t*>(&base), &size, p);
  if (e != hipSuccess) return static_cast<int>(e);
  hipIpcMemHandle_t mh;
  e = hipIpcGetMemHandle(&mh, base);
  if (e != hipSuccess) return static_cast<int>(e);
  std::memset(h, 0, sizeof(*h));
  std::memcpy(h->bytes, &mh, sizeof(mh));
  *offset = static_cast<size_t>(static_cast<char*>(p) - static_cast<char*>(base));
  return 0;
}
int gmt_rt_ipc_open(void** base, const gmt_ipc_handle* h) {
  hipIpcMemHandle_t mh;
  std::memcpy(&mh, h->bytes, sizeof(mh));
  RT_RET(hipIpcOpenMemHandle(base, mh, hipIpcMemLazyEnablePeerAccess));
}
int gmt_rt_ipc_close(void* base) { RT_RET(hipIpcCloseMemHandle(base)); }

// rocBLAS is dlopen'ed on first use: the cross-check path should not make
// every libgmt user (Python included) pay for loading the BLAS runtime.
typedef int (*rb_create_t)(void**);
typedef int (*rb_set_stream_t)(void*, hipStream_t);
typedef int (*rb_daxpy64_t)(void*, int64_t, const double*, const double*, int64_t, double*, int64_t);
typedef int (*rb_set_ptr_mode_t)(void*, int);
int gmt_blas_daxpy(int64_t n, double a, const double* x, double* y, gmt_stream_t s) {
  static void* lib = nullptr;
  static void* handle = nullptr;
  static rb_set_stream_t set_stream = nullptr;
  static rb_daxpy64_t daxpy = nullptr;
  if (!lib) {
    lib = dlopen("librocblas.so", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) lib = dlopen("/opt/rocm/lib/librocblas.so", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) {
      std::fprintf(stderr, "gmt_blas_daxpy: cannot load librocblas.so: %s\n", dlerror());
      return static_cast<int>(hipErrorSharedObjectInitFailed);
    }
    auto create = reinterpret_cast<rb_create_t>(dlsym(lib, "rocblas_create_handle"));
    set_stream = reinterpret_cast<rb_set_stream_t>(dlsym(lib, "rocblas_set_stream"));
    daxpy = reinterpret_cast<rb_daxpy64_t>(dlsym(lib, "rocblas_daxpy_64"));
    auto set_mode = reinterpret_cast<rb_set_ptr_mode_t>(dlsym(lib, "rocblas_set_pointer_mode"));
    if (!create || !set_stream || !daxpy || create(&handle) != 0)
      return static_cast<int>(hipErrorSharedObjectInitFailed);
    if (set_mode) set_mode(handle, 0 /* rocblas_pointer_mode_host */);
  }
  if (set_stream(handle, S(s)) != 0) return static_cast<int>(hipErrorInvalidValue);
  int st = daxpy(handle, n, &a, x, 1, y, 1);
  return st == 0 ? 0 : static_cast<int>(hipErrorLaunchFailure);
}

void gmt_trace_push(const char* name) { roctxRangePushA(name); }
void gmt_trace_pop(void) { roctxRangePop(); }
void gmt_trace_mark(const char* name) { roctxMarkA(name); }
void gmt_profiler_start(void) { roctxProfilerResume(0); }
void gmt_profiler_stop(void) { roctxProfilerPause(0); }

}  // extern "C"
