/*
 * gmt/rt.h — device-runtime C ABI shared by every native binary.
 *
 * Two implementations with the same symbols and the same SONAME (libgmt.so):
 *   * HIP   (csrc/runtime/rt_hip.cpp, built with hipcc for gfx950) —
 *     gpu_mpi_tests_amd/_lib/libgmt.so;
 *   * host  (csrc/host/rt_host.cpp, plain C++) — build/lib-host/libgmt.so,
 *     the CPU backend that mirrors the reference's gtensor `host` device
 *     (/root/reference/CMakeLists.txt:59-69) so the MPI apps and their tests
 *     run without a GPU.
 * The apps (csrc/apps) are compiled once against this header and linked
 * twice (build/bin = HIP, build/bin-host = host).  They never include HIP
 * headers, which is what keeps them single-source without any
 * multi-backend #ifdef.
 *
 * Replaces the reference's per-binary CUDA runtime use and its error/pointer
 * introspection header (/root/reference/cuda_error.h:1-136).
 * Every function returns 0 on success or a backend error code (hipError_t
 * for the HIP build); gmt_rt_error_string() decodes it.
 */
#ifndef GMT_RT_H
#define GMT_RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gmt_stream_s* gmt_stream_t; /* NULL = the default (null) stream */
typedef struct gmt_event_s* gmt_event_t;
typedef struct gmt_graph_s* gmt_graph_t;

/* memory spaces (reference: malloc / cudaMalloc / cudaMallocHost / cudaMallocManaged) */
enum gmt_space {
  GMT_SPACE_HOST = 0,    /* pageable host memory (plain malloc)            */
  GMT_SPACE_DEVICE = 1,  /* device HBM (hipMalloc)                          */
  GMT_SPACE_PINNED = 2,  /* page-locked host memory (hipHostMalloc)         */
  GMT_SPACE_MANAGED = 3, /* unified/managed memory (hipMallocManaged)       */
  GMT_SPACE_FLAGS = 4,   /* device memory for cross-process flags: uncached
                            (every access reaches memory), zeroed, exportable
                            by IPC (hipExtMallocWithFlags Uncached)       */
  GMT_SPACE_PINNED_COHERENT = 5, /* page-locked host memory the GPU writes
                            through (hipHostMallocCoherent): kernel-driven
                            staging and GPU -> host completion flags      */
  GMT_SPACE_UNREGISTERED = -1
};

enum gmt_backend { GMT_BACKEND_HOST = 0, GMT_BACKEND_HIP = 1 };

typedef struct gmt_device_info {
  char name[256];
  char arch[64];            /* e.g. "gfx950:sramecc+:xnack-" */
  size_t total_mem;         /* bytes of device memory */
  uint32_t vendor_id;       /* PCI vendor id: 0x1002 for AMD, 0 for the host backend */
  int pci_domain, pci_bus, pci_device;
  char uuid[40];            /* hex string, may be empty */
  int compute_units;
  int clock_khz;
  int managed_memory;             /* hipDeviceAttributeManagedMemory */
  int concurrent_managed_access;  /* page-migrating managed memory (XNACK on) */
  int xnack;                      /* arch string reports xnack+ */
  int l2_bytes;
  int max_shared_per_block;       /* LDS bytes per workgroup */
} gmt_device_info;

typedef struct gmt_ipc_handle {
  unsigned char bytes[64]; /* hipIpcMemHandle_t (64 B) or the host backend's memfd descriptor */
} gmt_ipc_handle;

/* ---- backend / devices */
int gmt_rt_backend(void);
const char* gmt_rt_backend_name(void);
const char* gmt_rt_error_string(int err);
int gmt_rt_device_count(int* n);
int gmt_rt_set_device(int dev);
int gmt_rt_get_device(int* dev);
int gmt_rt_device_info(int dev, gmt_device_info* out);
int gmt_rt_mem_info(size_t* free_bytes, size_t* total_bytes);
int gmt_rt_device_synchronize(void);
int gmt_rt_device_reset(void);

/* ---- memory */
int gmt_rt_malloc(void** p, size_t bytes, int space);
int gmt_rt_free(void* p, int space);
int gmt_rt_memcpy(void* dst, const void* src, size_t bytes); /* synchronous, any direction */
int gmt_rt_memcpy_async(void* dst, const void* src, size_t bytes, gmt_stream_t s);
/* strided 2-D copy: `height` rows of `width_bytes`, pitches in bytes (DMA engine) */
int gmt_rt_memcpy2d_async(void* dst, size_t dpitch, const void* src, size_t spitch,
                          size_t width_bytes, size_t height, gmt_stream_t s);
int gmt_rt_memset_async(void* p, int value, size_t bytes, gmt_stream_t s);
/* PTRINFO: which space a pointer lives in (GMT_SPACE_*; UNREGISTERED if unknown) */
int gmt_rt_pointer_space(const void* p, int* space);
/* MEMINFO: managed-range preferred location: >=0 device id, -1 CPU, -2 invalid */
int gmt_rt_mem_preferred_location(const void* p, size_t bytes, int* location);
int gmt_rt_mem_prefetch_async(const void* p, size_t bytes, int device, gmt_stream_t s);

/* ---- streams / events / graphs */
int gmt_rt_stream_create(gmt_stream_t* s, int high_priority);
/* A stream whose kernels run only on the compute units whose bits are set
   in mask[0..n_words) (bit i of word w = CU 32 w + i; hipExtStreamCreateWithCUMask).
   The host backend ignores the mask. */
int gmt_rt_stream_create_cumask(gmt_stream_t* s, int n_words, const uint32_t* mask);
/* compute units of the current device */
int gmt_rt_device_cu_count(int* n);
/* Bind every thread of the process to the CPUs of device dev's NUMA node
   (gmt/numa_bind.hpp; opt-in: GMT_NUMA_BIND=1).  *node = the node, or -1
   when nothing changed (the host backend: always -1). */
int gmt_rt_bind_numa(int dev, int* node);
/* Pin every thread of this process to one physical core near its GPU
   (gmt/numa_bind.hpp pin_rank_core): local ranks map to devices by the
   reference's block rule (ranks_per_device ranks per GPU, local rank r on
   device r / ranks_per_device), the ranks sharing a NUMA node take distinct
   cores.  Default on with the HIP backend, off on the host backend;
   GMT_PIN=0/1 overrides.  *cpu = the core's first CPU, or -1 when nothing
   changed. */
int gmt_rt_pin_rank(int local_rank, int local_size, int ranks_per_device, int* cpu);
int gmt_rt_stream_destroy(gmt_stream_t s);
int gmt_rt_stream_synchronize(gmt_stream_t s);
int gmt_rt_stream_wait_event(gmt_stream_t s, gmt_event_t e);
int gmt_rt_event_create(gmt_event_t* e, int enable_timing);
int gmt_rt_event_destroy(gmt_event_t e);
int gmt_rt_event_record(gmt_event_t e, gmt_stream_t s);
int gmt_rt_event_synchronize(gmt_event_t e);
int gmt_rt_event_query(gmt_event_t e); /* 0 = complete, 1 = pending, else error */
int gmt_rt_stream_query(gmt_stream_t s); /* 0 = idle, 1 = work pending, else the stream's error */
int gmt_rt_event_elapsed_ms(float* ms, gmt_event_t start, gmt_event_t end);
int gmt_rt_stream_begin_capture(gmt_stream_t s);
int gmt_rt_stream_end_capture(gmt_stream_t s, gmt_graph_t* g);
int gmt_rt_graph_launch(gmt_graph_t g, gmt_stream_t s);
int gmt_rt_graph_destroy(gmt_graph_t g);

/* ---- inter-process memory (HIP IPC over xGMI / same device; memfd on host) */
/* handle of the allocation containing `p` plus p's byte offset inside it */
int gmt_rt_ipc_get_handle(gmt_ipc_handle* h, size_t* offset, void* p);
int gmt_rt_ipc_open(void** base, const gmt_ipc_handle* h);
int gmt_rt_ipc_close(void* base);

/* ---- BLAS cross-check (rocBLAS on HIP; loop on host).  reference: cublasDaxpy */
int gmt_blas_daxpy(int64_t n, double a, const double* x, double* y, gmt_stream_t s);

/* ---- tracing: roctx ranges + profiler capture window (reference NVTX +
 *      cudaProfilerStart/Stop, daxpy_nvtx.cu:65-105, mpi_daxpy_nvtx.cc:167-328) */
void gmt_trace_push(const char* name);
void gmt_trace_pop(void);
void gmt_trace_mark(const char* name);
void gmt_profiler_start(void);
void gmt_profiler_stop(void);

#ifdef __cplusplus
}
#endif
#endif /* GMT_RT_H */
