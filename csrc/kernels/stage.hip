// Kernel-driven host staging (gmt_stage_copy, gmt/kernels.h), gfx950.
//
// The mpi-host transport stages every halo message through page-locked host
// memory for a non-GPU-aware MPI (the reference's stage_host / buf:1 path,
// mpi_stencil2d_gt.cc:147-176, mpi_stencil2d_sycl.cc:248-283).  Round 2 did
// the device -> host leg as one SDMA hipMemcpyAsync per 1 MiB chunk with an
// event after each: 6.9 GB/s per rank at 8 MiB against 25 GB/s for MPI
// itself (profiles/r02_xport2).  Here the CUs write the staging buffers
// directly over PCIe (posted writes, many workgroups in flight), and each
// chunk publishes its own completion flag in coherent host memory, so the
// host sends chunk k while chunks k+1.. are still being written — one launch
// per exchange instead of one copy command and one event per chunk.
#include "common.hpp"
#include "gmt/kernels.h"

namespace gmt {
namespace stage {

// packed doubles [first, first + n) of a column-major block (rows per column,
// pitch ld) <-> a contiguous run: one double per lane per step (halo faces
// are 2..20 rows deep, so a column's rows are adjacent lanes: one 16..160-B
// run per column, the field read or written once)
template <bool GATHER>
__device__ __forceinline__ void strided_part(const gmt_stage_chunk& c, int part, int g) {
  const int64_t n = c.bytes / 8;
  const uint32_t rows = static_cast<uint32_t>(c.rows);
  const int64_t step = static_cast<int64_t>(g) * kBlock;
  double* run = GATHER ? static_cast<double*>(c.dst) : const_cast<double*>(static_cast<const double*>(c.src));
  for (int64_t t = static_cast<int64_t>(part) * kBlock + threadIdx.x; t < n; t += step) {
    const uint64_t e = static_cast<uint64_t>(c.first + t);
    const uint64_t col = e / rows, row = e - col * rows;
    double* f = c.block + row + col * static_cast<uint64_t>(c.ld);
    if constexpr (GATHER) run[t] = *f;
    else *f = run[t];
  }
}

// Every workgroup takes its slice of chunk 0, then of chunk 1, ...: the
// chunks complete in order, so the host sends chunk 0 after ~1/n of the
// launch.  (Round 4's grid of n x G workgroups, G per chunk, had every chunk
// in flight at once and raised all flags within ~5 us of each other at the
// end of the launch: the host-side trace of profiles/r05_xport/.)
__global__ __launch_bounds__(kBlock) void stage_copy_kernel(const gmt_stage_chunk* __restrict__ chunks, int n_chunks,
                                                            unsigned* __restrict__ counters,
                                                            uint64_t* __restrict__ flags, uint64_t value) {
  const int g = static_cast<int>(gridDim.x), part = static_cast<int>(blockIdx.x);
  for (int k = 0; k < n_chunks; ++k) {
    const gmt_stage_chunk c = chunks[k];
    const char* src = static_cast<const char*>(c.src);
    char* dst = static_cast<char*>(c.dst);
    const int64_t step = static_cast<int64_t>(g) * kBlock * 16;
    if (c.rows > 0) {
      strided_part<true>(c, part, g);
    } else if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
      const int64_t n16 = c.bytes / 16 * 16;
      int64_t o = (static_cast<int64_t>(part) * kBlock + threadIdx.x) * 16;
      // two 16-B loads in flight per lane per iteration
      for (; o + step < n16; o += 2 * step) {
        const d2 x = *reinterpret_cast<const d2*>(src + o);
        const d2 y = *reinterpret_cast<const d2*>(src + o + step);
        *reinterpret_cast<d2*>(dst + o) = x;
        *reinterpret_cast<d2*>(dst + o + step) = y;
      }
      if (o < n16) *reinterpret_cast<d2*>(dst + o) = *reinterpret_cast<const d2*>(src + o);
      if (part == 0)
        for (int64_t t = n16 + threadIdx.x; t < c.bytes; t += kBlock) dst[t] = src[t];
    } else {
      for (int64_t o = static_cast<int64_t>(part) * kBlock + threadIdx.x; o < c.bytes;
           o += static_cast<int64_t>(g) * kBlock)
        dst[o] = src[o];
    }
    // this workgroup's bytes of chunk k reach memory before its arrival is
    // counted; the chunk's last arrival publishes the flag (system-scope
    // release store)
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
      if (__hip_atomic_fetch_add(counters + k, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
          static_cast<unsigned>(g - 1)) {
        __hip_atomic_store(counters + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(flags + k, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// received chunks from page-locked host memory into the field (strided) or
// a device buffer: the GPU reads the host buffer over the link
__global__ __launch_bounds__(kBlock) void stage_scatter_kernel(const gmt_stage_chunk* __restrict__ chunks, int g) {
  const int k = blockIdx.x / g, part = blockIdx.x % g;
  const gmt_stage_chunk c = chunks[k];
  if (c.rows > 0) {
    strided_part<false>(c, part, g);
    return;
  }
  const char* src = static_cast<const char*>(c.src);
  char* dst = static_cast<char*>(c.dst);
  for (int64_t o = static_cast<int64_t>(part) * kBlock + threadIdx.x; o < c.bytes;
       o += static_cast<int64_t>(g) * kBlock)
    dst[o] = src[o];
}

}  // namespace stage
}  // namespace gmt

extern "C" int gmt_stage_copy(int n_chunks, const gmt_stage_chunk* chunks, unsigned* counters, uint64_t* flags,
                              uint64_t value, int wgs, void* stream) {
  using namespace gmt;
  if (n_chunks < 0 || wgs < 1 || (n_chunks > 0 && (!chunks || !counters || !flags)))
    return static_cast<int>(hipErrorInvalidValue);
  if (n_chunks == 0) return 0;
  stage::stage_copy_kernel<<<grid_1d(wgs), kBlock, 0, static_cast<hipStream_t>(stream)>>>(chunks, n_chunks, counters,
                                                                                         flags, value);
  GMT_RET_LAUNCH();
}

// the table is read by the kernel: a host (pinned) or device pointer
extern "C" int gmt_stage_scatter(int n_chunks, const gmt_stage_chunk* chunks, int wgs_per_chunk, void* stream) {
  using namespace gmt;
  if (n_chunks < 0 || wgs_per_chunk < 1 || (n_chunks > 0 && !chunks)) return static_cast<int>(hipErrorInvalidValue);
  if (n_chunks == 0) return 0;
  stage::stage_scatter_kernel<<<grid_1d(static_cast<int64_t>(n_chunks) * wgs_per_chunk), kBlock, 0,
                                static_cast<hipStream_t>(stream)>>>(chunks, wgs_per_chunk);
  GMT_RET_LAUNCH();
}
