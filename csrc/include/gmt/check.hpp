// gmt/check.hpp — fail-fast error checking and pointer introspection.
//
// Reference: /root/reference/cuda_error.h — CHECK/WARN (:16-41, cuBLAS
// overload :45-63), PTRINFO (:66-96), MEMINFO (:99-135); the MPI `check`
// helper repeated in mpi_stencil2d_gt.cc:32-40, mpi_stencil2d_sycl.cc:27-35,
// mpi_stencil2d_sycl_oo.cc:268-276.
//
// Differences, deliberately: a failed check aborts the WHOLE
// job with MPI_Abort (the reference's exit() strands the other ranks), and
// the checks are always on unless GMT_NO_CHECK_CALLS is defined (the
// reference's header comment promises a GPU_CHECK_CALLS switch that does
// nothing, cuda_error.h:7-8 vs :16).
#pragma once

#include <cstdio>
#include <cstdlib>

#include "gmt/ccl.h"
#include "gmt/kernels.h"
#include "gmt/rt.h"

namespace gmt {

// Job-wide abort.  MPI programs install an MPI_Abort hook (gmt/mpi.hpp) so a
// failed check takes every rank down; the MPI-free engine library used from
// Python exits the process (the launcher tears the job down).
using AbortHook = void (*)(int);
inline AbortHook& abort_hook() {
  static AbortHook h = nullptr;
  return h;
}
[[noreturn]] inline void abort_job(int code) {
  std::fflush(stdout);
  std::fflush(stderr);
  if (abort_hook()) abort_hook()(code);
  std::exit(code);
}

inline int check_rt(const char* msg, int val, const char* file, int line, bool abort) {
  if (val != 0) {
    std::fprintf(stderr, "%s(%i): HIP Error (%s) %i: %s\n", file, line, msg, val,
                 gmt_rt_error_string(val));
    if (abort) {
      gmt_rt_device_reset();
      abort_job(EXIT_FAILURE);
    }
  }
  return val;
}

inline int check_ccl(const char* msg, int val, const char* file, int line) {
  if (val != 0) {
    std::fprintf(stderr, "%s(%i): RCCL Error (%s) %i: %s\n", file, line, msg, val,
                 gmt_ccl_error_string(val));
    abort_job(EXIT_FAILURE);
  }
  return val;
}

inline const char* space_name(int space) {
  switch (space) {
    case GMT_SPACE_DEVICE: return "Device";
    case GMT_SPACE_MANAGED: return "Managed";
    case GMT_SPACE_PINNED:
    case GMT_SPACE_PINNED_COHERENT: return "Host";
    default: return "Unregistered";
  }
}

// PTRINFO: "HIP pointer <label> (<addr>): Device|Managed|Host|Unregistered"
inline void print_ptr_info(const char* label, const void* ptr) {
  if (ptr == nullptr) {
    std::printf("HIP pointer %s (%zx): NULL\n", label, reinterpret_cast<size_t>(ptr));
    return;
  }
  int space = GMT_SPACE_UNREGISTERED;
  gmt_rt_pointer_space(ptr, &space);
  std::printf("HIP pointer %s (%zx): %s\n", label, reinterpret_cast<size_t>(ptr),
              space_name(space));
}

// MEMINFO: managed-memory preferred location of [ptr, ptr+size).
// Unlike the reference call sites (which pass sizeof(pointer)),
// callers here pass the real byte count.
inline void print_mem_info(const char* label, const void* ptr, size_t size) {
  int space = GMT_SPACE_UNREGISTERED;
  gmt_rt_pointer_space(ptr, &space);
  if (space == GMT_SPACE_UNREGISTERED) {
    std::printf("HIP PreferredLocation of '%s' is NOT HIP\n", label);
    return;
  }
  if (space != GMT_SPACE_MANAGED) {
    std::printf("HIP PreferredLocation of '%s' is UNMANAGED\n", label);
    return;
  }
  int loc = -123;
  gmt_rt_mem_preferred_location(ptr, size, &loc);
  if (loc == -1)
    std::printf("HIP PreferredLocation of '%s' is CPU (%d)\n", label, loc);
  else if (loc < -1)
    std::printf("HIP PreferredLocation of '%s' is INVALID (%d)\n", label, loc);
  else
    std::printf("HIP PreferredLocation of '%s' is DEVICE (%d)\n", label, loc);
}

}  // namespace gmt

#ifndef GMT_NO_CHECK_CALLS
#define GMT_CHECK(msg, val) ::gmt::check_rt((msg), (val), __FILE__, __LINE__, true)
#define GMT_WARN(msg, val) ::gmt::check_rt((msg), (val), __FILE__, __LINE__, false)
#define GMT_CCL_CHECK(msg, val) ::gmt::check_ccl((msg), (val), __FILE__, __LINE__)
#else
#define GMT_CHECK(msg, val) ((void)(val))
#define GMT_WARN(msg, val) ((void)(val))
#define GMT_CCL_CHECK(msg, val) ((void)(val))
#endif
#define GMT_PTRINFO(label, ptr) ::gmt::print_ptr_info((label), (ptr))
#define GMT_MEMINFO(label, ptr, size) ::gmt::print_mem_info((label), (ptr), (size))
