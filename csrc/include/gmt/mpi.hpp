// gmt/mpi.hpp — MPI control-plane helpers for the native apps.
//
// Reference: the `check(file, line, rval)` helper repeated in
// mpi_stencil2d_gt.cc:32-40, mpi_stencil2d_sycl.cc:27-35 and
// mpi_stencil2d_sycl_oo.cc:268-276 (print + exit(2)).  Here a failure prints
// the MPI error string and aborts the whole job with MPI_Abort, and
// install_mpi_abort() routes every other failed check (GMT_CHECK, RCCL) to
// MPI_Abort too, so no rank is left waiting in a collective.
#pragma once

#include <mpi.h>
#include <unistd.h>

#include <cstdio>

#include "gmt/check.hpp"

namespace gmt {

inline void mpi_abort_hook(int code) {
  int init = 0, fin = 0;
  MPI_Initialized(&init);
  MPI_Finalized(&fin);
  if (init && !fin) {
    // give the launcher's stdout forwarding a moment: MPI_Abort tears the job
    // down at once and can drop the error message just printed
    usleep(300000);
    MPI_Abort(MPI_COMM_WORLD, code);
  }
}

inline void install_mpi_abort() { abort_hook() = &mpi_abort_hook; }

inline void check_mpi(const char* file, int line, int rval) {
  if (rval != MPI_SUCCESS) {
    char s[MPI_MAX_ERROR_STRING];
    int len = 0;
    MPI_Error_string(rval, s, &len);
    std::printf("%s:%d error %d (%s)\n", file, line, rval, s);
    install_mpi_abort();
    abort_job(2);
  }
}

}  // namespace gmt

#define GMT_MPI_CHECK(x) ::gmt::check_mpi(__FILE__, __LINE__, (x))
