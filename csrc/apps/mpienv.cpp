// mpienv — host-only probe of MEMORY_PER_CORE on every rank.
//
// Reference: /root/reference/mpienv.f90:1-35 (Fortran).  The local mpif90
// wrapper points at a missing gfortran, so this is C++ with
// the same semantics: read at most 5 characters of the variable, parse them
// as the Fortran `(i6)` edit does (blanks -> 0), print
// " rank <r:12> MEMORY_PER_CORE=<v:12>" in gfortran list-directed layout.
#include <mpi.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>

int main(int argc, char** argv) {
  int ierr = MPI_Init(&argc, &argv);
  if (ierr != 0) {
    std::printf(" Failed MPI_Init: %12d\n", ierr);
    return 0;
  }
  int rank = 0, nmpi = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &nmpi);
  char read_env[6] = "     ";
  if (const char* e = std::getenv("MEMORY_PER_CORE")) {
    const size_t l = std::strlen(e);
    std::memcpy(read_env, e, l < 5 ? l : 5);
  }
  long v = 0;
  bool neg = false;
  for (int i = 0; i < 5; ++i) {
    const char c = read_env[i];
    if (c == '-') neg = true;
    else if (std::isdigit(static_cast<unsigned char>(c))) v = v * 10 + (c - '0');
  }
  const int memory_per_core = static_cast<int>(neg ? -v : v);
  std::printf(" rank %12d  MEMORY_PER_CORE=%12d\n", rank, memory_per_core);
  MPI_Finalize();
  return 0;
}
