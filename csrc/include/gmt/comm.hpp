// gmt/comm.hpp — MPI-bootstrapped transport factory for the native apps.
//
// MPI is the control plane (rank/size, RCCL unique-id broadcast, IPC handle
// exchange, ready/done tokens); the data plane is picked per gmt/transport.hpp.
#pragma once

#include <mpi.h>

#include <memory>
#include <string>

#include "gmt/device.hpp"
#include "gmt/transport.hpp"

namespace gmt {
namespace comm {

Kind parse_kind(const std::string& s);
// GPU-aware MPI: GMT_MPI_GPU_AWARE=1/0 overrides, else MPIX_Query_rocm_support
// when the MPI library has it; MPICH 3.3 ch3 here has neither (not GPU-aware).
// mpi-direct refuses device buffers unless this is true.
bool mpi_gpu_aware();
const char* mpi_gpu_aware_source();  // how mpi_gpu_aware() decided (for logs)
// Resolve Auto for a device-resident exchange: rccl if one rank per GPU and
// RCCL exists, else ipc; mpi-direct on the host backend, for managed
// buffers or with a GPU-aware MPI.  GMT_TRANSPORT=<kind> overrides Auto.
Kind resolve(Kind k, const RankBinding& b, bool buffers_managed = false);
std::unique_ptr<Transport> make_transport(Kind k, MPI_Comm comm, const RankBinding& b);

}  // namespace comm
}  // namespace gmt
