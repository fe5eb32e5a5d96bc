// gmt/device.hpp — rank -> GPU binding, node counting, device identity.
//
// Reference: set_rank_device, copy-pasted five times (mpi_daxpy.cc:36-62,
// mpi_daxpy_nvtx.cc:43-69, mpi_daxpy_gt.cc:26-45, mpi_stencil_gt.cc:61-81,
// mpi_stencil2d_gt.cc:112-133) and get_node_count (mpi_daxpy_nvtx.cc:72-82).
//
// Same policy (block mapping when ranks oversubscribe GPUs, exact-multiple
// requirement, the RANK[..] => DEVICE[..] report line) but computed from the
// NODE-LOCAL rank and size (MPI_Comm_split_type SHARED): the reference uses
// the global rank against the per-node device count, which binds ranks of
// the second node to non-existent devices.
#pragma once

#include <mpi.h>

#include <cstdio>
#include <cstdlib>

#include "gmt/mpi.hpp"
#include "gmt/numa_bind.hpp"
#include "gmt/watchdog.hpp"

namespace gmt {

struct RankBinding {
  int rank = 0, world_size = 1;
  int local_rank = 0, local_size = 1;
  int device = 0, n_devices = 1, ranks_per_device = 1;
  size_t mem_per_rank = 0;
  int numa_node = -1;  // CPUs bound to this NUMA node (gmt_rt_bind_numa), -1 = unbound
  int pinned_cpu = -1;  // the core this rank is pinned to (gmt_rt_pin_rank), -1 = not pinned
  gmt_device_info info{};
};

inline void local_rank_size(MPI_Comm comm, int* lrank, int* lsize) {
  MPI_Comm shm;
  GMT_MPI_CHECK(MPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, 0, MPI_INFO_NULL, &shm));
  MPI_Comm_rank(shm, lrank);
  MPI_Comm_size(shm, lsize);
  MPI_Comm_free(&shm);
}

// reference get_node_count: ranks / ranks-per-shared-memory-domain
inline int get_node_count(MPI_Comm comm) {
  int n_ranks = 1, lrank = 0, lsize = 1;
  MPI_Comm_size(comm, &n_ranks);
  local_rank_size(comm, &lrank, &lsize);
  // a node with fewer ranks than the first would make this inexact; count
  // node leaders instead
  int leader = lrank == 0 ? 1 : 0, nodes = 0;
  MPI_Allreduce(&leader, &nodes, 1, MPI_INT, MPI_SUM, comm);
  (void)lsize;
  return nodes > 0 ? nodes : 1;
}

// The core this process pinned itself to before MPI_Init (-1: not pinned
// then).
inline int& early_pinned_cpu() {
  static int cpu = -1;
  return cpu;
}

// MPI_Init with the rank pinned first (gmt_rt_pin_rank from the launcher's
// local rank variables): MPI's shared-memory segments, touched during
// MPI_Init, then land next to the core the rank runs on.  Pinning after
// MPI_Init reliably gave the host-staged exchange's slow mode (7.3-7.6 GB/s
// per rank against 15.1-15.3 unpinned, profiles/r06_pin/).  Without the
// variables the rank is pinned by set_rank_device, after MPI_Init.
inline void mpi_init_pinned(int* argc, char*** argv) {
  int lr = 0, ls = 0, ndev = 0;
  if (launcher_local_rank(&lr, &ls) && gmt_rt_device_count(&ndev) == 0 && ndev > 0) {
    const int per = ls > ndev && ls % ndev == 0 ? ls / ndev : 1;
    (void)gmt_rt_pin_rank(lr, ls, per, &early_pinned_cpu());
  }
  GMT_MPI_CHECK(MPI_Init(argc, argv));
}

// Select and set this rank's device.  print: emit the reference's
// "RANK[r/N] => DEVICE[d/D] mem=%zd" line (mpi_daxpy.cc:58-59).
inline RankBinding set_rank_device(MPI_Comm comm, bool print) {
  install_mpi_abort();
  RankBinding b;
  MPI_Comm_rank(comm, &b.rank);
  MPI_Comm_size(comm, &b.world_size);
  local_rank_size(comm, &b.local_rank, &b.local_size);
  GMT_CHECK("get device count", gmt_rt_device_count(&b.n_devices));
  if (b.n_devices <= 0) {
    std::printf("ERROR: no devices visible to rank %d\n", b.rank);
    abort_job(EXIT_FAILURE);
  }
  if (b.local_size > b.n_devices) {
    if (b.local_size % b.n_devices != 0) {
      std::printf("ERROR: Number of ranks (%d) not a multiple of number of GPUs (%d)\n",
                  b.local_size, b.n_devices);
      abort_job(EXIT_FAILURE);
    }
    b.ranks_per_device = b.local_size / b.n_devices;
    b.device = b.local_rank / b.ranks_per_device;
  } else {
    b.ranks_per_device = 1;
    b.device = b.local_rank;
  }
  GMT_CHECK("get device props", gmt_rt_device_info(b.device, &b.info));
  b.mem_per_rank = b.info.total_mem / b.ranks_per_device;
  if (print)
    std::printf("RANK[%d/%d] => DEVICE[%d/%d] mem=%zd\n", b.rank + 1, b.world_size, b.device + 1,
                b.n_devices, b.mem_per_rank);
  GMT_CHECK("set device", gmt_rt_set_device(b.device));
  // the GPU's socket: before any transport allocates its staging buffers
  GMT_CHECK("numa bind", gmt_rt_bind_numa(b.device, &b.numa_node));
  // one core near the GPU per rank, distinct per local rank (GMT_PIN=0: off)
  if (early_pinned_cpu() >= 0)
    b.pinned_cpu = early_pinned_cpu();
  else
    GMT_CHECK("pin rank", gmt_rt_pin_rank(b.local_rank, b.local_size, b.ranks_per_device, &b.pinned_cpu));
  watchdog_start(b.rank, b.device);
  watchdog_kick("device bound");
  return b;
}

}  // namespace gmt
