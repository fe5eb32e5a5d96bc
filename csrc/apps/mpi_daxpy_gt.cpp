// mpi_daxpy_gt — per-rank DAXPY through the portable kernel layer.
//
// Reference: /root/reference/mpi_daxpy_gt.cc:48-97 (gtensor containers +
// gt::blas::axpy on any gtensor backend, including `host`).  Here the same
// source runs on the gfx950 kernels (build/bin) or the CPU backend
// (build/bin-host).  Output: "%d/%d [%d:0x%08x] SUM = %f" (device id, PCI
// vendor id: 0x00001002 on AMD, 0 on the host backend), SUM = 524800 at n = 1024.
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gmt/buffer.hpp"
#include "gmt/device.hpp"
#include "gmt/util.hpp"

using namespace gmt;

int main(int argc, char** argv) {
  Cli cli(argc, argv);
  const size_t n = static_cast<size_t>(cli.geti("n", 1024));
  const double a = 2.0;
  mpi_init_pinned(&argc, &argv);  // pinned near the GPU first (gmt/device.hpp)
  int world_size = 1, world_rank = 0;
  MPI_Comm_size(MPI_COMM_WORLD, &world_size);
  MPI_Comm_rank(MPI_COMM_WORLD, &world_rank);
  RankBinding b = set_rank_device(MPI_COMM_WORLD, false);
  {
    std::vector<double> x(n), y(n);
    Buffer<double> d_x(n, GMT_SPACE_DEVICE), d_y(n, GMT_SPACE_DEVICE);
    for (size_t i = 0; i < n; ++i) {
      x[i] = static_cast<double>(i + 1);
      y[i] = -static_cast<double>(i + 1);
    }
    GMT_CHECK("d_x = x", gmt_rt_memcpy(d_x.data(), x.data(), n * sizeof(double)));
    GMT_CHECK("d_y = y", gmt_rt_memcpy(d_y.data(), y.data(), n * sizeof(double)));
    GMT_CHECK("axpy", gmt_daxpy(n, a, d_x.data(), d_y.data(), nullptr));
    GMT_CHECK("sync", gmt_rt_device_synchronize());
    GMT_CHECK("y = d_y", gmt_rt_memcpy(y.data(), d_y.data(), n * sizeof(double)));
    double sum = 0.0;
    for (size_t i = 0; i < n; ++i) sum += y[i];
    std::printf("%d/%d [%d:0x%08x] SUM = %f\n", world_rank, world_size, b.device,
                b.info.vendor_id, sum);
  }
  MPI_Finalize();
  return EXIT_SUCCESS;
}
