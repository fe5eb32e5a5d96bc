// mpi_daxpy — MPI + managed-memory DAXPY plumbing probe.
//
// Reference: /root/reference/mpi_daxpy.cc:65-169.  Every rank binds a GPU
// (RANK[..] => DEVICE[..] line), allocates device and MANAGED x/y, prints
// their managed preferred locations (MEMINFO), runs DAXPY on the managed
// arrays and sums the result on the host straight out of managed memory:
// "%d/%d SUM = %f" = 524800.000000 at n = 1024.
//
// On MI355X the managed mode depends on XNACK (page migration); the header
// line reports it.
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
  GMT_MPI_CHECK(MPI_Init(&argc, &argv));
  int world_size = 1, world_rank = 0;
  MPI_Comm_size(MPI_COMM_WORLD, &world_size);
  MPI_Comm_rank(MPI_COMM_WORLD, &world_rank);

  std::vector<double> x(n), y(n);
  for (size_t i = 0; i < n; ++i) {
    x[i] = static_cast<double>(i + 1);
    y[i] = -static_cast<double>(i + 1);
  }
  if (world_rank == 0) {
    const char* mb = std::getenv("MEMORY_PER_CORE");
    if (mb == nullptr)
      std::printf("MEMORY_PER_CORE is not set\n");
    else
      std::printf("MEMORY_PER_CORE=%s\n", mb);
  }
  RankBinding b = set_rank_device(MPI_COMM_WORLD, true);
  {
    Buffer<double> d_x(n, GMT_SPACE_DEVICE), d_y(n, GMT_SPACE_DEVICE);
    Buffer<double> m_x(n, GMT_SPACE_MANAGED), m_y(n, GMT_SPACE_MANAGED);
    GMT_CHECK("d_x = x", gmt_rt_memcpy(d_x.data(), x.data(), n * sizeof(double)));
    GMT_CHECK("d_y = y", gmt_rt_memcpy(d_y.data(), y.data(), n * sizeof(double)));
    GMT_CHECK("m_x = x", gmt_rt_memcpy(m_x.data(), x.data(), n * sizeof(double)));
    GMT_CHECK("m_y = y", gmt_rt_memcpy(m_y.data(), y.data(), n * sizeof(double)));
    GMT_MEMINFO("d_x", d_x.data(), d_x.bytes());
    GMT_MEMINFO("d_y", d_y.data(), d_y.bytes());
    GMT_MEMINFO("m_x", m_x.data(), m_x.bytes());
    GMT_MEMINFO("m_y", m_y.data(), m_y.bytes());
    GMT_MEMINFO("x", x.data(), n * sizeof(double));
    GMT_MEMINFO("y", y.data(), n * sizeof(double));
    if (cli.flag("rocblas"))
      GMT_CHECK("daxpy", gmt_blas_daxpy(n, a, m_x.data(), m_y.data(), nullptr));
    else
      GMT_CHECK("daxpy", gmt_daxpy(n, a, m_x.data(), m_y.data(), nullptr));
    GMT_CHECK("daxpy sync", gmt_rt_device_synchronize());
    GMT_CHECK("y = d_y sync", gmt_rt_device_synchronize());
    double sum = 0.0;
    for (size_t i = 0; i < n; ++i) sum += m_y[i];  // host read of managed memory
    std::printf("%d/%d SUM = %f\n", world_rank, world_size, sum);
    if (world_rank == 0)
      std::printf("# backend=%s device=%s managed_memory=%d concurrent_managed_access=%d xnack=%d\n",
                  gmt_rt_backend_name(), b.info.name, b.info.managed_memory,
                  b.info.concurrent_managed_access, b.info.xnack);
  }
  MPI_Finalize();
  return EXIT_SUCCESS;
}
