// mpigatherinplace — host in-place MPI_Allgather of 1 GiB per rank.
//
// Reference: /root/reference/mpigatherinplace.f90:1-58 (Fortran, host only).
// allx(rank*N + i) = rank*i/N with INTEGER division (i = 1..N), the local
// and global sums accumulated in single precision (`real :: asum, lsum`),
// MPI_Allgather(MPI_IN_PLACE, ...) of N = 128 Mi doubles per rank.
// Fixed here: the Fortran default-integer products rank*i and N*nmpi
// overflow from 16 ranks on; they are 64-bit.
//
// Added: --n=N (elements per rank), --device (the same all-gather on device
// buffers through a gmt transport: RCCL over xGMI / IPC / staged MPI;
// --transport=...), --json=FILE with the gather time and GB/s.
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gmt/buffer.hpp"
#include "gmt/comm.hpp"
#include "gmt/device.hpp"
#include "gmt/util.hpp"

using namespace gmt;

int main(int argc, char** argv) {
  Cli cli(argc, argv);
  const long long N = cli.geti("n", 128LL * 1024 * 1024);
  const bool on_device = cli.flag("device");
  if (MPI_Init(&argc, &argv) != MPI_SUCCESS) {
    std::printf(" Failed MPI_Init\n");
    return 0;
  }
  int rank = 0, nmpi = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &nmpi);
  const size_t total = static_cast<size_t>(N) * nmpi;
  float lsum = 0.0f, asum = 0.0f;
  double t_gather = 0.0;
  std::string transport = "mpi-host-memory";
  {
    std::vector<double> allx(total, 0.0);
    for (long long i = 1; i <= N; ++i) {
      const double v = static_cast<double>((static_cast<long long>(rank) * i) / N);
      allx[static_cast<size_t>(rank) * N + (i - 1)] = v;
      lsum = lsum + static_cast<float>(v);
    }
    if (!on_device) {
      MPI_Barrier(MPI_COMM_WORLD);
      const double t0 = MPI_Wtime();
      int ierr = MPI_Allgather(MPI_IN_PLACE, 0, MPI_DOUBLE, allx.data(), static_cast<int>(N),
                               MPI_DOUBLE, MPI_COMM_WORLD);
      t_gather = MPI_Wtime() - t0;
      if (ierr != 0) {
        std::printf(" Failed MPI_Allgather: %12d\n", ierr);
        MPI_Abort(MPI_COMM_WORLD, 1);
      }
    } else {
      RankBinding b = set_rank_device(MPI_COMM_WORLD, false);
      auto tr = comm::make_transport(comm::parse_kind(cli.get("transport", "auto")), MPI_COMM_WORLD, b);
      transport = tr->name();
      Buffer<double> d(total, GMT_SPACE_DEVICE);
      const size_t bytes = static_cast<size_t>(N) * sizeof(double);
      GMT_CHECK("H2D", gmt_rt_memcpy(d.data() + static_cast<size_t>(rank) * N,
                                     allx.data() + static_cast<size_t>(rank) * N, bytes));
      MPI_Barrier(MPI_COMM_WORLD);
      const double t0 = MPI_Wtime();
      tr->allgather(d.data() + static_cast<size_t>(rank) * N, d.data(), bytes, nullptr);
      GMT_CHECK("sync", gmt_rt_device_synchronize());
      t_gather = MPI_Wtime() - t0;
      GMT_CHECK("D2H", gmt_rt_memcpy(allx.data(), d.data(), d.bytes()));
    }
    double s = 0.0;  // Fortran sum() of a real(8) array, then stored into a real
    for (double v : allx) s += v;
    asum = static_cast<float>(s);
  }
  std::printf("%12d /%12d  %15.8g  %15.8g\n", rank, nmpi, lsum, asum);
  double tmax = 0.0;
  MPI_Reduce(&t_gather, &tmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
  if (rank == 0) {
    const double gb = static_cast<double>(total) * sizeof(double) / 1e9;
    std::printf("# allgather %s: %.6f s, %.2f GB/s (gathered bytes per rank / time)\n",
                transport.c_str(), tmax, tmax > 0 ? gb / tmax : 0.0);
    JsonRecord j;
    j.add("app", "mpigatherinplace").add("ranks", nmpi).add("n_per_rank", static_cast<long long>(N))
        .add("transport", transport).add("time_s", tmax).add("GBps", tmax > 0 ? gb / tmax : 0.0);
    j.append_to(cli.get("json", ""));
  }
  MPI_Finalize();
  return 0;
}
