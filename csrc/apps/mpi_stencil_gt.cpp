// mpi_stencil_gt — 1-D distributed derivative; a small-message (16 B)
// GPU-to-GPU halo-exchange latency probe.
//
// Reference: /root/reference/mpi_stencil_gt.cc:124-230.  CLI `[n_global_Mi]`
// (default 32 -> 32 Mi points, strong scaling: n_local = n_global/world_size),
// y = x^3 on [0, 8), 2 ghost cells per side, ONE timed exchange of 2 doubles
// per neighbour, then dy/dx and the error norm against 3x^2.
// Output: "%d/%d exchange time %0.8f" (seconds) and
// "%d/%d [%d:0x%08x] err_norm = %.8f" on every rank.
//
// The halo cells are contiguous, so they go zero-copy through the selected
// transport (RCCL send/recv, IPC peer write, or MPI).  Added: --iters=K runs
// K more timed exchanges and reports min/median latency (the BASELINE
// "halo-exchange latency" metric), --transport=..., --json=FILE.
#include <mpi.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gmt/buffer.hpp"
#include "gmt/device.hpp"
#include "gmt/comm.hpp"
#include "gmt/halo.hpp"
#include "gmt/util.hpp"

using namespace gmt;

int main(int argc, char** argv) {
  Cli cli(argc, argv);
  long long n_global = 32LL * 1024 * 1024;
  if (cli.positional(0)) n_global = std::atoll(cli.positional(0)) * 1024 * 1024;
  if (cli.has("n")) n_global = cli.geti("n", n_global);
  const int iters = static_cast<int>(cli.geti("iters", 0));
  const int n_bnd = 2;

  mpi_init_pinned(&argc, &argv);  // pinned near the GPU first (gmt/device.hpp)
  int world_size = 1, world_rank = 0;
  MPI_Comm_size(MPI_COMM_WORLD, &world_size);
  MPI_Comm_rank(MPI_COMM_WORLD, &world_rank);
  if (n_global % world_size != 0) {
    std::printf("%d nmpi (%d) must be divisor of domain size (%lld), exiting\n", world_rank,
                world_size, n_global);
    // every rank sees the same condition: leave collectively (an MPI_Abort
    // can kill the job before the forwarded message reaches the terminal)
    std::fflush(stdout);
    MPI_Finalize();
    return 1;
  }
  const size_t n_local = static_cast<size_t>(n_global / world_size);
  const size_t n_ghost = n_local + 2 * n_bnd;
  RankBinding b = set_rank_device(MPI_COMM_WORLD, false);
  if (world_rank == 0) {
    std::printf("n procs  = %d\n", world_size);
    std::printf("n_global = %lld\n", n_global);
    std::printf("n_local  = %zu\n", n_local);
  }
  std::fflush(stdout);
  auto tr = comm::make_transport(comm::parse_kind(cli.get("transport", "auto")), MPI_COMM_WORLD, b);
  double seconds = 0.0, err_norm = 0.0;
  Stats lat;
  {
    Buffer<double> d_y(n_ghost, GMT_SPACE_DEVICE), d_dydx(n_local, GMT_SPACE_DEVICE);
    const double lx = 8.0, dx = lx / n_global, scale = n_global / lx;
    const double x_start = world_rank * (lx / world_size);
    gmt_stream_t s = nullptr;
    GMT_CHECK("stream", gmt_rt_stream_create(&s, 0));
    GMT_CHECK("memset", gmt_rt_memset_async(d_y.data(), 0, d_y.bytes(), s));
    // y = x^3 (fill mode 0 at y = 0) incl. the physical-boundary ghosts
    GMT_CHECK("fill", gmt_fill_poly(0, n_local, 1, x_start, dx, 0.0, 0.0, d_y.data() + n_bnd, n_local, s));
    if (world_rank == 0)
      GMT_CHECK("fill lo", gmt_fill_poly(0, n_bnd, 1, -n_bnd * dx, dx, 0.0, 0.0, d_y.data(), n_bnd, s));
    if (world_rank == world_size - 1)
      GMT_CHECK("fill hi", gmt_fill_poly(0, n_bnd, 1, lx, dx, 0.0, 0.0, d_y.data() + n_bnd + n_local,
                                         n_bnd, s));
    GMT_CHECK("sync", gmt_rt_stream_synchronize(s));
    // a 1-D array is a 1 x n_ghost column-major field: the halo is "dim 1",
    // contiguous, sent in place
    Neighbors nb;
    nb.south = world_rank > 0 ? world_rank - 1 : -1;
    nb.north = world_rank < world_size - 1 ? world_rank + 1 : -1;
    Halo2D halo(*tr, Span2D<double>(d_y.data(), 1, n_ghost), 0, n_bnd, nb, false, GMT_SPACE_DEVICE);
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = wtime();
    halo.exchange(s);
    seconds = wtime() - t0;
    std::printf("%d/%d exchange time %0.8f\n", world_rank, world_size, seconds);
    for (int k = 0; k < iters; ++k) {
      MPI_Barrier(MPI_COMM_WORLD);
      const double t1 = wtime();
      halo.exchange(s);
      lat.add(wtime() - t1);
    }
    const double c[5] = {1.0 / 12.0, -2.0 / 3.0, 0.0, 2.0 / 3.0, -1.0 / 12.0};
    GMT_CHECK("stencil", gmt_stencil5_1d(n_local, c, scale, d_y.data(), d_dydx.data(), s));
    std::vector<double> h(n_local);
    GMT_CHECK("sync", gmt_rt_stream_synchronize(s));
    GMT_CHECK("h = d_dydx", gmt_rt_memcpy(h.data(), d_dydx.data(), d_dydx.bytes()));
    double acc = 0.0;
    for (size_t i = 0; i < n_local; ++i) {
      const double x = x_start + i * dx;
      const double d = h[i] - 3 * x * x;
      acc += d * d;
    }
    err_norm = std::sqrt(acc);
    gmt_rt_stream_destroy(s);
  }
  std::printf("%d/%d [%d:0x%08x] err_norm = %.8f\n", world_rank, world_size, b.device,
              b.info.vendor_id, err_norm);
  if (iters > 0) {
    double med = lat.median(), mn = lat.min(), med_max = 0, mn_max = 0;
    MPI_Reduce(&med, &med_max, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    MPI_Reduce(&mn, &mn_max, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    if (world_rank == 0) {
      std::printf("# 16-byte halo exchange transport=%s: median %.2f us, min %.2f us (max over ranks, %d iters)\n",
                  tr->name(), med_max * 1e6, mn_max * 1e6, iters);
      JsonRecord j;
      j.add("app", "mpi_stencil_gt").add("ranks", world_size).add("transport", tr->name())
          .add("n_global", n_global).add("latency_us_median", med_max * 1e6)
          .add("latency_us_min", mn_max * 1e6).add("iters", iters);
      j.append_to(cli.get("json", ""));
    }
  }
  tr.reset();
  MPI_Finalize();
  return EXIT_SUCCESS;
}
