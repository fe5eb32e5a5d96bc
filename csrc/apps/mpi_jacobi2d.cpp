// mpi_jacobi2d — distributed 2-D 5-point Jacobi (fp64) with halo/interior
// overlap: the BASELINE stencil-MLUPS benchmark as a native MPI app.
//
// BASELINE.json configs "mpi_stencil2d 8192² fp64 single GPU" and
// "mpi_stencil2d 32768² on 8 GPUs (2×4 decomp), halo exchange/interior
// overlap".  The reference never overlaps and never reports a lattice-update
// rate; the loop it times is mpi_stencil2d_gt.cc:511-535.
//
// CLI: mpi_jacobi2d [n] [n_iter]       global n x n interior (default 8192, 100)
//   --nx=, --ny=            rectangular global domain
//   --weak                  n x n PER RANK (global = py*n x px*n)
//   --dims=PYxPX            process grid (default: minimise halo bytes)
//   --transport=auto|rccl|ipc|mpi-host|mpi-direct
//   --overlap=auto          time overlapped and serial passes once, keep the faster
//   --no-overlap --graph --periodic[=x|y] --warmup=W
//   --tblock                temporal blocking (gmt_jacobi5tb): K sweeps per memory pass
//                           and per (K-wide) halo exchange
//   --tsteps=K              sweeps per fused pass with --tblock (2-20; default 2; odd
//                           counts above 10 round down)
//   --wg-strips=N --seg-rows=L   gmt_tb_opts launch shape (0 = default)
//   --halo-iters=K          K blocking halo exchanges -> latency line
//   --push                  inline halo exchange of the fused passes (JacobiConfig::push: the
//                           pass stores its faces into the neighbours' ghost cells; ipc or
//                           a single rank)
//   --check                 rank 0 re-runs the whole problem serially on the host
//   --json=FILE
#include <mpi.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gmt/comm.hpp"
#include "gmt/device.hpp"
#include "gmt/jacobi.hpp"
#include "gmt/util.hpp"

using namespace gmt;

// Serial host reference of the same problem (init, boundary, update order).
static std::vector<double> serial_jacobi(int64_t ny, int64_t nx, int steps, bool periodic, int axes = 3) {
  const int64_t ld = nx + 2;
  const double h = 1.0 / (static_cast<double>(ny > nx ? ny : nx) + 1);
  std::vector<double> u((ny + 2) * ld), un;
  for (int64_t j = 0; j < ny + 2; ++j)
    for (int64_t i = 0; i < nx + 2; ++i) {
      const double x = (i - 1) * h, y = (j - 1) * h;
      u[j * ld + i] = x * x * x + y * y;
    }
  un = u;
  for (int s = 0; s < steps; ++s) {
    if (periodic && (axes & 1))
      for (int64_t j = 1; j <= ny; ++j) {
        u[j * ld] = u[j * ld + nx];
        u[j * ld + nx + 1] = u[j * ld + 1];
      }
    if (periodic && (axes & 2))
      for (int64_t i = 1; i <= nx; ++i) {
        u[i] = u[ny * ld + i];
        u[(ny + 1) * ld + i] = u[ld + i];
      }
    for (int64_t j = 1; j <= ny; ++j)
      for (int64_t i = 1; i <= nx; ++i) {
        const double* p = &u[j * ld + i];
        un[j * ld + i] = 0.25 * ((p[-1] + p[1]) + (p[-ld] + p[ld]));
      }
    std::swap(u, un);
  }
  std::vector<double> out(ny * nx);
  for (int64_t j = 0; j < ny; ++j)
    for (int64_t i = 0; i < nx; ++i) out[j * nx + i] = u[(j + 1) * ld + i + 1];
  return out;
}

int main(int argc, char** argv) {
  Cli cli(argc, argv);
  int64_t n = cli.positional(0) ? std::atoll(cli.positional(0)) : 8192;
  const int n_iter = cli.positional(1) ? std::atoi(cli.positional(1)) : 100;
  const int n_warmup = static_cast<int>(cli.geti("warmup", 10));
  mpi_init_pinned(&argc, &argv);  // pinned near the GPU first (gmt/device.hpp)
  int world = 1, rank = 0;
  MPI_Comm_size(MPI_COMM_WORLD, &world);
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  RankBinding b = set_rank_device(MPI_COMM_WORLD, false);

  JacobiConfig c;
  c.ny_global = cli.geti("ny", n);
  c.nx_global = cli.geti("nx", n);
  const std::string dims = cli.get("dims", "");
  if (!dims.empty()) {
    if (std::sscanf(dims.c_str(), "%dx%d", &c.py, &c.px) != 2 || c.py * c.px != world) {
      if (rank == 0) std::printf("ERROR: --dims=%s does not match %d ranks\n", dims.c_str(), world);
      MPI_Abort(MPI_COMM_WORLD, 1);
    }
  } else {
    choose_dims(world, c.ny_global, c.nx_global, &c.py, &c.px);
  }
  if (cli.flag("weak")) {
    c.ny_global *= c.py;
    c.nx_global *= c.px;
  }
  // --periodic wraps both axes, --periodic=x / =y one of them
  c.periodic = cli.has("periodic") && cli.get("periodic", "1") != "0";
  {
    const std::string pa = cli.get("periodic", "1");
    c.periodic_axes = pa == "x" ? 1 : (pa == "y" ? 2 : 3);
  }
  c.overlap = !cli.flag("no-overlap");
  c.overlap_auto = cli.get("overlap", "") == "auto";  // --overlap=auto: time both, keep the faster
  c.graph = cli.flag("graph");
  c.tblock = cli.has("tblock") && cli.get("tblock", "1") != "0";
  if (c.tblock) c.tsteps = static_cast<int>(cli.geti("tsteps", 2));
  c.wg_waves = static_cast<int>(cli.geti("wg-strips", 0));
  c.seg_rows = static_cast<int>(cli.geti("seg-rows", 0));
  c.push = cli.flag("push");
  // with one rank and no periodic wrap there is nothing to exchange; with a
  // periodic wrap a single rank exchanges with itself
  comm::Kind kind = comm::parse_kind(cli.get("transport", "auto"));
  if (kind == comm::Kind::Auto && world == 1) kind = comm::Kind::Local;
  auto tr = comm::make_transport(comm::resolve(kind, b), MPI_COMM_WORLD, b);

  double t_step = 0, resid = 0, halo_us = 0, max_diff = -1;
  bool graph = false, overlap = false, band = false, push = false;
  size_t hbytes = 0, hmsgs = 0;
  int64_t lnx = 0, lny = 0;
  {
    JacobiSolver solver(*tr, c);
    graph = solver.graph_active();
    overlap = solver.overlap_active();
    band = solver.band_first();
    push = solver.push_active();
    hbytes = solver.bytes_per_exchange();
    hmsgs = solver.messages();
    lnx = solver.nx();
    lny = solver.ny();
    solver.run(n_warmup);
    solver.synchronize();
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = wtime();
    solver.run(n_iter);
    solver.synchronize();
    double dt = wtime() - t0;
    MPI_Allreduce(MPI_IN_PLACE, &dt, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    t_step = dt / (n_iter > 0 ? n_iter : 1);

    if (cli.flag("check")) {
      std::vector<double> loc(static_cast<size_t>(lnx * lny));
      solver.copy_interior(loc.data());
      // gather every rank's block on rank 0 and compare with the serial run
      long long meta[4] = {solver.off_y(), solver.off_x(), lny, lnx};
      std::vector<long long> all(4 * world);
      MPI_Gather(meta, 4, MPI_LONG_LONG, all.data(), 4, MPI_LONG_LONG, 0, MPI_COMM_WORLD);
      std::vector<int> counts(world), displs(world);
      for (int r = 0; r < world; ++r) counts[r] = static_cast<int>(all[4 * r + 2] * all[4 * r + 3]);
      for (int r = 1; r < world; ++r) displs[r] = displs[r - 1] + counts[r - 1];
      std::vector<double> g(rank == 0 ? static_cast<size_t>(c.ny_global * c.nx_global) : 1);
      MPI_Gatherv(loc.data(), static_cast<int>(loc.size()), MPI_DOUBLE, g.data(), counts.data(),
                  displs.data(), MPI_DOUBLE, 0, MPI_COMM_WORLD);
      if (rank == 0) {
        std::vector<double> ref = serial_jacobi(c.ny_global, c.nx_global, n_warmup + n_iter, c.periodic, c.periodic_axes);
        max_diff = 0;
        for (int r = 0; r < world; ++r) {
          const long long oy = all[4 * r], ox = all[4 * r + 1], ny = all[4 * r + 2], nx = all[4 * r + 3];
          const double* blk = g.data() + displs[r];
          for (long long j = 0; j < ny; ++j)
            for (long long i = 0; i < nx; ++i)
              max_diff = std::fmax(max_diff, std::fabs(blk[j * nx + i] -
                                                       ref[(oy + j) * c.nx_global + ox + i]));
        }
      }
    }
    const int halo_iters = static_cast<int>(cli.geti("halo-iters", 0));
    if (halo_iters > 0 && hmsgs > 0) {
      Stats st;
      for (int k = 0; k < halo_iters + 3; ++k) {
        MPI_Barrier(MPI_COMM_WORLD);
        const double h0 = wtime();
        solver.exchange_only();
        if (k >= 3) st.add(wtime() - h0);
      }
      double med = st.median();
      MPI_Allreduce(&med, &halo_us, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
      halo_us *= 1e6;
    }
    resid = solver.residual();
  }
  if (rank == 0) {
    const double pts = static_cast<double>(c.ny_global) * c.nx_global;
    const double mlups = pts / t_step / 1e6;
    std::printf("n procs   = %d\n", world);
    std::printf("grid      = %dx%d (py x px)\n", c.py, c.px);
    std::printf("global    = %lld x %lld\n", (long long)c.ny_global, (long long)c.nx_global);
    std::printf("local     = %lld x %lld (rank 0)\n", (long long)lny, (long long)lnx);
    std::printf("transport = %s overlap=%d%s graph=%d periodic=%d tblock=%d backend=%s\n", tr->name(),
                overlap, band ? " (band-first)" : (push ? " (inline halo)" : ""), graph, c.periodic, c.tblock,
                gmt_rt_backend_name());
    std::printf("steps     = %d (warmup %d)\n", n_iter, n_warmup);
    std::printf("TIME step : %0.6f ms\n", t_step * 1e3);
    std::printf("MLUPS     : %0.1f (per GPU %0.1f, %0.1f GB/s per GPU at 16 B/pt)\n", mlups,
                mlups / world, 16.0 * pts / world / t_step / 1e9);
    if (halo_us > 0)
      std::printf("halo      : %0.2f us per exchange (%zu B, %zu msgs per rank)\n", halo_us, hbytes, hmsgs);
    std::printf("residual  : %.10e\n", resid);
    if (max_diff >= 0)
      std::printf("check     : max|diff| vs serial = %.3e %s\n", max_diff, max_diff < 1e-10 ? "OK" : "FAIL");
    JsonRecord j;
    j.add("app", "mpi_jacobi2d").add("ranks", world).add("py", c.py).add("px", c.px)
        .add("ny", (long long)c.ny_global).add("nx", (long long)c.nx_global).add("transport", tr->name())
        .add("overlap", overlap).add("band_first", band).add("push", push).add("graph", graph).add("tblock", c.tblock).add("steps", n_iter).add("ms_per_step", t_step * 1e3)
        .add("MLUPS", mlups).add("halo_us", halo_us).add("halo_bytes", hbytes).add("residual", resid)
        .add("check_max_diff", max_diff);
    j.append_to(cli.get("json", ""));
  }
  tr.reset();
  MPI_Finalize();
  return max_diff >= 1e-10 ? 3 : EXIT_SUCCESS;
}
