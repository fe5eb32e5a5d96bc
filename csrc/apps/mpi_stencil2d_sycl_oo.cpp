// mpi_stencil2d_sycl_oo — square-domain, strong-scaling dim-0 exchange.
//
// Reference: /root/reference/mpi_stencil2d_sycl_oo.cc:517-705 (span2d/array2d
// rewrite of the SYCL test).  CLI `[n_global_Ki] [stage_host 0|1] [n_iter]`
// (defaults 8 -> 8192, 0, 100; 5 warmups); the n_global x n_global domain is
// split in x (n_local = n_global / world_size, must divide).  Output:
// "%d: exchange time %0.8f ms" and "%d: [0x%08x] err_norm = %.8f".
// --debug mirrors the reference's DEBUG build: domain / 1024, one iteration,
// no warmup, and a rank-serialised dump of the halo rows.
// --check: ghost rows compared with the analytic field after every exchange
// (gmt/deriv.hpp DerivConfig::check); exit status 5 on a mismatch.
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "deriv_common.hpp"
#include "gmt/device.hpp"

using namespace gmt;
using namespace gmt::apps;

int main(int argc, char** argv) {
  Cli cli(argc, argv);
  long long n_global = 8 * 1024;
  bool stage_host = false;
  int n_iter = 100, n_warmup = 5;
  if (cli.positional(0)) n_global = std::atoll(cli.positional(0)) * 1024;
  if (cli.positional(1)) stage_host = cli.positional(1)[0] == '1';
  if (cli.positional(2)) n_iter = std::atoi(cli.positional(2));
  const bool debug = cli.flag("debug");
  if (debug) {
    n_global /= 1024;
    n_iter = 1;
    n_warmup = 0;
  }
  mpi_init_pinned(&argc, &argv);  // pinned near the GPU first (gmt/device.hpp)
  int world_size = 1, world_rank = 0;
  MPI_Comm_size(MPI_COMM_WORLD, &world_size);
  MPI_Comm_rank(MPI_COMM_WORLD, &world_rank);
  if (n_global % world_size != 0) {
    std::printf("%d: nmpi (%d) must be divisor of domain size (%lld), exiting\n", world_rank,
                world_size, n_global);
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  const size_t n_local = static_cast<size_t>(n_global / world_size);
  RankBinding b = set_rank_device(MPI_COMM_WORLD, false);
  if (world_rank == 0) {
    std::printf("n procs    = %d\n", world_size);
    std::printf("rank       = %d\n", world_rank);
    std::printf("n_global   = %lld\n", n_global);
    std::printf("n_local    = %zu\n", n_local);
    std::printf("n_iter     = %d\n", n_iter);
    std::printf("n_warmup   = %d\n", n_warmup);
    std::printf("stage_host = %d\n", stage_host ? 1 : 0);
  }
  std::fflush(stdout);
  {
    TransportPool pool(MPI_COMM_WORLD, b);
    DerivConfig c;
    c.dim = 0;
    c.n_local = n_local;
    c.n_other = static_cast<size_t>(n_global);
    c.n_iter = n_iter;
    c.n_warmup = n_warmup;
    c.buf = stage_host;
    c.transport = comm::parse_kind(cli.get("transport", "auto"));
    c.host_init = cli.flag("host-init");
    c.host_verify = cli.flag("host-verify");
    c.check = cli.flag("check");
    c.debug_dump = debug;
    DerivResult r = run_deriv(c, b, MPI_COMM_WORLD, pool);
    std::printf("%d: exchange time %0.8f ms\n", world_rank, r.total_time / (n_iter > 0 ? n_iter : 1) * 1000);
    std::printf("%d: [0x%08x] err_norm = %.8f\n", world_rank, b.info.vendor_id, r.err_norm);
    double med = r.iters.median(), mx = 0;
    MPI_Reduce(&med, &mx, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    if (world_rank == 0) {
      JsonRecord j;
      j.add("app", "mpi_stencil2d_sycl_oo").add("ranks", world_size).add("transport", r.transport)
          .add("stage_host", stage_host).add("n_global", n_global)
          .add("exchange_us_median", mx * 1e6).add("bytes_per_exchange", r.bytes_per_exchange);
      j.append_to(cli.get("json", ""));
    }
  }
  MPI_Finalize();
  return halo_check_failed() ? 5 : EXIT_SUCCESS;
}
