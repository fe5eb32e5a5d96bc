// mpi_stencil2d_sycl — dim-0 halo-exchange benchmark with persistent buffers.
//
// Reference: /root/reference/mpi_stencil2d_sycl.cc:377-556 (hand-written SYCL
// version of the dim-0 test).  CLI `[nx_local] [stage_host 0|1] [n_iter]`
// (defaults 1024, 0, 100; 5 warmups), ny = 512 Ki, weak scaling in x.
// Output: per-rank device identity line, the header, "dev bytes  = ...",
// "%d/%d exchange time %0.8f ms" (average per iteration) and
// "%d/%d [%d:0x%08x] err_norm = %.8f" on every rank.
//
// The reference prints PCI BDF + UUID only for Intel GPUs
// (ext_intel_pci_address) and leaves device_id/vendor_id uninitialised
// (:403-404); here both come from the HIP device.
#include <mpi.h>

#include <cstdio>
#include <cstdlib>

#include "deriv_common.hpp"
#include "gmt/device.hpp"

using namespace gmt;
using namespace gmt::apps;

int main(int argc, char** argv) {
  Cli cli(argc, argv);
  size_t nx_local = 1024;
  bool stage_host = false;
  int n_iter = 100;
  const int n_warmup = 5;
  if (cli.positional(0)) nx_local = std::atol(cli.positional(0));
  if (cli.positional(1)) stage_host = cli.positional(1)[0] == '1';
  if (cli.positional(2)) n_iter = std::atoi(cli.positional(2));
  const size_t ny = static_cast<size_t>(cli.geti("ny", 512 * 1024));
  const int n_bnd = 2;

  GMT_MPI_CHECK(MPI_Init(&argc, &argv));
  int world_size = 1, world_rank = 0;
  MPI_Comm_size(MPI_COMM_WORLD, &world_size);
  MPI_Comm_rank(MPI_COMM_WORLD, &world_rank);
  const size_t nx_global = nx_local * world_size;
  RankBinding b = set_rank_device(MPI_COMM_WORLD, false);
  if (b.info.vendor_id != 0)
    std::printf("%d %04x:%02x:%02x.0(%.8s)\n", world_rank, b.info.pci_domain, b.info.pci_bus,
                b.info.pci_device, b.info.uuid);
  if (world_rank == 0) {
    std::printf("n procs    = %d\n", world_size);
    std::printf("rank       = %d\n", world_rank);
    std::printf("ny         = %zu\n", ny);
    std::printf("nx_global  = %zu\n", nx_global);
    std::printf("nx_local   = %zu\n", nx_local);
    std::printf("n_iter     = %d\n", n_iter);
    std::printf("n_warmup   = %d\n", n_warmup);
    std::printf("stage_host = %d\n", stage_host ? 1 : 0);
    const double MB = 1024.0 * 1024.0, GB = MB * 1024.0;
    const double dev_bytes =
        ((nx_local + 2 * n_bnd) * ny + nx_local * ny + 4.0 * n_bnd * ny) * sizeof(double);
    if (dev_bytes > GB)
      std::printf("dev bytes  = %g GB\n", dev_bytes / GB);
    else
      std::printf("dev bytes  = %g MB\n", dev_bytes / MB);
  }
  std::fflush(stdout);
  {
    TransportPool pool(MPI_COMM_WORLD, b);
    DerivConfig c;
    c.dim = 0;
    c.n_local = nx_local;
    c.n_other = ny;
    c.n_iter = n_iter;
    c.n_warmup = n_warmup;
    c.buf = stage_host;
    c.transport = comm::parse_kind(cli.get("transport", "auto"));
    c.host_init = cli.flag("host-init");
    c.host_verify = cli.flag("host-verify");
    DerivResult r = run_deriv(c, b, MPI_COMM_WORLD, pool);
    std::printf("%d/%d exchange time %0.8f ms\n", world_rank, world_size,
                r.total_time / n_iter * 1000);
    std::printf("%d/%d [%d:0x%08x] err_norm = %.8f\n", world_rank, world_size, b.device,
                b.info.vendor_id, r.err_norm);
    double med = r.iters.median(), mx = 0;
    MPI_Reduce(&med, &mx, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    if (world_rank == 0) {
      JsonRecord j;
      j.add("app", "mpi_stencil2d_sycl").add("ranks", world_size).add("transport", r.transport)
          .add("stage_host", stage_host).add("nx_local", nx_local).add("ny", ny)
          .add("exchange_us_median", mx * 1e6).add("bytes_per_exchange", r.bytes_per_exchange)
          .add("GBps_per_rank", mx > 0 ? r.bytes_per_exchange / mx / 1e9 : 0.0);
      j.append_to(cli.get("json", ""));
    }
  }
  MPI_Finalize();
  return EXIT_SUCCESS;
}
