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
//
// --test-buf-view[=N] runs the reference's pack/unpack self-test
// (test_buf_view, mpi_stencil2d_sycl.cc:118-159, wired in but commented out
// of its main at :379-381) on an N x N field (default 6) through the gfx950
// halo copy kernel (gmt_copy2d_batched): print the field and a second
// buffer, pack ghost-side rows [0, n_bnd) into a buffer, unpack the second
// buffer into rows [N-n_bnd, N), print again.  No MPI.
//
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

namespace {

// Copy rows [start, end) of a col-major nrows x ncols field to/from a
// contiguous (end-start) x ncols buffer on `stream` (nullptr = default).
void buf_view_copy(bool to_buf, int ncols, int buf_nrows, double* buf, int nrows, double* data,
                   int start, int end) {
  gmt_copy2d_desc d;
  d.width = end - start;
  d.height = ncols;
  if (to_buf) {
    d.src = data + start, d.src_ld = nrows, d.dst = buf, d.dst_ld = buf_nrows;
  } else {
    d.src = buf, d.src_ld = buf_nrows, d.dst = data + start, d.dst_ld = nrows;
  }
  GMT_CHECK("copy2d", gmt_copy2d_batched(1, &d, sizeof(double), nullptr));
  GMT_CHECK("sync", gmt_rt_device_synchronize());
}

int test_buf_view(int n) {
  const int n_bnd = 2, n_with_ghost = n + 2 * n_bnd;
  std::vector<double> data(size_t(n_with_ghost) * n), buf(size_t(n_bnd) * n),
      buf2(size_t(n_bnd) * n);
  for (int j = 0; j < n; j++) {
    for (int i = 0; i < n_with_ghost; i++) data[i + size_t(j) * n_with_ghost] = (i - n_bnd) + j / 1000.0;
    buf2[0 + size_t(j) * n_bnd] = 100.0 + j;
    buf2[1 + size_t(j) * n_bnd] = 100.0 + j + 0.1;
  }
  auto print_data = [&] {
    for (int j = 0; j < n; j++)
      for (int i = 0; i < n; i++)
        std::printf("data[%d, %d] = %f\n", i, j, data[i + size_t(j) * n_with_ghost]);
  };
  auto print_buf = [&](const char* name, const std::vector<double>& b) {
    for (int j = 0; j < n; j++)
      for (int i = 0; i < n_bnd; i++) std::printf("%s[%d, %d] = %f\n", name, i, j, b[i + size_t(j) * n_bnd]);
  };
  print_data();
  print_buf("buf2", buf2);
  Buffer<double> d_data(data.size(), GMT_SPACE_DEVICE), d_buf(buf.size(), GMT_SPACE_DEVICE),
      d_buf2(buf2.size(), GMT_SPACE_DEVICE);
  GMT_CHECK("H2D", gmt_rt_memcpy(d_data.data(), data.data(), d_data.bytes()));
  GMT_CHECK("H2D", gmt_rt_memcpy(d_buf2.data(), buf2.data(), d_buf2.bytes()));
  buf_view_copy(true, n, n_bnd, d_buf.data(), n_with_ghost, d_data.data(), 0, n_bnd);
  GMT_CHECK("D2H", gmt_rt_memcpy(buf.data(), d_buf.data(), d_buf.bytes()));
  print_buf("buf", buf);
  buf_view_copy(false, n, n_bnd, d_buf2.data(), n_with_ghost, d_data.data(), n - n_bnd, n);
  GMT_CHECK("D2H", gmt_rt_memcpy(data.data(), d_data.data(), d_data.bytes()));
  print_data();
  // self-check (the reference only prints): packed rows are rows 0..1 of the
  // field, unpacked rows n-2..n-1 now hold buf2
  int bad = 0;
  for (int j = 0; j < n; j++)
    for (int i = 0; i < n_bnd; i++) {
      bad += buf[i + size_t(j) * n_bnd] != (i - n_bnd) + j / 1000.0;
      bad += data[n - n_bnd + i + size_t(j) * n_with_ghost] != buf2[i + size_t(j) * n_bnd];
    }
  std::printf("test_buf_view %s\n", bad ? "FAILED" : "OK");
  return bad ? EXIT_FAILURE : EXIT_SUCCESS;
}

}  // namespace

int main(int argc, char** argv) {
  Cli cli(argc, argv);
  if (cli.has("test-buf-view")) {
    GMT_CHECK("set device", gmt_rt_set_device(0));
    const long long n = cli.geti("test-buf-view", 6);  // bare flag = "1" -> default 6
    return test_buf_view(n >= 4 ? static_cast<int>(n) : 6);
  }
  size_t nx_local = 1024;
  bool stage_host = false;
  int n_iter = 100;
  const int n_warmup = 5;
  if (cli.positional(0)) nx_local = std::atol(cli.positional(0));
  if (cli.positional(1)) stage_host = cli.positional(1)[0] == '1';
  if (cli.positional(2)) n_iter = std::atoi(cli.positional(2));
  const size_t ny = static_cast<size_t>(cli.geti("ny", 512 * 1024));
  const int n_bnd = 2;

  mpi_init_pinned(&argc, &argv);  // pinned near the GPU first (gmt/device.hpp)
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
    c.check = cli.flag("check");
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
  return halo_check_failed() ? 5 : EXIT_SUCCESS;
}
