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
//
// --bench[=N] (not in the reference; BASELINE config "mpi_daxpy 8 ranks x 1
// GPU, RCCL allreduce of partial sums over xGMI"): every rank runs DAXPY on N
// device doubles (default 2^28, 6 GiB moved per call) --iters times, reduces
// y to a partial sum on the device (gmt_sum_axis) and all-reduces the
// partial sums through the transport (--transport=auto: RCCL for one rank
// per GPU, IPC/MPI otherwise).  Reports per-rank and aggregate GB/s, the
// all-reduce latency and ALLSUM against its closed form; --json=FILE.
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
  const size_t n = static_cast<size_t>(cli.geti("n", 1024));
  const double a = 2.0;
  mpi_init_pinned(&argc, &argv);  // pinned near the GPU first (gmt/device.hpp)
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
  int rc = EXIT_SUCCESS;
  if (cli.has("bench")) {
    const std::string bv = cli.get("bench", "1");
    const size_t nb = bv == "1" ? (size_t(1) << 28) : static_cast<size_t>(std::atoll(bv.c_str()));
    const int iters = static_cast<int>(cli.geti("iters", 20));
    comm::Kind kind = comm::parse_kind(cli.get("transport", "auto"));
    if (kind == comm::Kind::Auto && world_size == 1) kind = comm::Kind::Local;
    auto tr = comm::make_transport(comm::resolve(kind, b), MPI_COMM_WORLD, b);
    gmt_stream_t s = nullptr;
    GMT_CHECK("stream", gmt_rt_stream_create(&s, 0));
    Buffer<double> dx(nb, GMT_SPACE_DEVICE), dy(nb, GMT_SPACE_DEVICE);
    Buffer<double> ws(gmt_sum_axis_workspace(1, static_cast<int64_t>(nb), 1) + 1, GMT_SPACE_DEVICE);
    Buffer<double> part(1, GMT_SPACE_DEVICE);
    // x = (i+1)/n, y = -x (the reference's mpi_daxpy_nvtx initialisation)
    GMT_CHECK("fill x", gmt_fill_poly(3, static_cast<int64_t>(nb), 1, 1.0 / nb, 1.0 / nb, 0.0, 0.0, dx.data(),
                                      static_cast<int64_t>(nb), s));
    GMT_CHECK("fill y", gmt_fill_poly(3, static_cast<int64_t>(nb), 1, -1.0 / nb, -1.0 / nb, 0.0, 0.0, dy.data(),
                                      static_cast<int64_t>(nb), s));
    GMT_CHECK("daxpy", gmt_daxpy(nb, a, dx.data(), dy.data(), s));  // warm-up: y = x
    GMT_CHECK("sync", gmt_rt_stream_synchronize(s));
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = wtime();
    for (int it = 0; it < iters; ++it) GMT_CHECK("daxpy", gmt_daxpy(nb, a, dx.data(), dy.data(), s));
    GMT_CHECK("sync", gmt_rt_stream_synchronize(s));
    double dt = wtime() - t0;
    MPI_Allreduce(MPI_IN_PLACE, &dt, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    // partial sum on the device, then the all-reduce of the partial sums
    GMT_CHECK("sum", gmt_sum_axis(1, static_cast<int64_t>(nb), 1, dy.data(), static_cast<int64_t>(nb),
                                  part.data(), ws.data(), s));
    Buffer<double> red(1, GMT_SPACE_DEVICE);
    Stats ar;
    for (int it = 0; it < iters + 3; ++it) {
      GMT_CHECK("copy", gmt_rt_memcpy_async(red.data(), part.data(), sizeof(double), s));
      GMT_CHECK("sync", gmt_rt_stream_synchronize(s));
      MPI_Barrier(MPI_COMM_WORLD);
      const double a0 = wtime();
      tr->allreduce_sum(red.data(), 1, s);
      GMT_CHECK("sync", gmt_rt_stream_synchronize(s));
      if (it >= 3) ar.add(wtime() - a0);
    }
    double psum = 0, allsum = 0;
    GMT_CHECK("d2h", gmt_rt_memcpy(&psum, part.data(), sizeof(double)));
    GMT_CHECK("d2h", gmt_rt_memcpy(&allsum, red.data(), sizeof(double)));
    double med = ar.median(), med_max = 0;
    MPI_Allreduce(&med, &med_max, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    // after the warm-up y = x; each timed call adds 2x: y = (1 + 2*iters) x
    const double expect = (1.0 + 2.0 * iters) * (static_cast<double>(nb) + 1) / 2.0 * world_size;
    const double rel = std::fabs(allsum - expect) / expect;
    if (world_rank == 0) {
      const double gbs = 24.0 * nb * iters / dt / 1e9;
      std::printf("BENCH daxpy n=%zu per rank x %d ranks: %0.4f ms/call, %0.1f GB/s per rank, %0.1f GB/s aggregate\n",
                  nb, world_size, dt / iters * 1e3, gbs, gbs * world_size);
      std::printf("BENCH allreduce of partial sums (%s): %0.2f us median (max over ranks); "
                  "ALLSUM = %0.6e (expected %0.6e, rel err %0.2e) %s\n",
                  tr->name(), med_max * 1e6, allsum, expect, rel, rel < 1e-9 ? "OK" : "FAIL");
      JsonRecord j;
      j.add("app", "mpi_daxpy").add("ranks", world_size).add("n_per_rank", nb).add("iters", iters)
          .add("ms_per_call", dt / iters * 1e3).add("GBps_per_rank", gbs).add("GBps_aggregate", gbs * world_size)
          .add("transport", tr->name()).add("allreduce_us", med_max * 1e6).add("allsum_rel_err", rel);
      j.append_to(cli.get("json", ""));
    }
    if (rel >= 1e-9) rc = 3;
    (void)psum;
    GMT_CHECK("stream", gmt_rt_stream_destroy(s));
  }
  MPI_Finalize();
  return rc;
}
