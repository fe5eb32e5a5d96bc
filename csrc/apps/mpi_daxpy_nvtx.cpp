// mpi_daxpy_nvtx_{managed,unmanaged} — distributed DAXPY + all-gather.
//
// Reference: /root/reference/mpi_daxpy_nvtx.cc:85-343, built twice
// (Makefile:16-20): -DMANAGED uses managed arrays initialised in place on the
// host; otherwise pinned host + device arrays with explicit copies.  n =
// nodes * 48 Mi / world_size doubles per rank; x = (i+1)/n, y = -x, so
// SUM = (n+1)/2 and ALLSUM = world_size*(n+1)/2.  roctx ranges carry the
// reference's NVTX names; the profiler window brackets the run
// (rocprofv3 --selected-regions).  TIME lines are printed after
// MPI_Finalize, as in the reference.
//
// MI355X data plane for the two all-gathers: RCCL over xGMI for device
// arrays with one rank per GPU, IPC/staged otherwise, MPI directly on
// managed memory (gmt/comm.hpp).  Added: --barrier (the reference's
// -DBARRIER), --n-per-node=N, --iters=K (K extra timed DAXPYs -> GB/s),
// --transport=..., --json=FILE.
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#include "gmt/buffer.hpp"
#include "gmt/comm.hpp"
#include "gmt/device.hpp"
#include "gmt/util.hpp"

using namespace gmt;

#ifdef GMT_MANAGED
static constexpr bool kManaged = true;
static constexpr const char* kName = "mpi_daxpy_nvtx_managed";
#else
static constexpr bool kManaged = false;
static constexpr const char* kName = "mpi_daxpy_nvtx_unmanaged";
#endif

int main(int argc, char** argv) {
  Cli cli(argc, argv);
  const size_t MB = 1024 * 1024;
  const size_t n_per_node = static_cast<size_t>(cli.geti("n-per-node", 48 * MB));
  const bool barrier = cli.flag("barrier");
  const int iters = static_cast<int>(cli.geti("iters", 0));
  const double a = 2.0;
  double start_time = 0, end_time = 0, k_start = 0, k_end = 0, g_start = 0, g_end = 0,
         b_start = 0, b_end = 0;

  mpi_init_pinned(&argc, &argv);  // pinned near the GPU first (gmt/device.hpp)
  int world_size = 1, world_rank = 0;
  MPI_Comm_size(MPI_COMM_WORLD, &world_size);
  MPI_Comm_rank(MPI_COMM_WORLD, &world_rank);
  const int nodes = get_node_count(MPI_COMM_WORLD);
  const size_t nall = nodes * n_per_node;
  const size_t n = nall / world_size;
  if (world_rank == 0)
    std::printf("%d nodes, %d ranks, %zu elements each, total %zu\n", nodes, world_size, n, nall);
  if (world_rank == 0) {
    const char* mb = std::getenv("MEMORY_PER_CORE");
    if (mb == nullptr)
      std::printf("MEMORY_PER_CORE is not set\n");
    else
      std::printf("MEMORY_PER_CORE=%s\n", mb);
  }
  RankBinding b = set_rank_device(MPI_COMM_WORLD, true);
  std::unique_ptr<comm::Transport> tr = comm::make_transport(
      comm::resolve(comm::parse_kind(cli.get("transport", "auto")), b, kManaged), MPI_COMM_WORLD, b);
  double kbest = 0.0;

  gmt_profiler_start();
  start_time = MPI_Wtime();
  {
    const int dspace = kManaged ? GMT_SPACE_MANAGED : GMT_SPACE_DEVICE;
    Buffer<double> h_x, h_y, h_allx, h_ally, d_x, d_y, d_allx, d_ally;
    {
      TraceRange r("allocateArrays");
      if (!kManaged) {
        h_x = Buffer<double>(n, GMT_SPACE_PINNED);
        h_y = Buffer<double>(n, GMT_SPACE_PINNED);
      }
      d_x = Buffer<double>(n, dspace);
      d_y = Buffer<double>(n, dspace);
      d_allx = Buffer<double>(n * world_size, dspace);
      d_ally = Buffer<double>(n * world_size, dspace);
      if (!kManaged) {
        h_allx = Buffer<double>(n * world_size, GMT_SPACE_PINNED);
        h_ally = Buffer<double>(n * world_size, GMT_SPACE_PINNED);
      }
    }
    if (world_rank == 0) {
      size_t free_mem = 0, total_mem = 0;
      GMT_CHECK("memInfo", gmt_rt_mem_info(&free_mem, &total_mem));
      std::printf("GPU memory %0.3f / %0.3f (%0.3f) MB\n", free_mem / (double)MB,
                  (double)total_mem / MB, (double)(total_mem - free_mem) / MB);
    }
    {
      TraceRange r("initializeArrays");
      double* ix = kManaged ? d_x.data() : h_x.data();
      double* iy = kManaged ? d_y.data() : h_y.data();
      for (size_t i = 0; i < n; ++i) {
        ix[i] = (i + 1) / static_cast<double>(n);
        iy[i] = -ix[i];
      }
      if (!kManaged) {
        TraceRange c("copyInput");
        GMT_CHECK("d_x = h_x", gmt_rt_memcpy(d_x.data(), h_x.data(), d_x.bytes()));
        GMT_CHECK("d_y = h_y", gmt_rt_memcpy(d_y.data(), h_y.data(), d_y.bytes()));
      }
    }
    GMT_MEMINFO("d_x", d_x.data(), d_x.bytes());
    GMT_MEMINFO("d_y", d_y.data(), d_y.bytes());
    if (!kManaged) {
      GMT_MEMINFO("h_x", h_x.data(), h_x.bytes());
      GMT_MEMINFO("h_y", h_y.data(), h_y.bytes());
      GMT_MEMINFO("h_allx", h_allx.data(), h_allx.bytes());
      GMT_MEMINFO("h_ally", h_ally.data(), h_ally.bytes());
    }

    k_start = MPI_Wtime();
    {
      TraceRange r("cublasDaxpy");
      GMT_CHECK("daxpy", gmt_daxpy(n, a, d_x.data(), d_y.data(), nullptr));
      GMT_CHECK("daxpy sync", gmt_rt_device_synchronize());
    }
    k_end = MPI_Wtime();

    double sum = 0.0;
    {
      TraceRange r("localSum");
      const double* py = d_y.data();
      if (!kManaged) {
        TraceRange c("copyOutput");
        GMT_CHECK("h_y = d_y", gmt_rt_memcpy(h_y.data(), d_y.data(), d_y.bytes()));
        py = h_y.data();
      }
      for (size_t i = 0; i < n; ++i) sum += py[i];
    }
    std::printf("%d/%d SUM = %f\n", world_rank, world_size, sum);

    {
      TraceRange r("copyPrepAllxInplace");
      GMT_CHECK("allx[rank] = x",
                gmt_rt_memcpy(d_allx.data() + world_rank * n, d_x.data(), d_x.bytes()));
    }
    if (barrier) {
      b_start = MPI_Wtime();
      TraceRange r("mpiBarrier");
      MPI_Barrier(MPI_COMM_WORLD);
      b_end = MPI_Wtime();
    }
    g_start = MPI_Wtime();
    {
      TraceRange r("mpiAllGather");
      {
        TraceRange rx("x");
        tr->allgather(d_allx.data() + world_rank * n, d_allx.data(), n * sizeof(double), nullptr);
        GMT_CHECK("gather x sync", gmt_rt_device_synchronize());
      }
      {
        TraceRange ry("y");
        tr->allgather(d_y.data(), d_ally.data(), n * sizeof(double), nullptr);
        GMT_CHECK("gather y sync", gmt_rt_device_synchronize());
      }
    }
    g_end = MPI_Wtime();

    sum = 0.0;
    {
      TraceRange r("allSum");
      const double* pa = d_ally.data();
      if (!kManaged) {
        TraceRange c("copyAlly");
        GMT_CHECK("h_ally = d_ally", gmt_rt_memcpy(h_ally.data(), d_ally.data(), d_ally.bytes()));
        pa = h_ally.data();
      }
      for (size_t i = 0; i < n * world_size; ++i) sum += pa[i];
    }
    std::printf("%d/%d ALLSUM = %f\n", world_rank, world_size, sum);

    if (iters > 0) {  // steady-state DAXPY rate (the single timed call above is cold)
      gmt_event_t e0, e1;
      gmt_rt_event_create(&e0, 1);
      gmt_rt_event_create(&e1, 1);
      Stats st;
      for (int k = 0; k < iters; ++k) {
        gmt_rt_event_record(e0, nullptr);
        GMT_CHECK("daxpy", gmt_daxpy(n, a, d_x.data(), d_y.data(), nullptr));
        gmt_rt_event_record(e1, nullptr);
        gmt_rt_event_synchronize(e1);
        float ms = 0;
        gmt_rt_event_elapsed_ms(&ms, e0, e1);
        st.add(ms * 1e-3);
      }
      kbest = st.median();
      gmt_rt_event_destroy(e0);
      gmt_rt_event_destroy(e1);
    }
    TraceRange r("free");
  }
  end_time = MPI_Wtime();
  gmt_profiler_stop();

  const std::string tname = tr->name();
  double kmax = 0.0;
  MPI_Reduce(&kbest, &kmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
  tr.reset();
  MPI_Finalize();

  std::printf("%d/%d TIME total  : %0.3f\n", world_rank, world_size, end_time - start_time);
  std::printf("%d/%d TIME kernel : %0.3f\n", world_rank, world_size, k_end - k_start);
  std::printf("%d/%d TIME barrier: %0.3f\n", world_rank, world_size, b_end - b_start);
  std::printf("%d/%d TIME gather : %0.3f\n", world_rank, world_size, g_end - g_start);
  if (world_rank == 0) {
    const double gather_bytes = 2.0 * n * world_size * sizeof(double);
    if (kmax > 0)
      std::printf("# DAXPY steady state: %.4f ms/call, %.1f GB/s per rank (%d iters, max over ranks)\n",
                  kmax * 1e3, 24.0 * n / kmax / 1e9, iters);
    std::printf("# all-gather transport=%s: %.1f GB/s (2 gathers of %zu B)\n", tname.c_str(),
                gather_bytes / (g_end - g_start) / 1e9, n * world_size * sizeof(double));
    JsonRecord j;
    j.add("app", kName).add("ranks", world_size).add("nodes", nodes).add("n", n)
        .add("transport", tname).add("time_total_s", end_time - start_time)
        .add("time_kernel_s", k_end - k_start).add("time_gather_s", g_end - g_start)
        .add("daxpy_ms_steady", kmax * 1e3).add("daxpy_GBps_per_rank", kmax > 0 ? 24.0 * n / kmax / 1e9 : 0.0);
    j.append_to(cli.get("json", ""));
  }
  return EXIT_SUCCESS;
}
