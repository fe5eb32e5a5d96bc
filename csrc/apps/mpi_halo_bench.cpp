// mpi_halo_bench — halo-exchange latency / bandwidth sweep per transport.
//
// The reference measures halo exchanges only at its fixed shapes: 16 B
// (mpi_stencil_gt.cc:200-204), 8 MiB (mpi_stencil2d_gt.cc:511-535), 128 KiB
// (mpi_stencil2d_sycl_oo.cc:679-680).  This sweeps the message size for one
// transport on a 1-D ring (each rank exchanges with rank-1 and rank+1, both
// directions at once; a single rank exchanges with itself) and reports the
// median time per exchange and the bandwidth per rank — the BASELINE
// "halo-exchange latency" metric as a curve.  Each exchange is timed
// blocking (barrier, exchange, stream synchronize: the host round trip is
// part of it).  For stream-ordered transports (rccl, ipc, local) the
// us_stream column is the per-exchange time of `iters` exchanges enqueued
// back to back with one synchronize — what a solver loop that never waits
// on the host sees.
//
// CLI: mpi_halo_bench [min_bytes] [max_bytes] [iters]   (16 B .. 64 MiB, 50)
//      --transport=auto|rccl|ipc|mpi-host|mpi-direct|local  --json=FILE
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
  const size_t lo = cli.positional(0) ? std::atoll(cli.positional(0)) : 16;
  const size_t hi = cli.positional(1) ? std::atoll(cli.positional(1)) : 64ull << 20;
  const int iters = cli.positional(2) ? std::atoi(cli.positional(2)) : 50;
  mpi_init_pinned(&argc, &argv);  // pinned near the GPU first (gmt/device.hpp)
  int world = 1, rank = 0;
  MPI_Comm_size(MPI_COMM_WORLD, &world);
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  RankBinding b = set_rank_device(MPI_COMM_WORLD, false);
  comm::Kind kind = comm::parse_kind(cli.get("transport", "auto"));
  if (kind == comm::Kind::Auto && world == 1) kind = comm::Kind::Local;
  auto tr = comm::make_transport(comm::resolve(kind, b), MPI_COMM_WORLD, b);
  const int left = (rank + world - 1) % world, right = (rank + 1) % world;
  {  // where every rank runs (gmt_rt_pin_rank; -1: not pinned): one header line
    int cpu = b.pinned_cpu, node = b.numa_node;
    std::vector<int> all(2 * static_cast<size_t>(world));
    int mine[2] = {cpu, node};
    MPI_Gather(mine, 2, MPI_INT, all.data(), 2, MPI_INT, 0, MPI_COMM_WORLD);
    if (rank == 0) {
      std::printf("# pinned cpu per rank:");
      for (int r = 0; r < world; ++r) std::printf(" %d", all[2 * r]);
      std::printf("\n");
    }
  }
  if (rank == 0)
    std::printf("# halo exchange sweep: %d ranks, transport=%s, backend=%s, ring neighbours, %d iters\n"
                "# bytes_per_msg  msgs  us_median  us_min  GB/s_per_rank(sent+recv)  us_stream\n",
                world, tr->name(), gmt_rt_backend_name(), iters);
  gmt_stream_t s = nullptr;
  GMT_CHECK("stream", gmt_rt_stream_create(&s, 1));
  for (size_t bytes = lo; bytes <= hi; bytes *= 2) {
    Buffer<char> sl(bytes, GMT_SPACE_DEVICE), sr(bytes, GMT_SPACE_DEVICE),
        rl(bytes, GMT_SPACE_DEVICE), rr(bytes, GMT_SPACE_DEVICE);
    GMT_CHECK("memset", gmt_rt_memset_async(sl.data(), 1, bytes, s));
    GMT_CHECK("memset", gmt_rt_memset_async(sr.data(), 2, bytes, s));
    std::vector<comm::Msg> recvs{{rl.data(), bytes, left, 123}, {rr.data(), bytes, right, 456}};
    std::vector<comm::Msg> sends{{sl.data(), bytes, left, 456}, {sr.data(), bytes, right, 123}};
    auto ex = tr->plan(recvs, sends);
    Stats st;
    for (int k = 0; k < iters + 5; ++k) {
      MPI_Barrier(MPI_COMM_WORLD);
      const double t0 = wtime();
      ex->run(s);
      GMT_CHECK("sync", gmt_rt_stream_synchronize(s));
      if (k >= 5) st.add(wtime() - t0);
    }
    double streamed = -1.0;
    if (ex->graph_capturable()) {
      MPI_Barrier(MPI_COMM_WORLD);
      const double t0 = wtime();
      for (int k = 0; k < iters; ++k) ex->run(s);
      GMT_CHECK("sync", gmt_rt_stream_synchronize(s));
      streamed = (wtime() - t0) / iters;
      MPI_Allreduce(MPI_IN_PLACE, &streamed, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    }
    // correctness: rl holds the left neighbour's "send right" (2), rr its right's "send left" (1)
    char a = 0, c = 0;
    GMT_CHECK("chk", gmt_rt_memcpy(&a, rl.data() + bytes - 1, 1));
    GMT_CHECK("chk", gmt_rt_memcpy(&c, rr.data(), 1));
    int bad = (a != 2 || c != 1) ? 1 : 0;
    MPI_Allreduce(MPI_IN_PLACE, &bad, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
    double med = st.median(), mn = st.min();
    MPI_Allreduce(MPI_IN_PLACE, &med, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    MPI_Allreduce(MPI_IN_PLACE, &mn, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    if (rank == 0) {
      const double gbps = 4.0 * bytes / med / 1e9;
      char stream_col[32] = "        -";
      if (streamed > 0) std::snprintf(stream_col, sizeof(stream_col), "%9.2f", streamed * 1e6);
      std::printf("%14zu  %4d  %9.2f  %7.2f  %8.2f  %s%s\n", bytes, 2, med * 1e6, mn * 1e6, gbps, stream_col,
                  bad ? "  DATA MISMATCH" : "");
      JsonRecord j;
      j.add("app", "mpi_halo_bench").add("ranks", world).add("transport", tr->name())
          .add("bytes", bytes).add("us_median", med * 1e6).add("us_min", mn * 1e6)
          .add("GBps_per_rank", gbps).add("us_stream", streamed > 0 ? streamed * 1e6 : -1.0).add("ok", !bad);
      j.append_to(cli.get("json", ""));
    }
    if (bad) {
      if (rank == 0) std::printf("ERROR: halo data mismatch\n");
      MPI_Abort(MPI_COMM_WORLD, 3);
    }
  }
  gmt_rt_stream_destroy(s);
  tr.reset();
  MPI_Finalize();
  return EXIT_SUCCESS;
}
