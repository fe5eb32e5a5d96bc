// Shared engine of the distributed-derivative benchmarks
// (mpi_stencil2d_gt, mpi_stencil2d_sycl, mpi_stencil2d_sycl_oo).
//
// Reference: test_deriv<S, Dim> (mpi_stencil2d_gt.cc:385-572), test_sum<S, Dim>
// (:574-649) and the SYCL mains (mpi_stencil2d_sycl.cc:377-556,
// mpi_stencil2d_sycl_oo.cc:517-705).  Workload: z = x^3 + y^2 on a
// column-major 2-D array decomposed into 1-D slabs along `dim`, 2 ghost
// cells per side, 4th-order first derivative dz/d(dim) after every halo
// exchange; err_norm = ||numeric - analytic||_2 (the stencil is exact for
// cubics, so err_norm is round-off unless the halo exchange is wrong).
//
// MI355X-side choices: the analytic fill and the verification run on the
// GPU (gmt_fill_poly / gmt_diff_sq, no 12 GB of host arrays per rank —
// --host-init / --host-verify restore the reference's host loops), buffers
// are persistent, and the transport is explicit and reported.
#pragma once

#include <mpi.h>

#include <cmath>
#include <cstdio>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "gmt/buffer.hpp"
#include "gmt/comm.hpp"
#include "gmt/deriv.hpp"
#include "gmt/halo.hpp"
#include "gmt/util.hpp"

namespace gmt {
namespace apps {


// One transport per kind for the whole run (RCCL communicators and IPC
// streams are set up once, outside every timed loop).
class TransportPool {
 public:
  TransportPool(MPI_Comm c, const RankBinding& b) : c_(c), b_(b) {}
  comm::Transport& get(comm::Kind k) {
    auto it = pool_.find(k);
    if (it != pool_.end()) return *it->second;
    auto t = comm::make_transport(k, c_, b_);
    auto& ref = *t;
    pool_[k] = std::move(t);
    return ref;
  }

 private:
  MPI_Comm c_;
  RankBinding b_;
  std::map<comm::Kind, std::unique_ptr<comm::Transport>> pool_;
};



// Print rows [r0, r0+nr) of a column-major field (first <= 20 columns) for
// every rank in rank order (mpi_stencil2d_sycl_oo.cc:636-659 serialises the
// ranks with MPI_Barrier; here rank 0 gathers the formatted lines and prints
// them, so the forwarded stdout of several ranks cannot interleave).
inline void dump_rows(MPI_Comm comm, int rank, int ws, const char* what, const double* dev,
                      size_t nrows, size_t ncols, size_t r0, size_t nr) {
  const size_t nc = ncols < 20 ? ncols : 20;
  std::vector<double> h(nrows * nc);
  GMT_CHECK("dump D2H", gmt_rt_memcpy(h.data(), dev, h.size() * sizeof(double)));
  std::string text;
  char buf[64];
  for (size_t i = r0; i < r0 + nr; ++i) {
    std::snprintf(buf, sizeof(buf), "%d: %s [%zu, :]", rank, what, i);
    text += buf;
    for (size_t j = 0; j < nc; ++j) {
      std::snprintf(buf, sizeof(buf), " %f", h[i + j * nrows]);
      text += buf;
    }
    text += "\n";
  }
  int len = static_cast<int>(text.size());
  std::vector<int> lens(ws), offs(ws);
  GMT_MPI_CHECK(MPI_Gather(&len, 1, MPI_INT, lens.data(), 1, MPI_INT, 0, comm));
  std::string all;
  if (rank == 0) {
    int tot = 0;
    for (int r = 0; r < ws; ++r) {
      offs[r] = tot;
      tot += lens[r];
    }
    all.resize(tot);
  }
  GMT_MPI_CHECK(MPI_Gatherv(text.data(), len, MPI_CHAR, rank == 0 ? &all[0] : nullptr, lens.data(),
                            offs.data(), MPI_CHAR, 0, comm));
  if (rank == 0) {
    std::fwrite(all.data(), 1, all.size(), stdout);
    std::fflush(stdout);
  }
}



inline comm::Kind pick_transport(const DerivConfig& c, const RankBinding& b) {
  if (c.transport != comm::Kind::Auto) return comm::resolve(c.transport, b);
  if (c.dim == 0 && c.buf && c.staged_is_host) return comm::Kind::MpiHost;
  return comm::resolve(comm::Kind::Auto, b, c.space == GMT_SPACE_MANAGED);
}

// --check failed on some rank in some test (the app then exits with status 5)
inline bool& halo_check_failed() {
  static bool f = false;
  return f;
}

inline DerivResult run_deriv(const DerivConfig& c, const RankBinding& b, MPI_Comm comm,
                             TransportPool& pool) {
  comm::Transport& tr = pool.get(pick_transport(c, b));
  const int rank = b.rank, ws = b.world_size;
  DumpFn dump = [&](const char* what, const double* f, size_t nr, size_t nc, size_t r0, size_t n) {
    dump_rows(comm, rank, ws, what, f, nr, nc, r0, n);
  };
  DerivResult r = run_deriv_on(c, tr, rank, ws, dump);
  if (c.check) {  // per-exchange ghost check: one line per test on rank 0
    long long bad = r.bad_ghosts < 0 ? 0 : r.bad_ghosts, tot = 0;
    int n = r.checked_exchanges, nmin = 0;
    MPI_Allreduce(&bad, &tot, 1, MPI_LONG_LONG, MPI_SUM, comm);
    MPI_Allreduce(&n, &nmin, 1, MPI_INT, MPI_MIN, comm);
    if (rank == 0)
      std::printf("# halo check dim:%d buf:%d (%s): %lld bad ghost cells, %d exchanges checked per rank\n", c.dim,
                  c.buf ? 1 : 0, r.transport.c_str(), tot, nmin);
    if (tot != 0) halo_check_failed() = true;
    r.bad_ghosts = tot;
  }
  return r;
}

inline SumResult run_sum(int dim, int space, size_t n_local, size_t n_other, int n_iter,
                         int n_warmup, comm::Kind want, const RankBinding& b, TransportPool& pool) {
  comm::Kind k = want != comm::Kind::Auto ? comm::resolve(want, b)
                                          : comm::resolve(comm::Kind::Auto, b, space == GMT_SPACE_MANAGED);
  return run_sum_on(dim, space, n_local, n_other, n_iter, n_warmup, pool.get(k), b.world_size);
}

inline void device_tag(const RankBinding& b, char* out, size_t n) {
  std::snprintf(out, n, "[%d:0x%08x]", b.device, b.info.vendor_id);
}

}  // namespace apps
}  // namespace gmt
