// The reference's main benchmark (mpi_stencil2d_gt test_deriv / test_sum,
// SURVEY.md §3.1) behind the MPI-free engine ABI (gmt/engine.h), so
// bench.py can time the reference-shaped halo exchange over RCCL/xGMI on
// every rank of a torch.distributed job (IPC when ranks share a GPU): 8 MiB ghost faces per neighbour
// (2 x 524288 doubles), dim 0 packed by the gfx950 copy kernel, dim 1
// zero-copy, the derivative kernel after every exchange, err_norm against
// the analytic derivative, then the 1024-double in-place all-reduce.
#include <cstring>
#include <memory>

#include "gmt/deriv.hpp"
#include "gmt/engine.h"

namespace gmt {
std::unique_ptr<comm::Transport> engine_transport(int rank, int world, int transport, const void* id);
}

extern "C" int gmt_engine_deriv_bench(int64_t n_local, int64_t n_other, int n_iter, int n_warmup,
                                      int rank, int world, int transport, const void* ccl_id,
                                      double* out, int check) {
  std::unique_ptr<gmt::comm::Transport> t = gmt::engine_transport(rank, world, transport, ccl_id);
  if (!t) return 1;
  for (int dim = 0; dim < 2; ++dim) {
    gmt::watchdog_kick(dim == 0 ? "engine: reference halo test dim 0" : "engine: reference halo test dim 1");
    gmt::apps::DerivConfig c;
    c.dim = dim;
    c.n_local = static_cast<size_t>(n_local);
    c.n_other = static_cast<size_t>(n_other);
    c.n_iter = n_iter;
    c.n_warmup = n_warmup;
    c.buf = false;  // dim 0 packs into device buffers, dim 1 goes zero-copy
    c.check = check != 0;  // ghost rows vs the analytic field after every exchange
    const gmt::apps::DerivResult r = gmt::apps::run_deriv_on(c, *t, rank, world);
    double* o = out + 6 * dim;
    o[0] = r.iters.median();
    o[1] = r.iters.mean();
    o[2] = r.iters.min();
    o[3] = r.iters.max();
    o[4] = static_cast<double>(r.bytes_per_exchange);
    o[5] = r.err_norm;
    out[14 + dim] = r.exact_norm;
    out[16 + dim] = static_cast<double>(r.bad_ghosts);  // -1: not checked
  }
  gmt::watchdog_kick("engine: reference all-reduce test");
  const gmt::apps::SumResult s = gmt::apps::run_sum_on(0, GMT_SPACE_DEVICE, static_cast<size_t>(n_local),
                                                       static_cast<size_t>(n_other), n_iter, n_warmup,
                                                       *t, world);
  out[12] = s.iters.median();
  out[13] = s.max_abs_err;
  return 0;
}
